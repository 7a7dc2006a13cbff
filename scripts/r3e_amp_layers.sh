cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
scripts/gpu_run.sh \
  "f16act:300:python -u -m pytest tests/test_amp_f16_act_gpu.py -q --timeout 200 --timeout-method thread -m gpu" \
  "lt_amp_f16act:300:python3 scripts/layer_table.py --amp" \
  "lt_amp_f32act:300:HYRES_AMP_F16_ACT=0 python3 scripts/layer_table.py --amp"
