cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
scripts/gpu_run.sh \
  "tests:400:python -u -m pytest tests/test_parity_gpu.py tests/test_amp_f16_act_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k 'amp or f16 or wres or routing'" \
  "micro:200:python scripts/conv_micro.py --H 128 --Ci 64 --Co 64 --K 3 --f16 --res --relu && python scripts/conv_micro.py --H 128 --Ci 64 --Co 64 --K 3 --f16 && python scripts/conv_micro.py --H 256 --Ci 64 --Co 64 --K 3 --f16 --res --relu" \
  "step:300:for i in 1 2 3; do python3 scripts/step_profile.py --amp --steps 30; done; python3 scripts/step_profile.py --steps 20" || exit $?
