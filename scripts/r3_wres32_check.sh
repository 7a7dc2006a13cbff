cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
scripts/gpu_run.sh \
  "micro32:200:python scripts/conv_micro.py && python scripts/conv_micro.py --H 256 && python scripts/conv_micro.py --relu && HYRES_CONV_WRES32=0 python scripts/conv_micro.py && HYRES_CONV_WRES32=0 python scripts/conv_micro.py --H 256" \
  "convtests:600:python -u -m pytest tests/test_parity_gpu.py -q --timeout 300 --timeout-method thread -m gpu -k 'conv2d_fwd_bwd or c2_size or model_train or model_eval or stage'" || exit $?
