cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
scripts/gpu_run.sh \
  "tests:400:python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k 'conv2d or wres or routing or train_step or c2 or captured or amp' && python -u -m pytest tests/test_wgrad_defer_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k train_step" \
  "micro:200:python scripts/conv_micro.py --H 128 --Ci 64 --Co 64 --K 3 && HYRES_WRES_DYNAMIC=0 python scripts/conv_micro.py --H 128 --Ci 64 --Co 64 --K 3 && python scripts/conv_micro.py --H 256 --Ci 64 --Co 64 --K 3 && HYRES_WRES_DYNAMIC=0 python scripts/conv_micro.py --H 256 --Ci 64 --Co 64 --K 3" \
  "step:300:for d in 1 0 1 0; do echo dyn=\$d; HYRES_WRES_DYNAMIC=\$d python3 scripts/step_profile.py --steps 20; HYRES_WRES_DYNAMIC=\$d python3 scripts/step_profile.py --amp --steps 20; done" \
  "bench:420:python3 bench.py --no-cpu-baseline" || exit $?
