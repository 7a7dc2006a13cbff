cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ALT="HYRES_LIB_PATH=$GRAFT_REPO_ROOT/_alt/libhyres_hip_prev.so"
M="python scripts/conv_micro.py"
scripts/gpu_run.sh \
  "tests:400:python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k 'conv or routing or amp or c2'" \
  "micro:300:for v in new old; do echo == \$v; E=''; [ \$v = old ] && E=\"$ALT\"; env \$E $M --H 32 --Ci 192 --Co 384 --K 3; env \$E $M --H 32 --Ci 384 --Co 192 --K 3 --f16; env \$E $M --H 64 --Ci 128 --Co 192 --K 5 --stride 2; done" \
  "step:400:for i in 1 2 3; do for v in new old; do E=''; [ \$v = old ] && E=\"$ALT\"; echo == \$v; env \$E python3 scripts/step_profile.py --steps 20; env \$E python3 scripts/step_profile.py --amp --steps 20; done; done" || exit $?
