cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ALT="HYRES_LIB_PATH=$GRAFT_REPO_ROOT/_alt/libhyres_hip_p16.so"
W="python scripts/wgrad_micro.py"
scripts/gpu_run.sh \
  "tests:400:env $ALT python -u -m pytest tests/test_parity_gpu.py tests/test_wgrad_defer_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k 'amp or f16 or wgrad or deferred'" \
  "micro:300:for v in p16 base; do echo == \$v; E=''; [ \$v = p16 ] && E=\"$ALT\"; env \$E $W --H 128 --Ci 64 --Co 128 --K 1 --f16; env \$E $W --H 128 --Ci 128 --Co 64 --K 1 --f16; env \$E $W --H 128 --Ci 64 --Co 64 --K 3 --f16; done" \
  "step:400:for i in 1 2 3; do for v in p16 base; do E=''; [ \$v = p16 ] && E=\"$ALT\"; echo == \$v; env \$E python3 scripts/step_profile.py --amp --steps 30; done; done" || exit $?
