cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ALT="HYRES_LIB_PATH=$GRAFT_REPO_ROOT/_alt/libhyres_hip_nowpe.so"
scripts/gpu_run.sh \
  "step:400:rocm-smi --showclocks --showpower 2>/dev/null | grep -E 'sclk|Power' | head -4; for i in 1 2; do for v in new old; do E=''; [ \$v = old ] && E=\"$ALT\"; echo == \$v; env \$E python3 scripts/step_profile.py --steps 20; env \$E python3 scripts/step_profile.py --amp --steps 20; done; done" || exit $?
