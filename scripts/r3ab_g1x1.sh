cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
scripts/gpu_run.sh \
  "step:400:for i in 1 2 3; do for g in 2 1; do echo == groups=\$g; HYRES_WGRAD_1X1_GROUPS=\$g python3 scripts/step_profile.py --steps 20; HYRES_WGRAD_1X1_GROUPS=\$g python3 scripts/step_profile.py --amp --steps 20; done; done" || exit $?
