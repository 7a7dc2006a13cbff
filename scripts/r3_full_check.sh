cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
scripts/gpu_run.sh \
  "gputests:900:python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu" \
  "wgmicro:200:python scripts/wgrad_micro.py --H 128 --Ci 64 --Co 64 --K 3 && python scripts/wgrad_micro.py --H 128 --Ci 128 --Co 64 --K 1 && HYRES_WGRAD_ROWS_REDUCE=0 python scripts/wgrad_micro.py --H 128 --Ci 64 --Co 64 --K 3 && HYRES_WGRAD_ROWS_REDUCE=0 python scripts/wgrad_micro.py --H 128 --Ci 128 --Co 64 --K 1" || exit $?
bash scripts/dist_rehearsal.sh
