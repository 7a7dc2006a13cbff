cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for A in 0 1 2 4 3 6 7 0; do
  echo "ABLATE=$A $(HYRES_WRES32_ABLATE=$A timeout -k 10 120 python3 scripts/conv_micro.py --H 128 2>&1 | grep conv)"
done
