cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for t in 0 2 4 8; do
  echo "TPB=$t"
  HYRES_WRES_TPB=$t timeout 120 python scripts/conv_micro.py 2>&1 | grep conv || exit 1
  HYRES_WRES_TPB=$t timeout 120 python scripts/conv_micro.py --H 256 2>&1 | grep conv || exit 1
  HYRES_WRES_TPB=$t timeout 300 python bench.py --steps 20 --warmup 5 --no-eval --no-amp --no-host-jpeg --no-cpu-baseline 2>&1 | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('step', d['ms_per_step'], d['value'], d['roofline']['kernel'][:40], d['roofline']['frac'], d['roofline']['frac_isolated'])" || exit 1
done
