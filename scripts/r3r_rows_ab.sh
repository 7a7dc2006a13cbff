cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in 3 1 3 1 3 1; do
  echo "== HYRES_WGRAD_HALO_ROWS=$r"
  for m in "" "--amp"; do timeout -k 10 120 env HYRES_WGRAD_HALO_ROWS=$r python3 scripts/step_profile.py --steps 30 $m 2>&1 | grep "ms/step" || exit 1; done
done > gpurun_out/r3r_rows_ab.txt
cat gpurun_out/r3r_rows_ab.txt
