cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() { echo "== $1"; for m in "" "--amp"; do timeout -k 10 120 env $1 python3 scripts/step_profile.py --steps 20 $m 2>&1 | grep "ms/step" || return 1; done; }
for cfg in "HYRES_X=0" "HYRES_WGRAD_BLOCKS=1024" "HYRES_WGRAD_BLOCKS=4096" "HYRES_WGRAD_MAXSPLIT=128" "HYRES_SIDE_STREAM=1" "HYRES_WGRAD_HALO_ROWS=1" "HYRES_BRANCH_MAX_PIXELS=65536" "HYRES_WGRAD_MINCHUNKS=16" "HYRES_X=0"; do
  run "$cfg" >> gpurun_out/r3p_sweep.txt || exit 1
done
cat gpurun_out/r3p_sweep.txt
