cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() { echo "== $1"; for m in "" "--amp"; do timeout -k 10 120 env $1 python3 scripts/step_profile.py --steps 30 $m 2>&1 | grep "ms/step" || return 1; done; }
for cfg in "HYRES_X=0" "HYRES_WGRAD_1X1_GROUPS=1" "HYRES_CONV_PRIO=0" "HYRES_CONV_SPLIT_BLOCKS=1024" "HYRES_CONV_SPLIT_BLOCKS=2048" "HYRES_X=0" "HYRES_WGRAD_1X1_GROUPS=1" "HYRES_CONV_PRIO=0" "HYRES_CONV_SPLIT_BLOCKS=1024" "HYRES_CONV_SPLIT_BLOCKS=2048" "HYRES_X=0"; do
  run "$cfg" >> gpurun_out/r3s_sweep.txt || exit 1
done
cat gpurun_out/r3s_sweep.txt
