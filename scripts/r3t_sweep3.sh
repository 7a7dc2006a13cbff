cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() { echo "== $1"; for m in "--amp" ""; do timeout -k 10 120 env $1 python3 scripts/step_profile.py --steps 30 $m 2>&1 | grep "ms/step" || return 1; done; }
for cfg in "HYRES_X=0" "HYRES_CONV_SPLIT_BLOCKS=256" "HYRES_CONV_SMALL_PIXELS=16384" "HYRES_CONV_SMALL_PIXELS=262144" "HYRES_CONV_SHORTK=0" "HYRES_CONV_HALO16=0" "HYRES_X=0" "HYRES_CONV_SPLIT_BLOCKS=256" "HYRES_CONV_SMALL_PIXELS=16384" "HYRES_CONV_SMALL_PIXELS=262144" "HYRES_CONV_SHORTK=0" "HYRES_CONV_HALO16=0" "HYRES_X=0"; do
  run "$cfg" >> gpurun_out/r3t_sweep.txt || exit 1
done
cat gpurun_out/r3t_sweep.txt
