# round 5: all 9 taps per block for the dilation-1 bf16x6 3x3 weight gradients (hyres_conv_tuning key 15 = 1) vs rows of 3
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/r5_rows_micro.log
for a in "--H 128 --Ci 64 --Co 64 --K 3" "--H 256 --Ci 64 --Co 64 --K 3" "--H 64 --Ci 64 --Co 64 --K 3" "--H 64 --Ci 128 --Co 128 --K 3" "--H 32 --Ci 96 --Co 96 --K 3"; do
  for k in 0 1; do
    HYRES_TUNE=15=$k timeout -k 10 60 python3 scripts/wgrad_micro.py $a --iters 30 2>&1 | grep "bias=1" | sed "s/^/all9=$k /" >> gpurun_out/r5_rows_micro.log || exit 1
  done
done
cat gpurun_out/r5_rows_micro.log
