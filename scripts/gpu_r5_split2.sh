# round 5: split cap sweep for the AMP (fp16-operand) weight gradients and the 256^2 fp32 ones
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/r5_split2_micro.log
for a in "--H 128 --Ci 64 --Co 64 --K 3 --f16" "--H 256 --Ci 64 --Co 64 --K 3 --dil 2 --f16" "--H 128 --Ci 64 --Co 128 --K 1 --f16" "--H 32 --Ci 96 --Co 96 --K 3 --f16" "--H 64 --Ci 128 --Co 128 --K 3 --f16" "--H 256 --Ci 64 --Co 64 --K 3" "--H 256 --Ci 64 --Co 64 --K 1"; do
  for k in 512 256 128 64 32; do
    HYRES_TUNE=6=$k timeout -k 10 60 python3 scripts/wgrad_micro.py $a --iters 30 2>&1 | grep "bias=1" | sed "s/^/maxsplit=$k /" >> gpurun_out/r5_split2_micro.log || exit 1
  done
done
cat gpurun_out/r5_split2_micro.log
