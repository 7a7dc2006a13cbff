# round 5 PROBE: wgrad_halo_bf6_kernel<1,3,1,1> timed without the bf16 split's VALU work (key 15 = 1; wrong results)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/r5_nosplit_micro.log
for a in "--H 128 --Ci 64 --Co 64 --K 3" "--H 256 --Ci 64 --Co 64 --K 3" "--H 64 --Ci 128 --Co 128 --K 3"; do
  for k in 0 1 0 1; do
    HYRES_TUNE=15=$k timeout -k 10 60 python3 scripts/wgrad_micro.py $a --iters 30 2>&1 | grep "bias=0" | sed "s/^/nosplit=$k /" >> gpurun_out/r5_nosplit_micro.log || exit 1
  done
done
cat gpurun_out/r5_nosplit_micro.log
