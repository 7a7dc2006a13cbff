# round 5: bf16x6 halo weight gradient with hand-issued transposed reads one unit ahead (hyres_conv_tuning key 15 = 1) — bit identity, isolated, step
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_bf6_gpu.py -k read_ahead -s > gpurun_out/r5_ra_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -a "read-ahead:\|passed\|failed" gpurun_out/r5_ra_tests.log | tail -4; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/r5_ra_micro.log
for a in "--H 128 --Ci 64 --Co 64 --K 3" "--H 256 --Ci 64 --Co 64 --K 3" "--H 64 --Ci 64 --Co 64 --K 3" "--H 64 --Ci 128 --Co 128 --K 3" "--H 32 --Ci 96 --Co 96 --K 3"; do
  for k in 0 1; do
    HYRES_TUNE=15=$k timeout -k 10 60 python3 scripts/wgrad_micro.py $a --iters 30 2>&1 | grep "bias=1" | sed "s/^/ra=$k /" >> gpurun_out/r5_ra_micro.log || exit 1
  done
done
cat gpurun_out/r5_ra_micro.log
for k in 1 0 1 0; do
  HYRES_TUNE=15=$k timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5_ra_bench.log 2>&1 || exit 1
  python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/r5_ra_bench.log') if l.startswith('{')][-1]; print('ra=$k step', d['ms_per_step'], 'amp', d['amp']['ms_per_step'])"
done
