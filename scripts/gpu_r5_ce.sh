# round 5: coalesced (LDS-staged) epilogue of the bf16x6 streaming 1x1 kernel — parity, micro A/B, then the bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_stream_b6_gpu.py -s \
  > gpurun_out/r5_ce_tests.log 2>&1
echo "tests rc=$?"
rm -f gpurun_out/r5_ce_micro.log
for args in "--H 128 --Ci 64 --Co 128 --K 1 --res --relu" "--H 128 --Ci 128 --Co 64 --K 1 --relu" \
            "--H 64 --Ci 64 --Co 128 --K 1 --res --relu" "--H 256 --Ci 64 --Co 64 --K 1 --relu" \
            "--H 256 --Ci 64 --Co 64 --K 1 --res"; do
  for v in "" "--stream-cm 0" "--no-stream-b6"; do
    timeout -k 10 60 python -u scripts/conv_micro.py --bf6 $args $v --iters 50 2>&1 | grep conv >> gpurun_out/r5_ce_micro.log || exit 1
  done
done
cat gpurun_out/r5_ce_micro.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_bench_ce.log 2>&1
echo "bench rc=$?"
tail -1 gpurun_out/r5_bench_ce.log
