# round 5: conv3x3_wres_bf6_kernel scheduling variants (key 12) — bit-identity, then isolated timings
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_bf6_gpu.py -k "variants or as_accurate" -s \
  > gpurun_out/r5_wres_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/r5_wres_micro.log
for rep in 1 2; do
for args in "--H 128" "--H 128 --res --relu" "--H 256"; do
  for v in 0 1 2 3; do
    timeout -k 10 60 python -u scripts/conv_micro.py --bf6 $args --wres-v $v --iters 100 2>&1 | grep conv >> gpurun_out/r5_wres_micro.log || exit 1
  done
done
done
cat gpurun_out/r5_wres_micro.log
