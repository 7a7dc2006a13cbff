# round 5: weight-resident bf16x6 3x3 at dilation 2 — parity, isolated A/B, eval / train step A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bf6_gpu.py tests/test_parity_gpu.py \
  -k "dilation2 or refine_layers_match_native or refine_branch or c2_size or model_eval_matches or wres_bf6_variants or kernels_beside" -s > gpurun_out/r5_dil_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -a "passed\|failed" gpurun_out/r5_dil_tests.log | tail -1; [ $rc -eq 0 ] || exit $rc
grep -a "y vs fp64: wres" gpurun_out/r5_dil_tests.log | cut -c1-220
rm -f gpurun_out/r5_dil_micro.log
for a in "--H 256 --dil 2" "--H 128 --dil 2" "--H 64 --dil 2" "--H 128"; do
  for k in 1 0; do
    HYRES_TUNE=14=$k timeout -k 10 60 python3 scripts/conv_micro.py --bf6 $a --iters 30 2>&1 | grep conv | sed "s/^/wres=$k /" >> gpurun_out/r5_dil_micro.log || exit 1
  done
done
cat gpurun_out/r5_dil_micro.log
timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5_dil_bench.log 2>&1 || exit 1
tail -c 600 gpurun_out/r5_dil_bench.log
