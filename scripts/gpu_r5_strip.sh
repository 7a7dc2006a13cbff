# round 5: conv_narrow_strip_kernel (key 13) — parity, isolated A/B, eval / train step A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bf6_gpu.py tests/test_parity_gpu.py \
  -k "narrow_strip or fp16_activation_ops or deconv2d_fwd_bwd or conv2d_fwd_bwd or model_eval_matches or c2_size or refine_branch_fwd" -s > gpurun_out/r5_strip_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -a "passed\|failed" gpurun_out/r5_strip_tests.log | tail -1; [ $rc -eq 0 ] || exit $rc
grep -a "error vs fp64: strip" gpurun_out/r5_strip_tests.log | cut -c1-200
rm -f gpurun_out/r5_strip_micro.log
for a in "--H 256 --Ci 64 --Co 3 --K 3" "--H 128 --Ci 128 --Co 3 --K 3"; do
  for k in 1 0; do
    HYRES_TUNE=13=$k timeout -k 10 60 python3 scripts/conv_micro.py --bf6 $a --iters 50 2>&1 | grep conv | sed "s/^/key13=$k /" >> gpurun_out/r5_strip_micro.log || exit 1
  done
done
cat gpurun_out/r5_strip_micro.log
for r in 1 2; do for k in 1 0; do
  HYRES_TUNE=13=$k timeout -k 10 120 python3 scripts/step_profile.py --eval --steps 30 2>&1 | grep "ms/step" | sed "s/^/key13=$k /"
  HYRES_TUNE=13=$k timeout -k 10 120 python3 scripts/step_profile.py --steps 20 2>&1 | grep "ms/step" | sed "s/^/key13=$k /"
done; done
