# round 5: SpatialAttention multiply folded into the fusion 1x1 (inference) — parity, eval A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bf6_gpu.py tests/test_parity_gpu.py \
  -k "sa_mul_fold or model_eval_matches or c3_bs32 or c5_kodak or fp16_activation_ops or autocast_eval or amp_matches" -s > gpurun_out/r5_fold_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -a "passed\|failed\|folded vs" gpurun_out/r5_fold_tests.log | tail -4; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for f in 1 0; do
  HYRES_FOLD_SA_MUL=$f timeout -k 10 120 python3 scripts/step_profile.py --eval --steps 30 2>&1 | grep "ms/step" | sed "s/^/fold=$f /"
  HYRES_FOLD_SA_MUL=$f timeout -k 10 120 python3 scripts/step_profile.py --eval --amp --steps 30 2>&1 | grep "ms/step" | sed "s/^/fold=$f /"
done; done
