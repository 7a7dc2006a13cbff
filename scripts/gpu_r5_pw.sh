# round 5: SA / SE pointwise kernels (32-bit indices, 4 float4 in flight) — parity, isolated, serial eval profile
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_parity_gpu.py \
  -k "bilinear_se_spatial or refine_branch or fp16_activation_ops or c2_size or amp_train_step_vs_fp32" -s > gpurun_out/r5_pw_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -a "passed\|failed" gpurun_out/r5_pw_tests.log | tail -1; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 scripts/refine_micro.py 2>&1 | grep us
cd /tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5q_eval_serial -o run -- python3 scripts/step_profile.py --eval --serial --marker --steps 20 > gpurun_out/r5q.log 2>&1 || exit 1
python3 scripts/prof_summary.py gpurun_out/r5q_eval_serial/run_kernel_trace.csv 20 > gpurun_out/r5q_eval_serial_summary.txt
grep -a "sa_\|se_\|total" gpurun_out/r5q_eval_serial_summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5p_train_serial -o run -- python3 scripts/step_profile.py --serial --marker --steps 10 > gpurun_out/r5p.log 2>&1 || exit 1
python3 scripts/prof_summary.py gpurun_out/r5p_train_serial/run_kernel_trace.csv 10 > gpurun_out/r5p_train_serial_summary.txt
head -70 gpurun_out/r5p_train_serial_summary.txt
