# round 5: the interference reproducer (guarded / unguarded) and the new GPU tests
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 100 scripts/bf6_interference_repro 20 30 wres > gpurun_out/repro3.log 2>&1 || exit 1
timeout -k 10 100 scripts/bf6_interference_repro 20 30 ru >> gpurun_out/repro3.log 2>&1 || exit 1
timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_coresidency_gpu.py \
  tests/test_parity_gpu.py::test_captured_step_survives_eager_step_with_new_layouts_and_bigger_workspace \
  tests/test_parity_gpu.py::test_captured_step_with_rccl_group_single_rank tests/test_ddp_gpu.py \
  tests/test_ru_fused_gpu.py tests/test_bf6_gpu.py -s > gpurun_out/r5_tests1.log 2>&1
echo rc=$?
