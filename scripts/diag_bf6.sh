# bf16x6 concurrency diagnostics (tests/test_bf6_gpu.py, printed): in-tree library, then the alternative build in
# hyres_hip/_alt (HYRES_LIB_PATH) -> gpurun_out/diag_bf6.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out || exit 1
K="beside"
timeout -k 10 300 python -u -m pytest tests/test_bf6_gpu.py -v -s -k "$K" --timeout 180 --timeout-method thread -m gpu > gpurun_out/diag_bf6.log 2>&1 || exit $?
ALT=$GRAFT_REPO_ROOT/hyres-residual-enhanced-hybrid-image-compression_amd/hyres_hip/_alt/libhyres_hip.so
[ -f "$ALT" ] || { echo "exit 0 (no alternative build)" >> gpurun_out/diag_bf6.log; exit 0; }
echo "=== alt build" >> gpurun_out/diag_bf6.log
HYRES_LIB_PATH=$GRAFT_REPO_ROOT/hyres-residual-enhanced-hybrid-image-compression_amd/hyres_hip/_alt/libhyres_hip.so \
  timeout -k 10 300 python -u -m pytest tests/test_bf6_gpu.py -v -s -k "$K" --timeout 180 --timeout-method thread -m gpu >> gpurun_out/diag_bf6.log 2>&1
echo "exit $?" >> gpurun_out/diag_bf6.log
