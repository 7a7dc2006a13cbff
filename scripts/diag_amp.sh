# AMP fixture test twice with the in-tree library and twice with hyres_hip/_alt (HYRES_LIB_PATH) -> gpurun_out/diag_amp2.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out || exit 1
timeout -k 10 300 python -u scripts/diag_amp.py --quick > gpurun_out/diag_amp2.log 2>&1 || exit $?
echo "=== alt build" >> gpurun_out/diag_amp2.log
HYRES_LIB_PATH=$GRAFT_REPO_ROOT/hyres-residual-enhanced-hybrid-image-compression_amd/hyres_hip/_alt/libhyres_hip.so \
  timeout -k 10 300 python -u scripts/diag_amp.py --quick >> gpurun_out/diag_amp2.log 2>&1
echo "exit $?" >> gpurun_out/diag_amp2.log
