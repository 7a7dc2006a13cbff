#!/bin/bash
# HBM traffic + SQ counters of the 128^2 64->128 +res 1x1 conv (the RU / RBB tail), one pass each
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
M="scripts/conv_micro.py --H 128 --Ci 64 --Co 128 --K 1 --res --relu --iters 20"
timeout -k 10 60 python3 scripts/bw_probe.py > gpurun_out/bw_probe.log 2>&1 || exit $?
timeout -k 10 60 python3 $M > gpurun_out/m1x1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/p1x1_f -o run -- python3 $M > gpurun_out/p1x1_f.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/p1x1_w -o run -- python3 $M > gpurun_out/p1x1_w.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/p1x1_s -o run -- python3 $M > gpurun_out/p1x1_s.log 2>&1 || exit $?
