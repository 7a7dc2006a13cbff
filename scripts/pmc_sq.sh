#!/bin/bash
# SQ-counter passes (one pass, 8 SQ counters) of the bf16x6 kernels in isolation (scripts/conv_micro.py), one
# rocprofv3 run per kernel under its own time limit; summaries -> gpurun_out/<tag>_sq.txt
set -o pipefail
tag=${1:-sq}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
CNT="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
out=gpurun_out/${tag}_sq.txt
: > $out
run() {  # name kernel-substring micro-args...
  local n=$1 k=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d gpurun_out/${tag}_sq_$n -o run -- \
    python3 scripts/conv_micro.py --iters 10 "$@" > gpurun_out/${tag}_sq_$n.log 2>&1 || return 1
  echo "== $n: conv_micro $*" >> $out
  python3 scripts/pmc_sq.py gpurun_out/${tag}_sq_$n --kernel "$k" >> $out
}
run wres_bf6 conv3x3_wres_bf6 --H 128 --bf6 &&
run wres_f32 conv3x3_wres_f32 --H 128 &&
run b6_1x1 conv_fwd_b6 --H 128 --Ci 64 --Co 128 --K 1 --res --relu --bf6 &&
run b6_32 conv_fwd_b6 --H 32 --Ci 96 --Co 96 --K 3 --relu --bf6
