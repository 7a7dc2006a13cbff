#!/bin/bash
# SQ-counter pass (8 SQ counters) of the bf16x6 halo weight gradient in isolation (scripts/wgrad_micro.py)
set -o pipefail
tag=${1:-sqw}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
CNT="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
out=gpurun_out/${tag}_sq.txt
: > $out
run() {  # name kernel-substring micro-args...
  local n=$1 k=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d gpurun_out/${tag}_sq_$n -o run -- \
    python3 scripts/wgrad_micro.py --iters 10 "$@" > gpurun_out/${tag}_sq_$n.log 2>&1 || return 1
  echo "== $n: wgrad_micro $*" >> $out
  python3 scripts/pmc_sq.py gpurun_out/${tag}_sq_$n --kernel "$k" >> $out
}
run halo3 wgrad_halo_bf6_kernel --H 128 --Ci 64 --Co 64 --K 3 &&
run halo9 wgrad_halo_bf6_kernel --H 256 --Ci 64 --Co 64 --K 3 --dil 2 &&
run w1x1 wgrad1x1_bf6 --H 128 --Ci 64 --Co 128 --K 1
cat $out
