#!/bin/bash
# FETCH_SIZE / WRITE_SIZE and SQ passes of the conv families furthest below their roofline (VERDICT r5 "What's weak" 4),
# each in isolation on its step geometry (scripts/conv_micro.py): one rocprofv3 run per counter set and kernel, each
# under its own time limit. Summaries -> gpurun_out/<tag>_pmc_families.txt
set -o pipefail
tag=${1:-fam}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}_pmc_families.txt
: > $out
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
fam() {  # name kernel-substring micro-args... (MICRO=scripts/wgrad_micro.py for the weight-gradient kernels)
  local n=$1 k=$2; shift 2
  local M=${MICRO:-scripts/conv_micro.py}
  local d=gpurun_out/${tag}_fam_$n
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d ${d}_f -o run -- \
    python3 $M --iters 10 "$@" > ${d}_f.log 2>&1 || return 1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d ${d}_w -o run -- \
    python3 $M --iters 10 "$@" > ${d}_w.log 2>&1 || return 1
  timeout -s KILL 90 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d ${d}_sq -o run -- \
    python3 $M --iters 10 "$@" > ${d}_sq.log 2>&1 || return 1
  python3 $M --iters 50 "$@" > ${d}_t.log 2>&1 || return 1
  echo "== $n: conv_micro $*  ($(grep -h 'us' ${d}_t.log | tail -1))" >> $out
  python3 scripts/pmc_traffic.py ${d}_f ${d}_w --kernel "$k" --out ${d}_traffic.json | \
    python3 -c "import json,sys; d=json.load(sys.stdin); print('  kernel', d['kernel'][:70]); print('  HBM bytes per launch (2 x FETCH + WRITE)', round(d['traffic_bytes_per_launch'] / 1e6, 2), 'MB')" >> $out
  python3 scripts/pmc_sq.py ${d}_sq --kernel "$k" >> $out
}
if [ "$2" = thin ]; then  # the image-side thin weight gradients (wgrad_thin_kernel)
  MICRO=scripts/wgrad_micro.py fam thin_3to64 wgrad_thin --H 256 --Ci 3 --Co 64 --K 3 &&
  MICRO=scripts/wgrad_micro.py fam thin_64to3 wgrad_thin --H 256 --Ci 64 --Co 3 --K 3 &&
  MICRO=scripts/wgrad_micro.py fam thin_5x5s2 wgrad_thin --H 256 --Ci 3 --Co 128 --K 5 --stride 2
  exit $?
fi
MICRO=scripts/wgrad_micro.py fam wg_halo_128 wgrad_halo_bf6 --H 128 --Ci 64 --Co 64 --K 3 &&
MICRO=scripts/wgrad_micro.py fam wg_1x1_128 wgrad1x1_bf6 --H 128 --Ci 128 --Co 128 --K 1 &&
fam b6_32_3x3 conv_fwd_b6_kernel --H 32 --Ci 96 --Co 96 --K 3 --relu --bf6 &&
fam b6_1x1_32res conv_fwd_b6_kernel --H 32 --Ci 96 --Co 192 --K 1 --res --relu --bf6 &&
fam stream_mask conv1x1_stream_b6_kernel --H 128 --Ci 128 --Co 64 --K 1 --mask --bf6
