#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the 3x3 64->64 conv (128^2 and 256^2, B16) with and without the XCD-aware
# tile order (HYRES_CONV_XCD). Separate --pmc passes, as the microarch guide prescribes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for xcd in 0 1; do
  for H in 128 256; do
    for c in FETCH_SIZE WRITE_SIZE; do
      HYRES_CONV_XCD=$xcd timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv \
        -d gpurun_out/pmcx_${xcd}_${H}_${c} -o run -- python3 scripts/conv_micro.py --H $H --iters 20 \
        > gpurun_out/pmcx_${xcd}_${H}_${c}.log 2>&1 || exit $?
    done
  done
done
