#!/bin/bash
# 1x1 conv geometries of the C2 step: streaming kernel (occupancy-sized / 2 blocks per CU) and the tiled kernel
set -o pipefail
for env in "HYRES_CONV_STREAM1X1=1" "HYRES_CONV_STREAM_BLOCKS_PER_CU=2" "HYRES_CONV_STREAM1X1=0"; do
  echo "== $env"
  for args in "--H 128 --Ci 64 --Co 128 --K 1 --res --relu" "--H 128 --Ci 128 --Co 64 --K 1 --relu" \
              "--H 128 --Ci 128 --Co 128 --K 1" "--H 256 --Ci 64 --Co 192 --K 1" \
              "--H 32 --Ci 96 --Co 192 --K 1 --res --relu" "--H 32 --Ci 192 --Co 96 --K 1 --relu" \
              "--H 64 --Ci 64 --Co 128 --K 1 --res --relu" "--H 128 --Ci 64 --Co 128 --K 1 --res --relu --f16"; do
    env $env timeout -k 10 60 python3 scripts/conv_micro.py $args --iters 30 || exit $?
  done
done
