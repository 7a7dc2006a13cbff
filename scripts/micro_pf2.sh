#!/bin/bash
# small-grid convs (64-row tiles): K-loop prefetch distance 2 (conv_fwd_pf2_kernel) vs 1
set -o pipefail
for env in "HYRES_CONV_PF2=1" "HYRES_CONV_PF2=0"; do
  echo "== $env"
  for args in "--H 32 --Ci 96 --Co 96 --K 3" "--H 32 --Ci 192 --Co 384 --K 3" "--H 32 --Ci 384 --Co 192 --K 3" \
              "--H 64 --Ci 64 --Co 64 --K 3" "--H 32 --Ci 192 --Co 96 --K 1" "--H 32 --Ci 512 --Co 640 --K 1" \
              "--H 64 --Ci 128 --Co 192 --K 5 --stride 2" "--H 32 --Ci 96 --Co 96 --K 3 --f16" "--H 32 --Ci 384 --Co 192 --K 3 --f16"; do
    env $env timeout -k 10 60 python3 scripts/conv_micro.py $args --iters 50 || exit $?
  done
done
