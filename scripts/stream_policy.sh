#!/bin/bash
# C2 train-step time (graph replay) under different stream-concurrency policies
set -o pipefail
export PYTHONWARNINGS=ignore
run() { echo "== $1 $2"; env $1 timeout -k 10 120 python3 -W ignore scripts/step_profile.py --steps 20 $2 2>&1 | grep ms/step || exit 1; }
for amp in "" "--amp"; do
  for env in "X=0" "HYRES_SIDE_STREAM=0" "HYRES_SIDE_STREAM=0 HYRES_BRANCH_MAX_PIXELS=65536" \
             "HYRES_SIDE_STREAM=0 HYRES_BRANCH_MAX_PIXELS=16384" "X=1" "HYRES_SIDE_STREAM=0"; do
    run "$env" "$amp"
  done
done
