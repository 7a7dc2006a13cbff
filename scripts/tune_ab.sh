#!/bin/bash
# Same-box A/B of environment variants of the C2 train step (and the AMP leg): scripts/tune_ab.sh <tag> "<label>=<env>"...
# e.g. "default=" "nopf2=HYRES_TUNE=15=1,16=1" — each variant's bench.py line, alternating, twice.
# Output: gpurun_out/<tag>_tune_ab.txt
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}_tune_ab.txt
: > $out
for rep in 1 2; do
  for spec in "$@"; do
    label=${spec%%=*}; envs=${spec#*=}
    timeout -k 10 300 env $envs python3 bench.py --steps 20 --warmup 5 --no-eval --no-host-jpeg --no-cpu-baseline \
      > gpurun_out/tune_ab_bench.log 2>&1 || exit 1
    echo "$label rep$rep [$envs] $(grep '^{' gpurun_out/tune_ab_bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("fp32 step", d["ms_per_step"], "ms, AMP step", d["amp"]["ms_per_step"], "ms, AMP dominant", d["amp"]["roofline"]["kernel"][:40], d["amp"]["roofline"]["frac"])')" >> $out
  done
done
cat $out
