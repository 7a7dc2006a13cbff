#!/bin/bash
# A/B of the in-tree library against an alternative build (hyres_hip/_alt/libhyres_hip.so, HYRES_LIB_PATH) on one
# box: the bf16x6 3x3 micro at 128^2 / 256^2 and the C2 train step (headline only), alternating, twice.
# Output: gpurun_out/<tag>_ab.txt
set -o pipefail
tag=${1:-ab}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ALT=$GRAFT_REPO_ROOT/hyres-residual-enhanced-hybrid-image-compression_amd/hyres_hip/_alt/libhyres_hip.so
out=gpurun_out/${tag}_ab.txt
: > $out
for rep in 1 2; do
  for v in main alt; do
    if [ $v = alt ]; then export HYRES_LIB_PATH=$ALT; else unset HYRES_LIB_PATH; fi
    for H in 128 256; do
      timeout -k 10 120 python3 scripts/conv_micro.py --H $H --bf6 --res --relu > gpurun_out/ab_micro.log 2>&1 || exit 1
      echo "$v rep$rep $(grep 'us,' gpurun_out/ab_micro.log)" >> $out
    done
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-eval --no-amp --no-host-jpeg --no-cpu-baseline \
      > gpurun_out/ab_bench.log 2>&1 || exit 1
    echo "$v rep$rep $(grep '^{' gpurun_out/ab_bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("step", d["ms_per_step"], "ms;", d["roofline"]["kernel"][:28], d["roofline"]["avg_launch_us"], "us live,", d["roofline"]["avg_launch_us_isolated"], "us isolated")')" >> $out
  done
done
unset HYRES_LIB_PATH
cat $out
