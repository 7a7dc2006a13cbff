#!/bin/bash
# Round profile: bench (with CPU baseline), kernel-trace stats, and two separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) of the same bench command.  Usage: scripts/profile_round.sh <tag>
set -o pipefail
tag=${1:-r1}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
BENCH="bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-eval"
scripts/gpu_run.sh \
  "bench_full:420:python3 bench.py" \
  "stats:400:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_stats -o run -- python3 $BENCH" \
  "pmc_fetch:500:rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/${tag}_pmc_fetch -o run -- python3 $BENCH" \
  "pmc_write:500:rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/${tag}_pmc_write -o run -- python3 $BENCH"
rc=$?
[ $rc -ne 0 ] && exit $rc
# the dominant kernel named by the bench line's roofline (label in parentheses stripped)
KERNEL=$(grep '^{' gpurun_out/bench_full.log | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['roofline']['kernel'].split(' (')[0])")
python3 scripts/pmc_traffic.py gpurun_out/${tag}_pmc_fetch gpurun_out/${tag}_pmc_write \
  --kernel "$KERNEL" --out gpurun_out/${tag}_pmc_traffic.json \
  --command "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE --kernel-trace --output-format csv -- python3 $BENCH" \
  > gpurun_out/pmc_traffic.log 2>&1 && \
python3 scripts/prof_summary.py gpurun_out/${tag}_stats/run_kernel_stats.csv 11 > gpurun_out/${tag}_summary.txt
scripts/profile_steps.sh ${tag}
