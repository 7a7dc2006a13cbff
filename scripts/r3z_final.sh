#!/bin/bash
# Round-3 final evidence on one box: full GPU suite, smoke, the driver's bench command, kernel stats of the
# bench command, two PMC passes (FETCH_SIZE / WRITE_SIZE) -> HBM bytes per launch of the fp32 and AMP dominant
# kernels, per-step kernel summaries, the N>1 rehearsal.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=r3z
BENCH="bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-eval"
scripts/gpu_run.sh \
  "gputests:900:python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu" \
  "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_full:500:python3 bench.py --gpus 1 --steps 20 --warmup 5" \
  "stats:400:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_stats -o run -- python3 $BENCH" \
  "pmc_fetch:500:rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/${tag}_pmc_fetch -o run -- python3 $BENCH" \
  "pmc_write:500:rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/${tag}_pmc_write -o run -- python3 $BENCH" || exit $?
KERNEL=$(grep '^{' gpurun_out/bench_full.log | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['roofline']['kernel'].split(' (')[0])")
KAMP=$(grep '^{' gpurun_out/bench_full.log | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['amp']['roofline']['kernel'].split(' (')[0])")
python3 scripts/pmc_traffic.py gpurun_out/${tag}_pmc_fetch gpurun_out/${tag}_pmc_write --kernel "$KERNEL" \
  --out gpurun_out/${tag}_pmc_traffic.json --command "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE --kernel-trace --output-format csv -- python3 $BENCH" > gpurun_out/pmc_traffic.log 2>&1
python3 scripts/pmc_traffic.py gpurun_out/${tag}_pmc_fetch gpurun_out/${tag}_pmc_write --kernel "$KAMP" \
  --out gpurun_out/${tag}_pmc_traffic_amp.json --command "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE --kernel-trace --output-format csv -- python3 $BENCH" >> gpurun_out/pmc_traffic.log 2>&1
python3 scripts/prof_summary.py gpurun_out/${tag}_stats/run_kernel_stats.csv 11 > gpurun_out/${tag}_bench_summary.txt
bash scripts/profile_steps.sh ${tag} || exit $?
bash scripts/dist_rehearsal.sh
echo "dist rehearsal exit $?"
