#!/bin/bash
# Per-kernel stats of the fp32 and AMP train steps: 10 replayed steps each, counted from the kernel trace after
# the marker kernel (the capture's eager warm-up passes and the 2 warm-up replays excluded):
# scripts/profile_steps.sh <tag>
set -o pipefail
tag=${1:-r2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
scripts/gpu_run.sh \
  "stats_fp32:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_fp32 -o run -- python3 scripts/step_profile.py --marker --steps 10" \
  "stats_amp:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_amp -o run -- python3 scripts/step_profile.py --marker --amp --steps 10" || exit $?
python3 scripts/prof_summary.py gpurun_out/${tag}_fp32/run_kernel_trace.csv 10 > gpurun_out/${tag}_fp32_summary.txt && \
python3 scripts/prof_summary.py gpurun_out/${tag}_amp/run_kernel_trace.csv 10 > gpurun_out/${tag}_amp_summary.txt
