cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
scripts/gpu_run.sh \
  "lt_fp32:300:python3 scripts/layer_table.py" \
  "stats_fp32:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3j_fp32 -o run -- python3 scripts/step_profile.py --steps 10" || exit $?
python3 scripts/prof_summary.py gpurun_out/r3j_fp32/run_kernel_stats.csv 12 > gpurun_out/r3j_fp32_summary.txt
