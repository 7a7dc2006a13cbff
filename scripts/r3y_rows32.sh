cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
scripts/gpu_run.sh \
  "step:400:for i in 1 2 3; do for r in 3 1; do echo == rows=\$r; HYRES_WGRAD_HALO_ROWS=\$r python3 scripts/step_profile.py --steps 30; done; done" \
  "stats1:300:HYRES_WGRAD_HALO_ROWS=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3y_rows1 -o run -- python3 scripts/step_profile.py --steps 10" || exit $?
python3 scripts/prof_summary.py gpurun_out/r3y_rows1/run_kernel_stats.csv 12 > gpurun_out/r3y_rows1_summary.txt
