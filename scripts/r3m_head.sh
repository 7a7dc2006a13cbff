cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
scripts/gpu_run.sh \
  "gputests:900:python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu" \
  "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:420:python3 bench.py --no-cpu-baseline" \
  "stats32:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3m_f32 -o run -- python3 scripts/step_profile.py --steps 10" \
  "stats16:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3m_amp -o run -- python3 scripts/step_profile.py --amp --steps 10" || exit $?
python3 scripts/prof_summary.py gpurun_out/r3m_f32/run_kernel_stats.csv 12 > gpurun_out/r3m_fp32_summary.txt
python3 scripts/prof_summary.py gpurun_out/r3m_amp/run_kernel_stats.csv 12 > gpurun_out/r3m_amp_summary.txt
