cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
scripts/gpu_run.sh \
  "amp:400:python -u -m pytest tests/test_parity_gpu.py -v -s --timeout 200 --timeout-method thread -m gpu -k 'amp_fwd_bwd or amp_train or amp_matches'" \
  "bench:420:python3 bench.py --no-cpu-baseline" \
  "stats_amp:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3b_amp -o run -- python3 scripts/step_profile.py --amp --steps 10" || exit $?
python3 scripts/prof_summary.py gpurun_out/r3b_amp/run_kernel_stats.csv 12 > gpurun_out/r3b_amp_summary.txt
scripts/gpu_run.sh \
  "as_fetch:200:rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/r3_as_fetch -o run -- python3 scripts/as_traffic.py" \
  "as_write:200:rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/r3_as_write -o run -- python3 scripts/as_traffic.py" || exit $?
python3 scripts/as_traffic.py --summarize gpurun_out/r3_as_fetch gpurun_out/r3_as_write --out gpurun_out/r3_as_traffic.json
