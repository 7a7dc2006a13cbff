cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
scripts/gpu_run.sh \
  "f16act:600:python -u -m pytest tests/test_amp_f16_act_gpu.py tests/test_parity_gpu.py -v -s --timeout 200 --timeout-method thread -m gpu -k 'f16_act or fp16 or amp or c5 or f16_saved or residual_unit_chain or conv2d_fwd_bwd or deconv or gdn or narrow'" \
  "bench:420:python3 bench.py --no-cpu-baseline --no-eval --no-host-jpeg" \
  "stats_amp:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3d_amp -o run -- python3 scripts/step_profile.py --amp --steps 10" || exit $?
python3 scripts/prof_summary.py gpurun_out/r3d_amp/run_kernel_stats.csv 12 > gpurun_out/r3d_amp_summary.txt
