cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
scripts/gpu_run.sh \
  "defer_tests:400:python -u -m pytest tests/test_wgrad_defer_gpu.py tests/test_engine_gpu.py tests/test_ddp_gpu.py -x -v --timeout 200 --timeout-method thread -m gpu" \
  "step_on:200:python3 scripts/step_profile.py --steps 20 && python3 scripts/step_profile.py --amp --steps 20" \
  "step_off:200:HYRES_WGRAD_DEFER=0 python3 scripts/step_profile.py --steps 20 && HYRES_WGRAD_DEFER=0 python3 scripts/step_profile.py --amp --steps 20" \
  "stats32:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3n_f32 -o run -- python3 scripts/step_profile.py --steps 10" \
  "stats16:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3n_amp -o run -- python3 scripts/step_profile.py --amp --steps 10" || exit $?
python3 scripts/prof_summary.py gpurun_out/r3n_f32/run_kernel_stats.csv 12 > gpurun_out/r3n_fp32_summary.txt
python3 scripts/prof_summary.py gpurun_out/r3n_amp/run_kernel_stats.csv 12 > gpurun_out/r3n_amp_summary.txt
