cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
M="python scripts/wgrad_micro.py"
scripts/gpu_run.sh \
  "tests:400:python -u -m pytest tests/test_wgrad_defer_gpu.py tests/test_ddp_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu && python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k 'conv2d or wgrad or halo or amp or train_step or c2'" \
  "micro:300:for g in 1 2; do echo G=\$g; HYRES_WGRAD_HALO_GROUPS=\$g $M --H 128 --Ci 64 --Co 64 --K 3; HYRES_WGRAD_HALO_GROUPS=\$g $M --H 256 --Ci 64 --Co 64 --K 3; HYRES_WGRAD_HALO_GROUPS=\$g $M --H 128 --Ci 64 --Co 64 --K 3 --f16; HYRES_WGRAD_HALO_GROUPS=\$g $M --H 256 --Ci 64 --Co 64 --K 3 --dil 2; done" \
  "step:300:for g in 1 2 1 2; do HYRES_WGRAD_HALO_GROUPS=\$g python3 scripts/step_profile.py --steps 20; HYRES_WGRAD_HALO_GROUPS=\$g python3 scripts/step_profile.py --amp --steps 20; done" \
  "stats32:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3o_f32 -o run -- python3 scripts/step_profile.py --steps 10" \
  "stats16:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3o_amp -o run -- python3 scripts/step_profile.py --amp --steps 10" || exit $?
python3 scripts/prof_summary.py gpurun_out/r3o_f32/run_kernel_stats.csv 12 > gpurun_out/r3o_fp32_summary.txt
python3 scripts/prof_summary.py gpurun_out/r3o_amp/run_kernel_stats.csv 12 > gpurun_out/r3o_amp_summary.txt
