cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
scripts/gpu_run.sh \
  "t32:200:python3 scripts/step_profile.py --steps 10 --marker && python3 scripts/step_profile.py --steps 10 --marker --amp" \
  "f32:200:rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/r3u_f32_fetch -o run -- python3 scripts/step_profile.py --steps 10 --marker" \
  "w32:200:rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/r3u_f32_write -o run -- python3 scripts/step_profile.py --steps 10 --marker" \
  "f16:200:rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/r3u_amp_fetch -o run -- python3 scripts/step_profile.py --steps 10 --marker --amp" \
  "w16:200:rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/r3u_amp_write -o run -- python3 scripts/step_profile.py --steps 10 --marker --amp" || exit $?
M32=$(grep "train fp32" gpurun_out/t32.log | awk '{print $3}')
M16=$(grep "train amp" gpurun_out/t32.log | awk '{print $3}')
python3 scripts/step_traffic.py gpurun_out/r3u_f32_fetch gpurun_out/r3u_f32_write --steps 10 --ms $M32 --what "C2 train step fp32 (graph replay + Adam + aux)" --out gpurun_out/r3u_step_traffic_fp32.json
python3 scripts/step_traffic.py gpurun_out/r3u_amp_fetch gpurun_out/r3u_amp_write --steps 10 --ms $M16 --what "C2 train step AMP (graph replay + GradScaler Adam + aux)" --out gpurun_out/r3u_step_traffic_amp.json
