# round 5: weight-gradient split-K block target (hyres_conv_tuning key 3, default 2048; 4096 on small grids) re-swept on the bf16x6 step
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in -1 1024 4096 -1 1024 4096; do
  HYRES_TUNE=3=$k timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5_wblocks_bench.log 2>&1 || exit 1
  python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/r5_wblocks_bench.log') if l.startswith('{')][-1]; print('wgradblocks=$k step', d['ms_per_step'], 'amp', d['amp']['ms_per_step'], 'eval', d['eval']['bs16_256x256']['ms'])"
done
