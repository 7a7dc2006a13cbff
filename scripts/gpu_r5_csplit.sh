# round 5: conv split-K block target (hyres_conv_tuning key 1, default 512) re-swept on the bf16x6 step
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in -1 1024 256 -1 1024 256; do
  HYRES_TUNE=1=$k timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5_csplit_bench.log 2>&1 || exit 1
  python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/r5_csplit_bench.log') if l.startswith('{')][-1]; print('splitblocks=$k step', d['ms_per_step'], 'amp', d['amp']['ms_per_step'], 'eval', d['eval']['bs16_256x256']['ms'])"
done
