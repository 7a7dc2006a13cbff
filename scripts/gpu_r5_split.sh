# round 5: weight-gradient split cap (hyres_conv_tuning key 6; new per-family default) — step A/B vs 512 everywhere
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 0 512 0 512; do
  HYRES_TUNE=6=$k timeout -k 10 240 python3 -X faulthandler bench.py --steps 20 --warmup 5 > gpurun_out/r5_split_bench_$k.log 2>&1 || { tail -40 gpurun_out/r5_split_bench_$k.log; exit 1; }
  python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/r5_split_bench_$k.log') if l.startswith('{')][-1]; print('maxsplit=$k step', d['ms_per_step'], 'amp', d['amp']['ms_per_step'], 'eval', d['eval']['bs16_256x256']['ms'])"
done
