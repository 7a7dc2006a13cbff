# round 5: wgrad1x1_bf6 prefetch depth (key 13) and wres_bf6 V1 default — bit-identity, micro A/B, step A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_bf6_gpu.py tests/test_stream_b6_gpu.py -k "variants or prefetch or stream_b6" -s \
  > gpurun_out/r5_wg_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/r5_wg_micro.log
for rep in 1 2; do
for args in "--Ci 64 --Co 128" "--Ci 128 --Co 64" "--Ci 128 --Co 128" "--Ci 64 --Co 64 --H 256"; do
  for pf in 1 2; do
    timeout -k 10 60 python -u scripts/wgrad_micro.py $args --pf $pf --iters 50 2>&1 | grep wgrad >> gpurun_out/r5_wg_micro.log || exit 1
  done
done
done
for args in "--H 128 --Ci 64 --Co 128 --K 1 --res --relu" "--H 128 --Ci 128 --Co 64 --K 1 --relu" \
            "--H 64 --Ci 64 --Co 128 --K 1 --res --relu" "--H 256 --Ci 64 --Co 64 --K 1 --relu"; do
  for cm in 1 2; do
    timeout -k 10 60 python -u scripts/conv_micro.py --bf6 $args --stream-cm $cm --iters 50 2>&1 | grep conv >> gpurun_out/r5_wg_micro.log || exit 1
  done
done
cat gpurun_out/r5_wg_micro.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-eval --no-cpu-baseline > gpurun_out/r5_wg_bench_pf1.log 2>&1 || exit 1
HYRES_TUNE=13=2 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-eval --no-cpu-baseline > gpurun_out/r5_wg_bench_pf2.log 2>&1 || exit 1
HYRES_TUNE=11=2 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-eval --no-cpu-baseline > gpurun_out/r5_wg_bench_cx.log 2>&1 || exit 1
HYRES_TUNE=12=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-eval --no-cpu-baseline > gpurun_out/r5_wg_bench_v0.log 2>&1 || exit 1
for f in pf1 pf2 cx v0; do python3 -c "
import json,sys; d=json.loads([l for l in open('gpurun_out/r5_wg_bench_$f.log') if l.startswith('{')][-1]); print('$f', d['ms_per_step'], d['value'], d['amp']['ms_per_step'] if 'amp' in d else '')"; done
