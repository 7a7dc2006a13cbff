# round 5: bf16x6 halo weight gradient with branch-free raw buffer loads — parity, isolated, step
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/ -m gpu -k "wgrad or Wgrad or grad or bf6 or train_step" > gpurun_out/r5_wbuf_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r5_wbuf_tests.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/r5_wbuf_micro.log
for a in "--H 128 --Ci 64 --Co 64 --K 3" "--H 256 --Ci 64 --Co 64 --K 3" "--H 256 --Ci 64 --Co 64 --K 3 --dil 2" "--H 64 --Ci 64 --Co 64 --K 3" "--H 64 --Ci 128 --Co 128 --K 3" "--H 32 --Ci 96 --Co 96 --K 3"; do
  timeout -k 10 60 python3 scripts/wgrad_micro.py $a --iters 30 2>&1 | grep "bias=1" >> gpurun_out/r5_wbuf_micro.log || exit 1
done
cat gpurun_out/r5_wbuf_micro.log
for k in 1 2; do
  timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5_wbuf_bench_$k.log 2>&1 || exit 1
  python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/r5_wbuf_bench_$k.log') if l.startswith('{')][-1]; print('run $k step', d['ms_per_step'], 'amp', d['amp']['ms_per_step'], 'eval', d['eval']['bs16_256x256']['ms'])"
done
