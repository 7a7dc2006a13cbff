cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
scripts/gpu_run.sh "tests:400:python -u -m pytest tests/test_parity_gpu.py -q --timeout 200 --timeout-method thread -m gpu -k 'conv2d_fwd_bwd or wres or epilogue or c2 or captured'" || exit $?
for args in "--H 128" "--H 256" "--H 128 --res --relu"; do
  timeout -k 10 120 python3 scripts/conv_micro.py $args 2>&1 | grep conv || exit 1
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-eval --no-host-jpeg --no-amp > gpurun_out/wres_epi.json 2>&1 || exit 1
python3 -c "import json,sys; d=json.loads(open('gpurun_out/wres_epi.json').read().strip().splitlines()[-1]); print('step', d['ms_per_step'], d['roofline']['frac'], d['roofline']['frac_isolated'], d['roofline']['avg_launch_us'], d['roofline']['avg_launch_us_isolated'])"
