cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
scripts/gpu_run.sh "gputests:900:python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu" || exit $?
for args in "--H 128 --Ci 64 --Co 128 --K 1 --res --relu" "--H 128 --Ci 128 --Co 64 --K 1" "--H 128 --Ci 64 --Co 128 --K 1 --res --relu --f16" "--H 32 --Ci 96 --Co 96 --K 3" "--H 32 --Ci 96 --Co 192 --K 1 --res --relu"; do
  timeout -k 10 120 python3 scripts/conv_micro.py $args 2>&1 | grep conv || exit 1
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-eval --no-host-jpeg > gpurun_out/epi2.json 2>&1 || exit 1
python3 -c "import json,sys; d=json.loads(open('gpurun_out/epi2.json').read().strip().splitlines()[-1]); print('step', d['ms_per_step'], d['roofline']['frac'], d['roofline']['frac_isolated'], 'amp', d['amp']['ms_per_step'])"
