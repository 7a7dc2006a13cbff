cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
scripts/gpu_run.sh "tests:400:python -u -m pytest tests/test_parity_gpu.py -q --timeout 200 --timeout-method thread -m gpu -k 'wgrad or conv2d_fwd_bwd or c2'" || exit $?
for G in 1 2; do
  echo "HYRES_WGRAD_1X1_GROUPS=$G"
  for args in "--H 128 --Ci 128 --Co 64 --K 1" "--H 128 --Ci 64 --Co 128 --K 1" "--H 256 --Ci 64 --Co 192 --K 1" "--H 32 --Ci 96 --Co 192 --K 1"; do
    HYRES_WGRAD_1X1_GROUPS=$G timeout -k 10 120 python3 scripts/wgrad_micro.py $args 2>&1 | grep wgrad || exit 1
  done
  HYRES_WGRAD_1X1_GROUPS=$G timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-eval --no-host-jpeg --no-amp > gpurun_out/w1x1_$G.json 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/w1x1_$G.json').read().strip().splitlines()[-1]); print('G=$G step', d['ms_per_step'])"
done
