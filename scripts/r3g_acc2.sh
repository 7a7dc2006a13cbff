cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for A in 0 1 0 1; do
  echo "HYRES_WRES32_ACC2=$A"
  for args in "--H 128" "--H 256" "--H 128 --res --relu"; do
    HYRES_WRES32_ACC2=$A timeout -k 10 120 python3 scripts/conv_micro.py $args 2>&1 | grep conv || exit 1
  done
done
for A in 0 1; do
  HYRES_WRES32_ACC2=$A timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-eval --no-host-jpeg --no-amp > gpurun_out/acc2_$A.json 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/acc2_$A.json').read().strip().splitlines()[-1]); print('ACC2=$A step', d['ms_per_step'], d['roofline']['frac'], d['roofline']['frac_isolated'])"
done
