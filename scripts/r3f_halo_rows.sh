cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for R in 3 1; do
  echo "HYRES_WGRAD_HALO_ROWS=$R"
  for args in "--H 128 --Ci 64 --Co 64 --K 3" "--H 256 --Ci 64 --Co 64 --K 3" "--H 32 --Ci 96 --Co 96 --K 3" "--H 128 --Ci 64 --Co 64 --K 3 --f16" "--H 256 --Ci 64 --Co 64 --K 3 --dil 2"; do
    HYRES_WGRAD_HALO_ROWS=$R timeout -k 10 120 python3 scripts/wgrad_micro.py $args 2>&1 | grep wgrad || exit 1
  done
  HYRES_WGRAD_HALO_ROWS=$R timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-eval --no-host-jpeg > gpurun_out/halo_rows_$R.json 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/halo_rows_$R.json').read().strip().splitlines()[-1]); print('step', d['ms_per_step'], 'amp', d['amp']['ms_per_step'])"
done
