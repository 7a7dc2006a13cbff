# round 5: which change moved the AMP fixture's refine.act_in slope distance (split cap key 6, narrow strip key 13)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for t in "" "6=512" "13=0" "6=512,13=0"; do
  HYRES_TUNE=$t timeout -k 10 200 python -u -m pytest tests/test_parity_gpu.py -q --timeout 180 --timeout-method thread -m gpu -s -k test_amp_matches_reference_autocast_fixture > gpurun_out/r5_ampfix.log 2>&1
  rc=$?; [ $rc -le 1 ] || exit $rc
  echo "HYRES_TUNE=$t rc=$rc"; grep -a "PReLU slopes" gpurun_out/r5_ampfix.log | cut -c1-200
done
