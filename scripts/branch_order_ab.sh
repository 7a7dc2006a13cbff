# A/B of ops.BranchStreams.side_first on one box: the bit-identity test, then the graphed C2 fp32 step
# (scripts/step_profile.py, 20 steps) alternating default / side-first, three times -> gpurun_out/branch_order_ab.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out || exit 1
out=gpurun_out/branch_order_ab.txt
timeout -k 10 200 python -u -m pytest tests/test_parity_gpu.py -q -m gpu --timeout 150 --timeout-method thread \
  -k test_branch_side_first_order_same_gradients > $out 2>&1 || exit $?
for rep in 1 2 3; do
  for v in "" "--side-first"; do
    echo "rep$rep ${v:-default}: $(timeout -k 10 200 python3 scripts/step_profile.py --steps 20 $v 2>&1 | tail -1)" >> $out || exit 1
  done
done
cat $out
