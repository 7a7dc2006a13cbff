# AMP fixture test once per AMP storage switch (env read at import) -> gpurun_out/diag_amp2.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out || exit 1
: > gpurun_out/diag_amp2.log
for env in "HYRES_X=1" "HYRES_AMP_F16_GRAD=0" "HYRES_AMP_F16_ACT=0" "HYRES_AMP_WGRAD_F16=0"; do
  echo "##### $env" >> gpurun_out/diag_amp2.log
  env $env timeout -k 10 200 python -u scripts/diag_amp.py --once >> gpurun_out/diag_amp2.log 2>&1 || exit $?
done
echo "exit 0" >> gpurun_out/diag_amp2.log
