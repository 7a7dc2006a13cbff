#!/bin/bash
# SQ counters of the dominant conv in the live step vs the branch-serialised step (one pass each)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_live -o run -- python3 scripts/step_profile.py --steps 4 > gpurun_out/pmc_live.log 2>&1 || exit $?
HYRES_BRANCH_MAX_PIXELS=0 timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_serial -o run -- python3 scripts/step_profile.py --steps 4 > gpurun_out/pmc_serial.log 2>&1 || exit $?
python3 scripts/pmc_contention.py gpurun_out/pmc_live gpurun_out/pmc_serial --kernel "conv_fwd_kernel<2, 1, 2, 2, 0, false, false>" --out gpurun_out/pmc_contention.json
