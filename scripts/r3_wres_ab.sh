cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in 0 1 2; do for args in "" "--res --relu" "--H 256"; do echo "V=$v $args"; HYRES_WRES_VARIANT=$v timeout 60 python scripts/conv_micro.py --f16 $args 2>&1 | grep conv || exit 1; done; done
MICRO="scripts/conv_micro.py --B 16 --H 128 --Ci 64 --Co 64 --K 3 --iters 20 --f16"
scripts/gpu_run.sh \
 "pmcA:120:rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d gpurun_out/wpmcA -o run -- python3 $MICRO" \
 "pmcC:120:rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/wpmcC -o run -- python3 $MICRO" \
 "pmcD:120:rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/wpmcD -o run -- python3 $MICRO" \
 "pmcB:120:rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/wpmcB -o run -- python3 $MICRO"
