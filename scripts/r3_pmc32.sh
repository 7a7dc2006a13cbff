cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MICRO="scripts/conv_micro.py --B 16 --H 128 --Ci 64 --Co 64 --K 3 --iters 20"
scripts/gpu_run.sh \
 "p32a:120:rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/p32a -o run -- python3 $MICRO" \
 "p32b:120:HYRES_CONV_WRES32=0 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/p32b -o run -- python3 $MICRO"
