cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MICRO="scripts/conv_micro.py --B 16 --H 128 --Ci 64 --Co 64 --K 3 --iters 20 --f16"
scripts/gpu_run.sh \
 "ddp:400:python -u -m pytest tests/test_ddp_gpu.py tests/test_optim.py -v -s --timeout 300 --timeout-method thread -m gpu" \
 "amp:300:python -u -m pytest tests/test_parity_gpu.py -v -s --timeout 200 --timeout-method thread -m gpu -k 'amp_matches_reference or rccl'" \
 "f16micro:200:python scripts/conv_micro.py --f16 && python scripts/conv_micro.py --f16 --H 256 && python scripts/conv_micro.py && python scripts/conv_micro.py --f16 --Ci 64 --Co 64 --K 1" \
 "pmcA:120:rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d gpurun_out/f16pmcA -o run -- python3 $MICRO" \
 "pmcB:120:rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum --kernel-trace --output-format csv -d gpurun_out/f16pmcB -o run -- python3 $MICRO" \
 "pmcC:120:rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/f16pmcC -o run -- python3 $MICRO"
