cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MICRO="scripts/conv_micro.py --B 16 --H 128 --Ci 64 --Co 64 --K 3 --iters 20"
scripts/gpu_run.sh \
 "bench:200:python bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
 "micro:200:python scripts/conv_micro.py && python scripts/conv_micro.py --Ci 128 --Co 128 --K 1 && python scripts/conv_micro.py --Ci 128 --Co 64 --K 1 && python scripts/conv_micro.py --Ci 128 --Co 128 --K 5 --stride 2 && python scripts/conv_micro.py --H 256 --Ci 64 --Co 64" \
 "list:120:rocprofv3 -L > gpurun_out/counters_list.txt 2>&1" \
 "pmcA:200:rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmcA -o run -- python3 $MICRO" \
 "pmcB:200:rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/pmcB -o run -- python3 $MICRO" \
 "pmcC:200:rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d gpurun_out/pmcC -o run -- python3 $MICRO"
