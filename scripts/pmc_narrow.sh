# round 5: why the Co <= 4 convs run at ~1.4 TB/s — HBM bytes (FETCH_SIZE / WRITE_SIZE passes) and SQ counters of
# conv_narrow_kernel<3, 1> (MultiScaleRefine 3x3 64 -> 3 at bs16 256^2) in isolation
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
M="python3 scripts/conv_micro.py --bf6 --H 256 --Ci 64 --Co 3 --K 3 --iters 10"
out=gpurun_out/r5u_narrow_pmc.txt
: > $out
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/r5u_nf -o run -- $M > /dev/null 2>&1 || exit 1
python3 scripts/pmc_sq.py gpurun_out/r5u_nf --kernel conv_narrow >> $out || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/r5u_nw -o run -- $M > /dev/null 2>&1 || exit 1
python3 scripts/pmc_sq.py gpurun_out/r5u_nw --kernel conv_narrow >> $out || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/r5u_nsq -o run -- $M > /dev/null 2>&1 || exit 1
python3 scripts/pmc_sq.py gpurun_out/r5u_nsq --kernel conv_narrow >> $out || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/r5u_ntc -o run -- $M > /dev/null 2>&1 || exit 1
python3 scripts/pmc_sq.py gpurun_out/r5u_ntc --kernel conv_narrow >> $out || exit 1
cat $out
