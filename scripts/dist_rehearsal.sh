#!/bin/bash
# Rehearse bench.py's N>1 path on a one-GPU box. (1) two ranks on device 0 over gloo (RCCL refuses two
# ranks on one device): rendezvous, per-rank graph capture with the marker events, the graph-triggered
# segment all-reduce (default dist_mode graph+overlap) and the after-replay mode, barrier + max-over-ranks
# timing, the rank-0 line — timings meaningless (shared GPU); (2) ONE rank with a real RCCL group
# (HYRES_BENCH_FORCE_DIST=1): the graph+overlap path through RCCL proper.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
HYRES_BENCH_ONE_GPU=1 HYRES_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 4 --warmup 2 \
  > gpurun_out/dist2_graph_overlap.log 2>&1 || exit $?
HYRES_BENCH_ONE_GPU=1 HYRES_BENCH_BACKEND=gloo HYRES_DIST_MODE=graph+allreduce timeout -k 10 300 python3 -m \
  torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py \
  --gpus 2 --steps 4 --warmup 2 > gpurun_out/dist2_graph_allreduce.log 2>&1 || exit $?
HYRES_BENCH_FORCE_DIST=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29519 bench.py --steps 10 --warmup 3 --no-eval --no-amp \
  --no-host-jpeg --no-cpu-baseline > gpurun_out/dist1_rccl_overlap.log 2>&1
