#!/bin/bash
# Rehearse bench.py's N=2 path on a one-GPU box: two ranks on device 0, gloo instead of RCCL (RCCL refuses
# two ranks on one device). Exercises rendezvous, graph capture per rank, the flat-gradient reducer,
# barrier + max-over-ranks timing and the rank-0 JSON line; the timing itself is meaningless (shared GPU).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HYRES_BENCH_ONE_GPU=1 HYRES_BENCH_BACKEND=gloo
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 4 --warmup 2 > gpurun_out/dist2_graph.log 2>&1 || exit $?
HYRES_DIST_OVERLAP=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 4 --warmup 2 > gpurun_out/dist2_overlap.log 2>&1
