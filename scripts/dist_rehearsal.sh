#!/bin/bash
# Rehearse bench.py's N>1 path on a one-GPU box. (1) two ranks on device 0 over gloo (RCCL refuses two
# ranks on one device): rendezvous, per-rank graph capture, the default after-replay all-reduce
# (graph+allreduce), barrier + max-over-ranks timing, the rank-0 line; then the eager step whose all-reduce overlaps
# backward segment by segment (eager-overlap) — timings of a shared GPU, for the ratio only; (2) ONE rank with a real
# RCCL group (HYRES_BENCH_FORCE_DIST=1).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ARGS="--gpus 2 --steps 4 --warmup 2 --no-eval --no-amp --no-host-jpeg --no-cpu-baseline"
HYRES_BENCH_ONE_GPU=1 HYRES_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py $ARGS \
  > gpurun_out/dist2_graph_allreduce.log 2>&1 || exit $?
HYRES_BENCH_ONE_GPU=1 HYRES_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py $ARGS --no-graph \
  > gpurun_out/dist2_eager_overlap.log 2>&1 || exit $?
HYRES_BENCH_FORCE_DIST=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29519 bench.py --steps 10 --warmup 3 --no-eval --no-amp \
  --no-host-jpeg --no-cpu-baseline > gpurun_out/dist1_rccl.log 2>&1
for f in dist2_graph_allreduce dist2_eager_overlap dist1_rccl; do
  echo "$f: $(grep '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['dist_mode'], d['ms_per_step'], 'ms/step')")"
done | tee gpurun_out/dist_rehearsal.txt
