#!/bin/bash
# Rehearse bench.py's N>1 path on a one-GPU box. (1) two ranks on device 0 over gloo (RCCL refuses two
# ranks on one device): rendezvous, per-rank graph capture, the default graph+overlap (capture cut at the "hyper"
# marker, the finished segments' all-reduce between the two replays) and graph+allreduce (one replay, then the
# whole flat gradient), barrier + max-over-ranks timing, the rank-0 line — timings of a shared GPU, for the ratio
# only; (2) ONE rank with a real RCCL group (HYRES_BENCH_FORCE_DIST=1), graph+overlap and graph+allreduce alternating
# twice on one box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ARGS="--gpus 2 --steps 4 --warmup 2 --no-eval --no-amp --no-host-jpeg --no-cpu-baseline"
HYRES_DIST_MODE=graph+overlap HYRES_BENCH_ONE_GPU=1 HYRES_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py $ARGS \
  > gpurun_out/dist2_graph_overlap.log 2>&1 || exit $?
HYRES_DIST_MODE=graph+allreduce HYRES_BENCH_ONE_GPU=1 HYRES_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py $ARGS \
  > gpurun_out/dist2_graph_allreduce.log 2>&1 || exit $?
port=29520
names=""
for rep in 1 2; do
  for mode in graph+overlap graph+allreduce; do
    f=dist1_rccl_${mode/+/_}_$rep
    HYRES_DIST_MODE=$mode HYRES_BENCH_FORCE_DIST=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 \
      --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port bench.py --steps 20 --warmup 3 --no-eval \
      --no-amp --no-host-jpeg --no-cpu-baseline > gpurun_out/$f.log 2>&1 || exit $?
    port=$((port + 1))
    names="$names $f"
  done
done
for f in dist2_graph_overlap dist2_graph_allreduce $names; do
  echo "$f: $(grep '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['dist_mode'], d['ms_per_step'], 'ms/step')")"
done | tee gpurun_out/dist_rehearsal.txt
