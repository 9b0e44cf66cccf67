#!/bin/bash
# round-6 session 3, final build: the world-1 multi-GPU step (dist.ShardedCounter
# over RCCL + gloo, cross-run look-ahead) and the single-GPU step, one box
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r06h2
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-feed --no-c5 --no-sub"
timeout -k 10 300 python3 "$R/bench.py" $ARGS > "$O/single.json" 2> "$O/single.log"
SMASH_BENCH_SHARDED=1 timeout -k 10 300 python3 -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29581 "$R/bench.py" \
    $ARGS > "$O/sharded_w1.json" 2> "$O/sharded_w1.log"
timeout -k 10 300 python3 "$R/bench.py" $ARGS > "$O/single2.json" 2> "$O/single2.log"
