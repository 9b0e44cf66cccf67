#!/bin/bash
# tools/r03_sharded_diag.sh TAG -- where the multi-GPU step's time goes at
# world 1: a kernel trace of the sharded bench and a run with every phase of
# ShardedCounter.step closed by a device synchronisation (SMASH_DIST_TIMING=1).
set -euo pipefail
TAG=${1:?tag}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
SMASH_DIST_TIMING=1 SMASH_BENCH_SHARDED=1 timeout -k 10 600 python3 -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 "$R/bench.py" \
    --steps 2 --warmup 1 --no-cpu-baseline --no-feed --no-c5 > "$O/timing.json" 2> "$O/timing.log"
SMASH_BENCH_SHARDED=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29542 \
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-feed --no-c5 \
    > "$O/prof.log" 2>&1
