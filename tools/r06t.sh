#!/bin/bash
# round-6 session 3: resident-read searches for the sharded step (no input
# event: the next run's first searches start once their set is free) --
# the back-to-back and thread-rank driver tests, the world-1 multi-GPU step
# (cross-run look-ahead on / off) vs the single-GPU step, a kernel trace of
# the sharded step; then the C5 prepare variants (tools/r06s.sh)
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r06t
mkdir -p "$O"
cd "$R"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -v \
    -k "back_to_back or real_driver_threads" --timeout 400 --timeout-method thread \
    > "$O/tests.log" 2>&1
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-feed --no-c5 --no-sub"
timeout -k 10 300 python3 "$R/bench.py" $ARGS > "$O/single.json" 2> "$O/single.log"
SMASH_BENCH_SHARDED=1 timeout -k 10 300 python3 -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29551 "$R/bench.py" \
    $ARGS > "$O/sharded_w1.json" 2> "$O/sharded_w1.log"
SMASH_BENCH_CROSS=0 SMASH_BENCH_SHARDED=1 timeout -k 10 300 python3 -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29552 "$R/bench.py" \
    $ARGS > "$O/sharded_w1_nocross.json" 2> "$O/sharded_w1_nocross.log"
SMASH_BENCH_SHARDED=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29553 \
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-feed --no-c5 --no-sub \
    > "$O/prof.log" 2>&1
bash "$R/tools/r06s.sh"
