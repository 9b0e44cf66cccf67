#!/bin/bash
# round-6 session 3: k_emit_bin_lds with a pair's bin lookups batched --
# pipeline parity + production-batch / idx8 / back-to-back tests, the C3
# step A/B against the previous k_emit_bin_lds (libsmashgpu_e0.so), then the
# world-1 multi-GPU step (cross-run look-ahead on / off) vs the single-GPU
# step, with a kernel trace of the sharded step
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r06r
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_phases.py \
    tests/test_gpu_feed.py -m gpu -x -q --timeout 200 --timeout-method thread > "$O/parity.log" 2>&1
ROUNDS=2 TESTS='production or idx8 or back_to_back' bash tools/r06_ab.sh r06r 'libsmashgpu_e0.so -'
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-feed --no-c5 --no-sub"
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
T=$(ls "$O"/prof/*/run_kernel_trace.csv | head -1)
python3 "$R/tools/step_breakdown.py" "$T" 2 2 > "$O/step_breakdown.txt"
