#!/bin/bash
# round-6 session 3: the U rebuild (uniq_build.hip: wide loads, next tile in
# flight) -- its parity tests, then the C5 prepare A/B (round-5 code as
# libsmashgpu_u0.so vs HEAD, pass-1 tiles of 8 k and 16 k ranks); the
# back-to-back-run look-ahead tests; the world-1 multi-GPU step (cross-run
# look-ahead on / off) vs the single-GPU step, with a kernel trace of the
# sharded step
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r06q
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_mappability.py -m gpu -v -k "prepare" \
    --timeout 300 --timeout-method thread > "$O/tests_mid.log" 2>&1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -v \
    -k "c5_prepare or back_to_back or real_driver_threads" \
    --timeout 400 --timeout-method thread > "$O/tests_hg19.log" 2>&1
ROUNDS=2 timeout -k 10 300 python3 -u tools/c5_ab.py nt512: nt1024:SMASH_UPART_NT=1024 \
    > "$O/c5ab.log" 2>&1
ROUNDS=1 SMASH_LIB=$R/smash-paper_amd/lib/libsmashgpu_u0.so timeout -k 10 200 python3 -u \
    tools/c5_ab.py u0: > "$O/c5ab_u0.log" 2>&1
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
T=$(ls "$O"/prof/*/run_kernel_trace.csv | head -1)
python3 "$R/tools/step_breakdown.py" "$T" 2 2 > "$O/step_breakdown.txt"
