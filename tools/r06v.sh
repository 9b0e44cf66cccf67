#!/bin/bash
# round-6 session 3: kernel traces (queue ids) of the world-1 sharded step
# with the search streams at high priority, and of the single-GPU step with
# them at high priority
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r06v
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
SMASH_SEARCH_PRIO=high SMASH_BENCH_SHARDED=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 \
    MASTER_PORT=29571 timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/prof_sh" -o run \
    --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-feed \
    --no-c5 --no-sub > "$O/prof_sh.json" 2> "$O/prof_sh.log"
SMASH_SEARCH_PRIO=high timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/prof_1" -o run \
    --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-feed \
    --no-c5 --no-sub > "$O/prof_1.json" 2> "$O/prof_1.log"
