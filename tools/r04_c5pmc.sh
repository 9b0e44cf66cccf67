#!/bin/bash
# tools/r04_c5pmc.sh TAG -- the C5 scan's issue counters: one SQ pass over
# bench.py --config c5 (k_mapscan only), then its kernel trace.
set -euo pipefail
TAG=${1:?tag}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    --kernel-include-regex k_mapscan -d "$O/sq" -o pmc --output-format csv \
    -- python3 "$R/bench.py" --config c5 --steps 2 --warmup 1 --no-cpu-baseline > "$O/sq.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --config c5 --steps 3 --warmup 1 --no-cpu-baseline > "$O/prof.log" 2>&1
exit 0
