#!/bin/bash
# tools/r06_trace.sh TAG -- rocprofv3 kernel trace + stats of a 3-step C3 bench
# (no side lines) and its step breakdown (tools/step_breakdown.py)
set -euo pipefail
TAG=${1:?tag}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-feed --no-c5 --no-sub \
    > "$O/prof.json" 2> "$O/prof.log"
T=$(find "$O/prof" -name "*kernel_trace.csv" | head -1)
python3 "$R/tools/step_breakdown.py" "$T" 2 2 > "$O/step_breakdown.txt"
