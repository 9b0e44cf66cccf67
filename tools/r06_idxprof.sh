#!/bin/bash
# tools/r06_idxprof.sh TAG -- rocprofv3 kernel trace + stats of one hg19 index build
set -euo pipefail
TAG=${1:?tag}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv \
    -- python3 "$R/tools/index_time.py" base > "$O/idx.log" 2>&1
