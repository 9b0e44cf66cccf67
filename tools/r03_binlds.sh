#!/bin/bash
# tools/r03_binlds.sh TAG -- kernel trace of the C3 bench with the LDS bin
# counts (SMASH_BIN_LDS=1), for k_emit_bin_lds's duration beside k_emit_bin's
set -euo pipefail
TAG=${1:?tag}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
SMASH_BIN_LDS=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof_binlds" -o run \
    --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-feed \
    --no-c5 > "$O/prof_binlds.log" 2>&1
