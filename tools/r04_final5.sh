#!/bin/bash
# tools/r04_final5.sh TAG -- tools/r04_measure.sh TAG (bench line, kernel
# trace, FETCH_SIZE pass, calibration, the multi-GPU step at world 1 and the
# single-GPU step), then a rocprofv3 kernel trace of the C5 scan alone.
set -euo pipefail
TAG=${1:?tag}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
"$R/tools/r04_measure.sh" "$TAG"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_c5" -o run --output-format csv \
    -- python3 "$R/bench.py" --config c5 --steps 5 --warmup 1 --no-cpu-baseline \
    > "$O/prof_c5.json" 2> "$O/prof_c5.log"
exit 0
