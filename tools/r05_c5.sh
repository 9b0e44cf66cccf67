#!/bin/bash
# tools/r05_c5.sh TAG -- the round-5 checks of the C5 rebuild and the 12.5 M
# batch: the mappability tests, the hg19 C3/C5 tests, then the C5 bench line
# under rocprofv3 --kernel-trace --stats.
set -euo pipefail
TAG=${1:?tag}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_mappability.py -m gpu -v --timeout 200 \
    --timeout-method thread > "$O/tests_map.log" 2>&1
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -v --timeout 900 \
    --timeout-method thread -k "c5 or c3_full or c3_production" > "$O/tests_cfg.log" 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o c5 -- \
    python3 "$R/bench.py" --config c5 --steps 5 > "$O/bench_c5.json" 2> "$O/bench_c5.log"
exit 0
