#!/bin/bash
# tools/r05_mem.sh TAG -- the MEM mode on one box: its parity tests (reference
# triples, the mid genome with deferral thresholds and caps, hg19 vs the
# oracle), then the c3mem bench line.
set -euo pipefail
TAG=${1:?tag}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_modes.py tests/test_gpu_configs.py -m gpu -v \
    --timeout 600 --timeout-method thread -k "modes or mem" > "$O/tests.log" 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 python3 "$R/bench.py" --config c3mem --steps 3 > "$O/c3mem.json" 2> "$O/c3mem.log"
