#!/bin/bash
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r06h
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q \
    --timeout 500 --timeout-method thread -k "parity or c1 or device_index or idx8 or hg19_counts" > "$O/tests.log" 2>&1
timeout -k 10 400 python3 -u tools/index_time.py SMASH_LCP_KASAI=1 base SMASH_LCP_KASAI=1 base > "$O/index_time.log" 2>&1
