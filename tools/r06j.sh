#!/bin/bash
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r06j
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q \
    --timeout 500 --timeout-method thread -k "parity or c1 or device_index" > "$O/tests.log" 2>&1
bash "$R/tools/r06_idxprof.sh" r06j
