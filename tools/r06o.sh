#!/bin/bash
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/gpurun_out/r06o"
cd "$R"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_phases.py tests/test_gpu_feed.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06o/parity.log 2>&1
ROUNDS=3 TESTS='production or idx8' bash tools/r06_ab.sh r06o 'libsmashgpu_dec.so -'
bash tools/r06_trace.sh r06o/trace
