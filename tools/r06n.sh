#!/bin/bash
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/gpurun_out/r06n"
cd "$R"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_phases.py tests/test_gpu_feed.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06n/parity.log 2>&1
TESTS='production or idx8 or hg19_counts' bash tools/r06_ab.sh r06n 'libsmashgpu_base.so -'
timeout -k 10 400 python3 tools/c2_ab.py 500000 250000 125000 > gpurun_out/r06n/c2ab.log 2>&1
