#!/bin/bash
# round-6 session 3: the de-dup claim/decide rewrites (3e8a4ce, 9fecedc) --
# pipeline parity, production-batch + idx8 tests, then base (2eb69fe) vs HEAD
# C3 step A/B, 3 rounds, and a kernel trace + step breakdown of HEAD
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/gpurun_out/r06p"
cd "$R"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_phases.py tests/test_gpu_feed.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06p/parity.log 2>&1
ROUNDS=3 TESTS='production or idx8' bash tools/r06_ab.sh r06p 'libsmashgpu_base.so -'
bash tools/r06_trace.sh r06p/trace
