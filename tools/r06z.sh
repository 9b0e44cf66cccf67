#!/bin/bash
# round-6 session 3: U rebuild chunks alternating over two streams -- the
# prepare parity tests (mid genome, hg19), then the C5 A/B (SMASH_UPART_2S)
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r06z
mkdir -p "$O"
cd "$R"
#timeout -k 10 300 python3 -u -m pytest tests/test_gpu_mappability.py -m gpu -v -k "prepare" \
#    --timeout 200 --timeout-method thread > "$O/tests_mid.log" 2>&1
#timeout -k 10 400 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -v -k "c5_prepare" \
#    --timeout 300 --timeout-method thread > "$O/tests_hg19.log" 2>&1
ROUNDS=5 timeout -k 10 300 python3 -u tools/c5_ab.py two: one:SMASH_UPART_2S=0 > "$O/c5ab.log" 2>&1
