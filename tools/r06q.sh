#!/bin/bash
# round-6 session 3: the U rebuild (uniq_build.hip: wide loads, next tile in
# flight, 2^25 / 2^17 geometry) -- its parity tests, then the C5 prepare A/B
# (round-5 code as libsmashgpu_u0.so vs HEAD at S1 = 25 and 24), then the
# world-1 multi-GPU step vs the single-GPU step with a kernel trace of the
# sharded step
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r06q
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_mappability.py -m gpu -v -k "prepare" \
    --timeout 300 --timeout-method thread > "$O/tests_mid.log" 2>&1
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -v -k "c5_prepare" \
    --timeout 400 --timeout-method thread > "$O/tests_hg19.log" 2>&1
ROUNDS=2 timeout -k 10 300 python3 -u tools/c5_ab.py s25: s24:SMASH_UPART_S1=24 \
    s25e512:SMASH_UPART_E2MB=512 > "$O/c5ab.log" 2>&1
ROUNDS=1 SMASH_LIB=$R/smash-paper_amd/lib/libsmashgpu_u0.so timeout -k 10 200 python3 -u \
    tools/c5_ab.py u0: > "$O/c5ab_u0.log" 2>&1
STEPS=5 bash tools/r04_sharded.sh r06q/shard
