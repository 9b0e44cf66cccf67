#!/bin/bash
# tools/r06g.sh -- index-build changes (PLCP + gather LCP, word loads in
# k_kcode / k_pack_sa): the index parity tests, then the hg19 build timed in
# the bench (default) and with the rank-order Kasai (SMASH_LCP_KASAI=1)
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r06g
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v \
    --timeout 500 --timeout-method thread -k "parity or c1 or device_index or idx8 or c5" > "$O/tests.log" 2>&1
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-feed --no-c5 --no-sub"
SMASH_VERBOSE=1 timeout -k 10 300 python3 "$R/bench.py" $ARGS > "$O/new.json" 2> "$O/new.log"
SMASH_VERBOSE=1 SMASH_LCP_KASAI=1 timeout -k 10 300 python3 "$R/bench.py" $ARGS > "$O/kasai.json" 2> "$O/kasai.log"
