#!/bin/bash
# tools/r05_upart.sh TAG -- U rebuild partition passes with 1024-thread tiles
# (16 384 entries) vs 512 (SMASH_UPART_THREADS=512): the C5 and index parity
# tests, then the C5 line alternating, on one box.
# (the 1024-thread tiles were reverted after this run: the record of profiles/r05/upart1/)
set -euo pipefail
TAG=${1:?tag}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_configs.py tests/test_gpu_mappability.py -m gpu -v \
    --timeout 300 --timeout-method thread -k "c5 or mappability" > "$O/tests.log" 2>&1
cd /tmp && export TMPDIR=/tmp
ARGS="--config c5 --steps 5 --warmup 1 --no-cpu-baseline"
for k in 1 2; do
  SMASH_UPART_THREADS=512 timeout -k 10 200 python3 "$R/bench.py" $ARGS > "$O/t512_$k.json" 2> "$O/t512_$k.log"
  timeout -k 10 200 python3 "$R/bench.py" $ARGS > "$O/t1024_$k.json" 2> "$O/t1024_$k.log"
done
