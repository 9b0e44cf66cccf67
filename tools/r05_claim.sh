#!/bin/bash
# tools/r05_claim.sh TAG -- the de-dup claim flag (kSlotIns: a pair that filled
# an empty slot and was never contested wins without k_dedup_decide re-reading
# the slot): the pipeline parity tests (short key hashes included), then the
# C3 step with SMASH_CLAIM_FLAG=0 and the default, alternating, on one box.
set -euo pipefail
TAG=${1:?tag}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -v \
    --timeout 600 --timeout-method thread -k "not production and not mem_hg19 and not c5" \
    > "$O/tests.log" 2>&1
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-feed --no-c5"
for k in 1 2; do
  SMASH_CLAIM_FLAG=0 timeout -k 10 240 python3 "$R/bench.py" $ARGS > "$O/off$k.json" 2> "$O/off$k.log"
  timeout -k 10 240 python3 "$R/bench.py" $ARGS > "$O/on$k.json" 2> "$O/on$k.log"
done
