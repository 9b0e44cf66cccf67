#!/bin/bash
# tools/r05_geo.sh TAG [TESTS] -- k_mam_sm with the production geometry as constants
# (GEO 1): the production-batch and packed-index parity tests (they run the
# GEO instantiation), then the C3 step with SMASH_SM_GEO=0 / 1 alternating on
# one box.
set -euo pipefail
TAG=${1:?tag}
SEL=${2:-production or idx8}   # the parity tests to run first
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -v \
    --timeout 400 --timeout-method thread -k "$SEL" \
    > "$O/tests.log" 2>&1
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-feed --no-c5"
for k in 1 2; do
  SMASH_SM_GEO=0 timeout -k 10 240 python3 "$R/bench.py" $ARGS > "$O/off$k.json" 2> "$O/off$k.log"
  SMASH_SM_GEO=1 timeout -k 10 240 python3 "$R/bench.py" $ARGS > "$O/on$k.json" 2> "$O/on$k.log"
done
