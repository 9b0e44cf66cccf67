#!/bin/bash
# tools/r04_tsweep.sh TAG "TESTS" SETTING... -- the named -m gpu tests, then
# tools/r04_sweep.sh TAG SETTING...
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
TAG=$1; T=$2; shift 2
mkdir -p "$R/gpurun_out/$TAG"
cd "$R"
timeout -k 10 ${TLIM:-420} python3 -u -m pytest tests -m gpu -x -v --timeout 300 \
    --timeout-method thread -k "$T" > "$R/gpurun_out/$TAG/tests.log" 2>&1
"$R/tools/r04_sweep.sh" "$TAG" "$@"
