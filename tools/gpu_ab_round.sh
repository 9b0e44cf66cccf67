#!/bin/bash
# tools/gpu_ab_round.sh TAG "SETTING..." [TESTS] -- one GPU call: the -m gpu
# tests (pytest -k expression; "all" = the whole suite; "" = none), an
# in-process A/B of the full C3 step under the given settings
# (tools/sweep.py, 25 M pairs in 6.25 M-pair batches), then the default bench
# line.  Each GPU step has its own time limit; the chain stops at the first
# failure.
set -euo pipefail
TAG=${1:?tag}
SETTINGS=${2:-base}
TESTS=${3:-}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
if [ "$TESTS" = "all" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
      > "$O/tests.log" 2>&1
elif [ -n "$TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
      -k "$TESTS" > "$O/tests.log" 2>&1
fi
cd /tmp
timeout -k 10 500 python3 "$R/tools/sweep.py" --pairs 25000000 --batch 6250000 --steps 5 \
    $SETTINGS > "$O/sweep.log" 2>&1
timeout -k 10 600 python3 "$R/bench.py" > "$O/bench.json" 2> "$O/bench.log"
