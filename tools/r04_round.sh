#!/bin/bash
# tools/r04_round.sh TAG [TESTS] -- one box: the named -m gpu tests (pytest -k),
# the default bench line (C3 with the feed, C5 and the CPU baseline), then
# the C3 step with dense input (SMASH_BENCH_ROWS=0) for the native-row A/B.
# Each GPU step has its own limit; the chain stops at the first failure.
set -euo pipefail
TAG=${1:?tag}
TESTS=${2:-}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TLIM:-420} python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
      -k "$TESTS" > "$O/tests.log" 2>&1
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 480 python3 "$R/bench.py" > "$O/bench.json" 2> "$O/bench.log"
if [ "${DENSE:-1}" = "1" ]; then
  SMASH_BENCH_ROWS=0 timeout -k 10 300 python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline \
      --no-feed --no-c5 > "$O/dense.json" 2> "$O/dense.log"
fi
exit 0
