#!/bin/bash
# tools/r04_ab.sh TAG "ENV_A" "ENV_B" [TESTS] -- the named -m gpu tests
# (pytest -k; empty: none), then the C3 bench (no CPU baseline, feed or C5)
# alternating settings A, B, A, B on one box, each run with its own limit.
set -euo pipefail
TAG=${1:?tag}
A=${2:-}
B=${3:-}
TESTS=${4:-}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      -k "$TESTS" > "$O/tests.log" 2>&1
fi
cd /tmp && export TMPDIR=/tmp
ARGS="--steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-feed --no-c5"
for i in 1 2; do
  env $A timeout -k 10 400 python3 "$R/bench.py" $ARGS > "$O/a$i.json" 2> "$O/a$i.log"
  env $B timeout -k 10 400 python3 "$R/bench.py" $ARGS > "$O/b$i.json" 2> "$O/b$i.log"
done
exit 0
