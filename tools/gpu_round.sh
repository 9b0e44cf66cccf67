#!/bin/bash
# tools/gpu_round.sh TAG [TESTS] [CHECK_AB] -- one GPU call of a round: the
# named -m gpu tests (pytest -k expression, "" = none, "all" = the whole
# suite), then tools/measure_round.sh TAG (bench line, kernel trace + stats,
# FETCH_SIZE pass, randbench calibration) and, with CHECK_AB = 1, the
# SMASH_SM_CHECK=0 A/B of the search (two runs each, alternating).  Every GPU
# step has its own time limit; the chain stops at the first failure.
set -euo pipefail
TAG=${1:?tag}
TESTS=${2:-}
CHECK_AB=${3:-0}
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
"$R/tools/measure_round.sh" "$TAG"
[ "$CHECK_AB" = "1" ] || exit 0
cd /tmp
for i in 1 2; do
  for ck in 1 0; do
    SMASH_SM_CHECK=$ck timeout -k 10 300 python3 "$R/bench.py" --steps 10 --warmup 2 \
        --no-cpu-baseline --no-feed --no-c5 > "$O/check$ck.$i.json" 2> "$O/check$ck.$i.log"
  done
done
