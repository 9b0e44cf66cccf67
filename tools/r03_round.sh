#!/bin/bash
# tools/r03_round.sh TAG [TESTS] -- one GPU call: the named -m gpu tests
# (pytest -k; "all" = the suite), the schedule sweep (tools/r03_sched.sh,
# SETTINGS), then the measured round (tools/measure_round.sh: bench line,
# kernel trace + stats, FETCH_SIZE).  Every step has its own time limit; the
# chain stops at the first failure.
set -euo pipefail
TAG=${1:?tag}
TESTS=${2:-}
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
[ "${SWEEP:-1}" = "1" ] && "$R/tools/r03_sched.sh" "$TAG"
[ "${MEASURE:-1}" = "1" ] && "$R/tools/measure_round.sh" "$TAG"
exit 0
