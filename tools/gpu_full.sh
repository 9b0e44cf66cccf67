#!/bin/bash
# tools/gpu_full.sh TAG [BENCH_ARGS...] -- one GPU call: the whole `-m gpu`
# suite, smoke(), then bench.py; each step under its own time limit, the
# chain stops at the first failure.
set -uo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$1
shift
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 1100 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
    "$R/tests" > "$O/tests.log" 2>&1
rc=$?
tail -3 "$O/tests.log"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" \
    > "$O/smoke.log" 2>&1 || exit $?
tail -1 "$O/smoke.log"
timeout -k 10 900 python3 -u "$R/bench.py" "$@" > "$O/bench.json" 2> "$O/bench.log"
rc=$?
tail -4 "$O/bench.log"
exit $rc
