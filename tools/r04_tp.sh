#!/bin/bash
# tools/r04_tp.sh TAG "TESTS" "ENV_B" -- the named -m gpu tests, then
# tools/r04_prof_ab.sh TAG "ENV_B" (kernel trace of the default, A/B runs)
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$1
mkdir -p "$O"
cd "$R"
timeout -k 10 ${TLIM:-420} python3 -u -m pytest tests -m gpu -x -v --timeout 300 \
    --timeout-method thread -k "$2" > "$O/tests.log" 2>&1
"$R/tools/r04_prof_ab.sh" "$1" "$3"
