#!/bin/bash
# tools/gpu_ab.sh OUT SETTING... -- one GPU call: the device parity tests of
# the search + pipeline, then tools/sweep.py over the settings (one process:
# genome, index and reads built once), each step under its own time limit.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$1
shift
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
    "$R/tests/test_gpu_parity.py" "$R/tests/test_gpu_modes.py" > "$O/tests.log" 2>&1
timeout -k 10 600 python3 -u "$R/tools/sweep.py" --steps 5 "$@" > "$O/sweep.log" 2>&1
grep "sweep\]" "$O/sweep.log"
