#!/bin/bash
# phase / parity / dedup tests, then per-kernel times of one sweep run
set -uo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r02_t3
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
    $R/tests/test_gpu_phases.py $R/tests/test_gpu_parity.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash $R/tools/gpu_prof_sweep.sh r02_t3/prof
