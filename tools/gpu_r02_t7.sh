#!/bin/bash
# two-stream search sets: phase / feed / parity tests, then the C3 bench
set -uo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r02_t7
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread \
    $R/tests/test_gpu_phases.py $R/tests/test_gpu_feed.py $R/tests/test_gpu_parity.py \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python3 -u $R/bench.py --steps 3 --no-cpu-baseline --no-c5 > $O/bench.json 2> $O/bench.log
rc=$?
grep -E "timed|file-fed" $O/bench.log
exit $rc
