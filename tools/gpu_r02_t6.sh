#!/bin/bash
# file-fed pipeline: its GPU tests, then a short bench with the feed measurement
set -uo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r02_t6
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
    $R/tests/test_gpu_feed.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python3 -u $R/bench.py --steps 1 --pairs 4000000 --no-c5 > $O/bench.json 2> $O/bench.log
rc=$?
grep -E "file-fed|cpu baseline|timed" $O/bench.log
exit $rc
