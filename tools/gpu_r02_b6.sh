#!/bin/bash
# the 6.25 M-pair default: the C3 full-run property test at that split, then
# the default bench line
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02b6}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 500 --timeout-method thread $R/tests/test_gpu_configs.py -k c3_full_run > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python3 -u $R/bench.py > $O/bench.json 2> $O/bench.log || exit 1
grep -E "timed" $O/bench.log | cut -c1-120
