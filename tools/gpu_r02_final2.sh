#!/bin/bash
# round-2 closing measurement: the whole -m gpu suite, smoke(), the default
# bench line, then a kernel trace + stats of a 3-step bench
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02f2}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu $R/tests > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 600 python3 -u $R/bench.py > $O/bench.json 2> $O/bench.log || exit 1
grep -E "timed" $O/bench.log | cut -c1-150
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv \
    -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-feed --no-c5 > $O/prof.json 2> $O/prof.log || exit 1
grep timed $O/prof.log | cut -c1-150
