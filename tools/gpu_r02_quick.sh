#!/bin/bash
# the fused positions + varbin and 16-byte k_prep build on the GPU: the parity,
# phase-API and file-fed tests, smoke(), then the default bench line
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02q}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread $R/tests/test_gpu_parity.py $R/tests/test_gpu_phases.py $R/tests/test_gpu_feed.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -u -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 600 python3 -u $R/bench.py > $O/bench.json 2> $O/bench.log || exit 1
grep -E "timed" $O/bench.log | cut -c1-150
