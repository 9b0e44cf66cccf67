#!/bin/bash
# the parity + phase tests in one process (the order in which the look-ahead
# / forced-collision phase case failed) with the two-kernel positions path
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02iso}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
SMASH_FUSED_BIN=0 timeout -k 10 500 python3 -u -m pytest -q --timeout 300 --timeout-method thread $R/tests/test_gpu_parity.py $R/tests/test_gpu_phases.py > $O/twokernel.log 2>&1
echo "two-kernel: $(tail -1 $O/twokernel.log)"
grep -h FAILED $O/twokernel.log || true
