#!/bin/bash
# parity + phase tests in one process at the current build (fused positions
# path, word-access k_prep)
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02iso2}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest -q --timeout 300 --timeout-method thread $R/tests/test_gpu_parity.py $R/tests/test_gpu_phases.py > $O/fused.log 2>&1
echo "fused: $(tail -1 $O/fused.log)"
grep -h FAILED $O/fused.log || true
