#!/bin/bash
# the multi-rank phase emulation on the fused positions + varbin path and on
# the two-kernel path (SMASH_FUSED_BIN=0), same build
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02ph}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
SMASH_FUSED_BIN=0 timeout -k 10 300 python3 -u -m pytest -q --timeout 200 --timeout-method thread $R/tests/test_gpu_phases.py > $O/phases_twokernel.log 2>&1
echo "two-kernel: $(tail -1 $O/phases_twokernel.log)"
timeout -k 10 300 python3 -u -m pytest -q --timeout 200 --timeout-method thread $R/tests/test_gpu_phases.py > $O/phases_fused.log 2>&1
echo "fused: $(tail -1 $O/phases_fused.log)"
grep -h FAILED $O/*.log || true
