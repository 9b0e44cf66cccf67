#!/bin/bash
# tools/gpu_regions.sh OUT -- the STATS run of the tree's library: lane
# iterations per state and the share of wave iterations each region runs in
set -uo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/tools/sweep.py --steps 2 base SMASH_SM_STATS=1 > $O/stats.log 2>&1
rc=$?
grep -h "k_mam_sm\]\|sweep\] [a-zA-Z]" $O/stats.log | head -8
exit $rc
