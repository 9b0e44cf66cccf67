#!/bin/bash
# tools/gpu_prof_sweep.sh TAG -- per-kernel times of one sweep.py run
# (rocprofv3 kernel trace + stats) of the tree's library
set -uo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/tools/sweep.py --steps 5 base > $O/sweep.log 2>&1
rc=$?
tail -3 $O/sweep.log
python3 $R/tools/prof_top.py $O/prof/run_results.db | tee $O/top.txt
exit $rc
