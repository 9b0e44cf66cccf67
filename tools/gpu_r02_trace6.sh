#!/bin/bash
# rocprofv3 kernel trace + stats of the default C3 bench (6.25 M-pair batches)
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02t6}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv \
    -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-feed --no-c5 > $O/prof.json 2> $O/prof.log || exit 1
grep timed $O/prof.log | cut -c1-130
