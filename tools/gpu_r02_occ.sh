#!/bin/bash
# the C3 step (4 M-pair batches) with the search grid at 16 (default), 15 and
# 14 blocks per CU: room for the post stage of the previous batch to run
# beside the search instead of after it
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02occ}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for b in 16 15 14; do
  SMASH_SM_BLOCKS_PER_CU=$b timeout -k 10 500 python3 -u $R/bench.py --steps 3 --no-cpu-baseline --no-feed --no-c5 > $O/bench_occ$b.json 2> $O/bench_occ$b.log || exit 1
  echo "blocks/CU $b: $(grep timed $O/bench_occ$b.log)"
done
