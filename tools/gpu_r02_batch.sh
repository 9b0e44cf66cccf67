#!/bin/bash
# the C3 step at 4 M vs 6.25 M pairs per batch, alternating, same build
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02batch}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for k in 1 2; do
  for b in 4000000 6250000; do
    timeout -k 10 400 python3 -u $R/bench.py --steps 3 --no-cpu-baseline --no-feed --no-c5 --batch $b > $O/b$b.$k.json 2> $O/b$b.$k.log || exit 1
    echo "$b.$k $(grep timed $O/b$b.$k.log | cut -c20-75)"
  done
done
