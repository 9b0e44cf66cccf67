#!/bin/bash
# bench lines for the other BASELINE configs on one MI355X: C2 (hg19-shaped,
# 1 M x 100 bp, 100 k bins) and C1 (chr21-sized, 10 k x 100 bp, 500 k bins)
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02cfg}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in c2 c1; do
  timeout -k 10 500 python3 -u $R/bench.py --config $c --no-feed --no-c5 > $O/bench_$c.json 2> $O/bench_$c.log || exit 1
  echo "$c: $(grep timed $O/bench_$c.log | cut -c1-110)"
done
