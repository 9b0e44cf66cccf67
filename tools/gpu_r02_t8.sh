#!/bin/bash
# search-stream priority A/B on the C3 bench (same library, env switch)
set -uo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r02_t8
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for k in 1 2; do
  timeout -k 10 400 python3 -u $R/bench.py --steps 3 --no-cpu-baseline --no-c5 --no-feed > $O/hi$k.json 2> $O/hi$k.log || exit 1
  grep timed $O/hi$k.log
  SMASH_SEARCH_PRIORITY=0 timeout -k 10 400 python3 -u $R/bench.py --steps 3 --no-cpu-baseline --no-c5 --no-feed > $O/def$k.json 2> $O/def$k.log || exit 1
  grep timed $O/def$k.log
done
