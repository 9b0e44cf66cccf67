#!/bin/bash
# tools/r04_sweep.sh TAG SETTING... -- the C3 bench (no CPU baseline, feed or
# C5) for each setting "ENV=V ...|extra bench args", all settings in turn,
# twice, on one box.  Each run has its own limit; the chain stops at the
# first failure.
set -euo pipefail
TAG=${1:?tag}; shift
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  i=0
  for s in "$@"; do
    i=$((i + 1))
    E=${s%%|*}; A=${s#*|}
    [ "$A" = "$s" ] && A=""
    env $E timeout -k 10 300 python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline \
        --no-feed --no-c5 $A > "$O/s${i}_r$rep.json" 2> "$O/s${i}_r$rep.log"
    echo "s$i r$rep [$s] done" >> "$O/sweep.txt"
  done
done
exit 0
