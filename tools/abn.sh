#!/bin/bash
# tools/abn.sh OUT LIB... -- A/B/... timing of several builds of libsmashgpu.so
# on one box: tools/sweep.py once per library (SMASH_LIB), round-robin twice,
# each in its own process (genome + index + reads rebuilt per process).
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$1
shift
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for k in 1 2; do
  for L in "$@"; do
    n=$(basename "$L" .so)
    timeout -k 10 300 env SMASH_LIB="$R/$L" python3 -u "$R/tools/sweep.py" --steps 5 base > "$O/$n.$k.log" 2>&1
    echo "$n.$k $(grep -h 'sweep\] base' "$O/$n.$k.log")"
  done
done
