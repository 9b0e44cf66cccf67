#!/bin/bash
# tools/r05_cu.sh TAG -- the C3 step with the search held to fewer blocks per
# CU (SMASH_SM_BLOCKS_PER_CU), so the post stage of the previous batch gets
# wave slots while the search runs: default (16), 15, 14, 13, back to back.
set -euo pipefail
TAG=${1:?tag}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-feed --no-c5"
for B in ${BLOCKS:-16 15 14 13}; do
  SMASH_SM_BLOCKS_PER_CU=$B timeout -k 10 240 python3 "$R/bench.py" $ARGS > "$O/b$B.json" 2> "$O/b$B.log"
done
