#!/bin/bash
# tools/r03_ab.sh TAG -- round-3 schedule A/B: the gpu tests of the phases /
# parity files, the measured round (bench line, trace, FETCH_SIZE), then
# bench runs with SMASH_BENCH_RESIDENT=0 and SMASH_PREP_LDS=1.
set -euo pipefail
TAG=${1:?tag}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
"$R/tools/gpu_round.sh" "$TAG" "phases or parity"
cd /tmp
SMASH_BENCH_RESIDENT=0 timeout -k 10 300 python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline \
    --no-feed --no-c5 > "$O/nonres.json" 2> "$O/nonres.log"
SMASH_PREP_LDS=1 timeout -k 10 300 python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline \
    --no-feed --no-c5 > "$O/prep_lds.json" 2> "$O/prep_lds.log"
