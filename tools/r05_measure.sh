#!/bin/bash
# tools/r05_measure.sh TAG -- the round-5 measurement set, one box:
#   1. bench.py default line (C3 + CPU baseline + file-fed + C5)      -> bench.json/.log
#   2. A/B: the C3 step with plain index words (SMASH_PACK_IDX=0) and
#      packed (default), back to back                                  -> ab_plain / ab_packed
#   3. rocprofv3 --kernel-trace --stats of a 3-step C3 bench          -> prof/
#   4. rocprofv3 --pmc FETCH_SIZE on k_mam_sm (one step)              -> pmc/
#   5. FETCH_SIZE calibration for random 16-byte probes (randbench)  -> calib/
#   6. rocprofv3 --kernel-trace --stats of the C5 line               -> prof_c5/
# Each GPU step has its own time limit; the chain stops at the first failure.
set -euo pipefail
TAG=${1:?tag}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-feed --no-c5"
timeout -k 10 420 python3 "$R/bench.py" > "$O/bench.json" 2> "$O/bench.log"
SMASH_PACK_IDX=0 timeout -k 10 200 python3 "$R/bench.py" $ARGS > "$O/ab_plain.json" 2> "$O/ab_plain.log"
timeout -k 10 200 python3 "$R/bench.py" $ARGS > "$O/ab_packed.json" 2> "$O/ab_packed.log"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-feed --no-c5 \
    > "$O/prof.json" 2> "$O/prof.log"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_mam_sm -d "$O/pmc" -o pmc \
    --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-feed \
    --no-c5 > "$O/pmc.log" 2>&1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d "$O/calib" -o pmc --output-format csv \
    -- "$R/tools/randbench" calib > "$O/calib.log" 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/prof_c5" -o run --output-format csv \
    -- python3 "$R/bench.py" --config c5 --steps 5 --warmup 1 --no-cpu-baseline \
    > "$O/prof_c5.json" 2> "$O/prof_c5.log"
exit 0
