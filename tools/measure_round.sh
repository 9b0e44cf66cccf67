#!/bin/bash
# tools/measure_round.sh TAG -- the measurements committed under profiles/:
#   1. bench.py (default: C3, N=1, with the CPU baseline)          -> TAG_bench.json/.log
#   2. rocprofv3 --kernel-trace --stats of a 3-step bench          -> TAG_prof/
#   3. rocprofv3 --pmc FETCH_SIZE on k_mam_sm (one step)          -> TAG_pmc/
#   4. FETCH_SIZE calibration for random 16-byte probes (randbench) -> TAG_calib/
# Each GPU step has its own time limit; the chain stops at the first failure.
set -euo pipefail
TAG=${1:-r01}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 "$R/bench.py" > "$O/bench.json" 2> "$O/bench.log"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-feed --no-c5 > "$O/prof.log" 2>&1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_mam_sm -d "$O/pmc" -o pmc \
    --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-feed --no-c5 \
    > "$O/pmc.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$O/calib" -o pmc --output-format csv \
    -- "$R/tools/randbench" calib > "$O/calib.log" 2>&1
# 5. (POST_PMC=1) issue/wait counters of the post-stage kernels, one step
if [ "${POST_PMC:-0}" = "1" ]; then
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
      SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
      --kernel-include-regex 'k_post_fast|k_dedup|k_emit_bin|k_prep|k_scan|k_count_last' \
      -d "$O/pmc_post" -o pmc --output-format csv \
      -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-feed --no-c5 \
      > "$O/pmc_post.log" 2>&1
fi
