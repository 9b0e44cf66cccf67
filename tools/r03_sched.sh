#!/bin/bash
# tools/r03_sched.sh TAG -- the C3 step's schedule A/B in one process
# (tools/sweep.py, resident reads, 4 x 6.25 M-pair batches per run; every
# setting must give the base's counts), then FETCH_SIZE / WRITE_SIZE and the
# SQ issue counters of the post-stage kernels (rocprofv3 serialises the
# dispatches of a --pmc pass: isolated per-kernel figures; PMC=1).
# SETTINGS overrides the sweep's settings.
set -euo pipefail
TAG=${1:?tag}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u "$R/tools/sweep.py" --pairs 25000000 --batch 6250000 --steps 5 --resident \
    ${SETTINGS:-base SMASH_GATE_POST=0,SMASH_PREP_LDS=0 SMASH_PRIO=0 SMASH_ONE_SEARCH=1 SMASH_BIN_LDS=1 SMASH_ONE_SEARCH=1,SMASH_PRIO=0 base} \
    > "$O/sweep.log" 2>&1
[ "${PMC:-0}" = "1" ] || exit 0
POST='k_post_fast|k_dedup|k_emit_bin|k_prep|k_scan|k_post'
for C in FETCH_SIZE WRITE_SIZE; do   # one TCC counter per pass (3 + 2 > 4 TCC slots)
  timeout -s KILL 180 rocprofv3 --pmc $C --kernel-include-regex "$POST" \
      -d "$O/pmc_post_$C" -o pmc --output-format csv \
      -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-feed --no-c5 \
      > "$O/pmc_post_$C.log" 2>&1
done
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "$POST" \
    -d "$O/pmc_post_sq" -o pmc --output-format csv \
    -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-feed --no-c5 \
    > "$O/pmc_post_sq.log" 2>&1
