#!/bin/bash
# tools/diag_sq.sh [OUT] -- where k_mam_sm's time goes: a STATS run (lane
# iterations per state, active lanes per wave iteration), A/B timings of the
# issue-bound probes (SMASH_SM_PAD adds dependent VALU per iteration;
# SMASH_SM_BLOCKS_PER_CU caps occupancy), then the SQ counter passes.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/${1:-gpurun_out/diag}
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 env SMASH_SM_STATS=1 python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline \
    > "$O/stats.json" 2> "$O/stats.log"
timeout -k 10 400 python3 "$R/tools/sweep.py" --steps 3 base SMASH_SM_PAD=16 SMASH_SM_PAD=64 \
    SMASH_SM_BLOCKS_PER_CU=8 SMASH_SM_BLOCKS_PER_CU=12 > "$O/sweep.log" 2>&1
bash "$R/tools/profile_pmc.sh" c3 "${1:-gpurun_out/diag}/pmc"
