#!/bin/bash
# tools/r05_diag.sh TAG -- what bounds the packed-word k_mam_sm (round 5):
#   1. a STATS run (lane iterations per state, wave iterations per region) -> stats.log
#   2. tools/sweep.py on one 2 M-pair batch: base, +16 / +64 dependent VALU
#      per iteration (SMASH_SM_PAD), 12 blocks per CU, no probe bounds check
#      (SMASH_SM_CHECK=0)                                                   -> sweep.log
#   3. two SQ counter passes on k_mam_sm (issue and wait cycles, instruction
#      counts; one step)                                                    -> sq1/, sq2/
# NO_STATS=1 / NO_SWEEP=1 skip steps 1 / 2.
# Each GPU step has its own time limit; the chain stops at the first failure.
set -euo pipefail
TAG=${1:?tag}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --no-feed --no-c5"
if [ -z "${NO_STATS:-}" ]; then
  timeout -k 10 300 env SMASH_SM_STATS=1 python3 "$R/bench.py" $ARGS > "$O/stats.json" 2> "$O/stats.log"
fi
if [ -z "${NO_SWEEP:-}" ]; then
  timeout -k 10 400 python3 "$R/tools/sweep.py" --steps 3 base SMASH_SM_PAD=16 SMASH_SM_PAD=64 \
      SMASH_SM_BLOCKS_PER_CU=12 SMASH_SM_CHECK=0 base > "$O/sweep.log" 2>&1
fi
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-include-regex k_mam_sm \
    -d "$O/sq1" -o pmc --output-format csv -- python3 "$R/bench.py" $ARGS > "$O/sq1.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU \
    SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM --kernel-include-regex k_mam_sm \
    -d "$O/sq2" -o pmc --output-format csv -- python3 "$R/bench.py" $ARGS > "$O/sq2.log" 2>&1
exit 0
