#!/bin/bash
# tools/profile_pmc.sh CONFIG OUTDIR -- rocprofv3 counter passes on k_mam
# (each pass its own run, --kernel-trace/--pmc only, per the gfx950 rules).
set -euo pipefail
CFG=${1:-c3}
OUT=${2:-gpurun_out/pmc}
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_WAIT_INST_LDS" \
           "FETCH_SIZE TCC_HIT_sum" ; do
  i=$((i+1))
  timeout -k 10 420 rocprofv3 --pmc $SET --kernel-include-regex k_mam -d "$R/$OUT/p$i" -o pmc \
      --output-format csv -- python3 "$R/bench.py" --config "$CFG" --steps 1 --warmup 0 \
      --no-cpu-baseline --no-feed --no-c5 > "$R/$OUT/p$i.json" 2> "$R/$OUT/p$i.log"
done
