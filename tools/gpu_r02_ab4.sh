#!/bin/bash
# row LDS-DMA (C) vs prefetch-only (B): parity tests, then A/B sweeps
set -uo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r02_ab4
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
true && \
  true && \
  true

SWEEP_B=SMASH_SM_STATS=1 bash $R/tools/ab.sh gpurun_out/r02_ab4 ab/libA_head.so ab/libC_dma.so > $O/ab.txt 2>&1
cat $O/ab.txt
grep -h "k_mam_sm\]" $O/b1.log | head -3
