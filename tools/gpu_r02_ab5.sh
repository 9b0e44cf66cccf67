#!/bin/bash
# A_TOP one-codes-pass (D) vs row DMA (C): parity tests, then A/B sweeps
set -uo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r02_ab5
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
true && \
  true

bash $R/tools/ab.sh gpurun_out/r02_ab5 ab/libC_dma.so ab/libD_atop.so > $O/ab.txt 2>&1
cat $O/ab.txt
