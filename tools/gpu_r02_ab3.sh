#!/bin/bash
# round-2 A/B call: binary-search child prefetch (B = the tree's library) vs
# the previous head (A = ab/libA_head.so); the phase and parity tests first
set -uo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r02_ab3
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
    $R/tests/test_gpu_phases.py $R/tests/test_gpu_parity.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cp $R/smash-paper_amd/lib/libsmashgpu.so $R/ab/libB_pf.so
SWEEP_B=SMASH_SM_STATS=1 bash $R/tools/ab.sh gpurun_out/r02_ab3 ab/libA_head.so ab/libB_pf.so > $O/ab.txt 2>&1
cat $O/ab.txt
grep -h "k_mam_sm\]" $O/b1.log | head -3
