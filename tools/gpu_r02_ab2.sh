#!/bin/bash
# round-2 A/B call: exact-address probes (B) vs the round-2 base (A), the
# mappability scan tests, the random-probe ceilings on this box
set -uo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r02_ab2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
    $R/tests/test_gpu_mappability.py > $O/tests_map.log 2>&1 || { tail -30 $O/tests_map.log; exit 1; }
tail -2 $O/tests_map.log
SWEEP_B=SMASH_SM_STATS=1 bash $R/tools/ab.sh gpurun_out/r02_ab2 ab/libA_r02base.so ab/libB_ua.so > $O/ab.txt 2>&1
cat $O/ab.txt
grep -h "k_mam_sm\]" $O/b1.log | head -3
timeout -k 10 200 $R/tools/randbench lines 0.03 32 > $O/randbench.log 2>&1
timeout -k 10 200 $R/tools/randbench 32 >> $O/randbench.log 2>&1
cat $O/randbench.log
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 500 --timeout-method thread \
    "$R/tests/test_gpu_configs.py::test_c5_mappability_scan_full_genome" > $O/tests_c5.log 2>&1
tail -2 $O/tests_c5.log
