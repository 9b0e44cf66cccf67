#!/bin/bash
# A/B round 3 of this session: parity on the in-tree build (shared scan masks,
# k_bin cell directory); HEAD vs it vs it without the A_ROOT consolidation;
# the old (modulo, random 16-B offset) random-load ceiling next to the req one
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab3
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread $R/tests/test_gpu_parity.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash $R/tools/abn.sh ab3 ab/libA_head.so ab/libF_shared.so ab/libG_noroot.so || exit 1
timeout -k 10 300 $R/tools/randbench 64 > $O/randbench_chase.log 2>&1 || exit 1
cat $O/randbench_chase.log
