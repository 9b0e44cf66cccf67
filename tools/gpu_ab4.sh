#!/bin/bash
# A/B round 4 of this session: parity on the in-tree build (16-byte k_prep
# accesses), the committed build vs it on the C3 step (bench, 4 M batches)
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab4
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread $R/tests/test_gpu_parity.py $R/tests/test_gpu_modes.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
  for L in libH_final libI_prep; do
    SMASH_LIB=$R/ab/$L.so timeout -k 10 400 python3 -u $R/bench.py --steps 3 --no-cpu-baseline --no-feed --no-c5 > $O/$L.$k.json 2> $O/$L.$k.log || exit 1
    echo "$L.$k $(grep timed $O/$L.$k.log | cut -c1-120)"
  done
done
