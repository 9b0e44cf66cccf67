#!/bin/bash
# A/B round 5 of this session: parity on the in-tree build (fused positions +
# varbin, k_emit_bin), including the phase-API and CLI tests that read the
# positions back, then the committed build, + 16-byte k_prep, + fused on the C3 step
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab5
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread $R/tests/test_gpu_parity.py $R/tests/test_gpu_phases.py $R/tests/test_gpu_feed.py $R/tests/test_cli.py $R/tests/test_dropin.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
  for L in libH_final libI_prep libJ_fused; do
    SMASH_LIB=$R/ab/$L.so timeout -k 10 400 python3 -u $R/bench.py --steps 3 --no-cpu-baseline --no-feed --no-c5 > $O/$L.$k.json 2> $O/$L.$k.log || exit 1
    echo "$L.$k $(grep timed $O/$L.$k.log | cut -c1-120)"
  done
done
