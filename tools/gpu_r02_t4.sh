#!/bin/bash
# k_post_fast tiers + C5 scan changes: the affected GPU tests, a sweep
# profile, then a short bench (C3 5 M pairs + C5, no CPU baseline)
set -uo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r02_t4
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread \
    $R/tests/test_gpu_mappability.py $R/tests/test_gpu_phases.py $R/tests/test_gpu_parity.py \
    $R/tests/test_gpu_modes.py "$R/tests/test_gpu_configs.py::test_c5_mappability_scan_full_genome" \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash $R/tools/gpu_prof_sweep.sh r02_t4/prof || exit 1
timeout -k 10 600 python3 -u $R/bench.py --steps 2 --pairs 5000000 --no-cpu-baseline > $O/bench.json 2> $O/bench.log
rc=$?
tail -3 $O/bench.log
exit $rc
