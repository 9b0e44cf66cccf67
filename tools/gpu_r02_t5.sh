#!/bin/bash
# C5 fixup list: the mappability tests and a short bench; then the k_mam PMC
# passes (tools/profile_pmc.sh)
set -uo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r02_t5
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread \
    $R/tests/test_gpu_mappability.py "$R/tests/test_gpu_configs.py::test_c5_mappability_scan_full_genome" \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python3 -u $R/bench.py --steps 1 --pairs 2000000 --no-cpu-baseline > $O/bench.json 2> $O/bench.log || exit 1
tail -2 $O/bench.log
bash $R/tools/profile_pmc.sh c3 gpurun_out/r02_t5/pmc
