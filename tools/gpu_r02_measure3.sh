#!/bin/bash
# round-2 profiler evidence at the 4 M-pair default: the C3 full-run property
# test, kernel trace + stats, FETCH_SIZE on k_mam_sm with its calibration, and
# the C3 step at 6.25 M-pair batches for comparison
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02m3}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 500 --timeout-method thread $R/tests/test_gpu_configs.py -k c3_full_run > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv \
    -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-feed --no-c5 > $O/prof.json 2> $O/prof.log || exit 1
grep timed $O/prof.log
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_mam_sm -d $O/pmc -o pmc \
    --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-feed --no-c5 \
    > $O/pmc.json 2> $O/pmc.log || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/calib -o pmc --output-format csv \
    -- $R/tools/randbench calib > $O/calib.log 2>&1 || exit 1
timeout -k 10 600 python3 -u $R/bench.py --steps 3 --no-cpu-baseline --no-feed --no-c5 --batch 6250000 > $O/bench_b6m.json 2> $O/bench_b6m.log || exit 1
grep timed $O/bench_b6m.log
