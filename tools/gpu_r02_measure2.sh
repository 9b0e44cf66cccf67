#!/bin/bash
# the profiler passes of tools/measure_round.sh without the bench line (kernel
# trace, FETCH_SIZE + calibration), then the SQ counter passes
set -uo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/${1:-r02m2}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-feed --no-c5 > "$O/prof.log" 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_mam_sm -d "$O/pmc" -o pmc \
    --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-feed --no-c5 \
    > "$O/bench.json" 2> "$O/pmc.log" || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$O/calib" -o pmc --output-format csv \
    -- "$R/tools/randbench" calib > "$O/calib.log" 2>&1 || exit 1
bash $R/tools/profile_pmc.sh c3 gpurun_out/${1:-r02m2}/sq
