#!/bin/bash
# tools/r04_prof_ab.sh TAG "ENV_B" -- one box: a rocprofv3 kernel trace of the
# default C3 step (3 timed steps, its breakdown by tools/step_breakdown.py),
# then the C3 bench alternating the default (A) and ENV_B (B), twice each.
# Each GPU step has its own limit; the chain stops at the first failure.
set -euo pipefail
TAG=${1:?tag}
B=${2:-}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-feed --no-c5"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-feed --no-c5 \
    > "$O/prof.json" 2> "$O/prof.log"
T=$(ls "$O"/prof/run_kernel_trace.csv "$O"/prof/*/run_kernel_trace.csv 2>/dev/null | head -1 || true)
if [ -n "$T" ]; then
  python3 "$R/tools/step_breakdown.py" "$T" 4 4 > "$O/step_breakdown.txt" || true
  python3 "$R/tools/roofline_from_trace.py" "$T" "$O/prof.json" > "$O/roofline_from_trace.txt" || true
fi
for i in 1 2; do
  timeout -k 10 300 python3 "$R/bench.py" $ARGS > "$O/a$i.json" 2> "$O/a$i.log"
  env $B timeout -k 10 300 python3 "$R/bench.py" $ARGS > "$O/b$i.json" 2> "$O/b$i.log"
done
exit 0
