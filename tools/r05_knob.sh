#!/bin/bash
# tools/r05_knob.sh TAG -- A/B of the search with its policy knobs fixed at
# compile time (HEAD) against the previous build (lib/libsmashgpu_base.so),
# then the search parity tests and the C3 line on HEAD's build.
set -euo pipefail
TAG=${1:?tag}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
bash "$R/tools/ab.sh" "gpurun_out/$TAG/ab" smash-paper_amd/lib/libsmashgpu_base.so \
    smash-paper_amd/lib/libsmashgpu.so > "$O/ab.txt" 2>&1
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_modes.py -m gpu -v \
    --timeout 500 --timeout-method thread > "$O/tests.log" 2>&1
cd /tmp
timeout -k 10 240 python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-feed --no-c5 \
    > "$O/c3.json" 2> "$O/c3.log"
