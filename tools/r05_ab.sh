#!/bin/bash
# tools/r05_ab.sh TAG [TESTS] -- a search-kernel change: the production-batch
# and packed-index parity tests (they run the GEO kernel), then the C3 step
# on the previous build (lib/libsmashgpu_base.so) and this one, alternating,
# on one box.
set -euo pipefail
TAG=${1:?tag}
SEL=${2:-production or idx8}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -v \
    --timeout 400 --timeout-method thread -k "$SEL" > "$O/tests.log" 2>&1
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-feed --no-c5"
for k in 1 2; do
  SMASH_LIB="$R/smash-paper_amd/lib/libsmashgpu_base.so" timeout -k 10 240 python3 "$R/bench.py" $ARGS \
      > "$O/base$k.json" 2> "$O/base$k.log"
  timeout -k 10 240 python3 "$R/bench.py" $ARGS > "$O/new$k.json" 2> "$O/new$k.log"
done
