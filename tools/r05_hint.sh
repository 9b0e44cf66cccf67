#!/bin/bash
# tools/r05_hint.sh TAG -- the map hints (forward matches' right map.bin
# byte from the search): the pipeline tests that run packed indexes (idx8,
# the hg19 C2 / C3 checks against the oracle), then the C3 step with the
# hints off and on, twice, on one box.
set -euo pipefail
TAG=${1:?tag}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
rc=0
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -v --timeout 500 \
    --timeout-method thread -k "idx8 or c2 or c3_sample or c3_full or production" > "$O/tests.log" 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-feed --no-c5"
for k in 1 2; do
  SMASH_MAP_HINT=0 timeout -k 10 240 python3 "$R/bench.py" $ARGS > "$O/off$k.json" 2> "$O/off$k.log"
  timeout -k 10 240 python3 "$R/bench.py" $ARGS > "$O/on$k.json" 2> "$O/on$k.log"
done
exit $rc
