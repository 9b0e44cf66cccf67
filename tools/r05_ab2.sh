#!/bin/bash
# tools/r05_ab2.sh TAG -- checks of the round-5 kernels on one box: the
# mappability / MEM / packed-word tests, the C5 line, the C3 step with plain
# vs packed index words (A/B), and the c3mem line.
set -euo pipefail
TAG=${1:?tag}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
rc=0
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_mappability.py tests/test_gpu_configs.py -m gpu -v \
    --timeout 400 --timeout-method thread -k "${TESTS:-mappab or c5 or mem_hg19 or host_sample or idx8}" \
    > "$O/tests.log" 2>&1 || rc=$?
# (failed tests: go on with the measurements; a crash, abort or time limit: stop)
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-feed --no-c5"
timeout -k 10 200 python3 "$R/bench.py" --config c5 --steps 5 > "$O/c5.json" 2> "$O/c5.log"
SMASH_PACK_IDX=0 timeout -k 10 200 python3 "$R/bench.py" $ARGS > "$O/ab_plain.json" 2> "$O/ab_plain.log"
timeout -k 10 200 python3 "$R/bench.py" $ARGS > "$O/ab_packed.json" 2> "$O/ab_packed.log"
timeout -k 10 300 python3 "$R/bench.py" --config c3mem --steps 3 > "$O/c3mem.json" 2> "$O/c3mem.log"
exit 0
