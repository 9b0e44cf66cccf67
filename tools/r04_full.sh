#!/bin/bash
# tools/r04_full.sh TAG [TESTS] -- one box: the named -m gpu tests, the default
# bench line, then the single-GPU step and the multi-GPU step at world 1
# (dist.ShardedCounter over RCCL) back to back.  Each GPU step has its own
# limit; the chain stops at the first failure.
set -euo pipefail
TAG=${1:?tag}
TESTS=${2:-}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TLIM:-420} python3 -u -m pytest tests -m gpu -x -v --timeout 300 \
      --timeout-method thread -k "$TESTS" > "$O/tests.log" 2>&1
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 480 python3 "$R/bench.py" > "$O/bench.json" 2> "$O/bench.log"
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-feed --no-c5"
SMASH_BENCH_SHARDED=1 timeout -k 10 300 python3 -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29551 "$R/bench.py" \
    $ARGS > "$O/sharded_w1.json" 2> "$O/sharded_w1.log"
timeout -k 10 300 python3 "$R/bench.py" $ARGS > "$O/single.json" 2> "$O/single.log"
exit 0
