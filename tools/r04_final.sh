#!/bin/bash
# tools/r04_final.sh TAG -- the whole -m gpu suite, smoke(), then the
# multi-GPU step at world 1 and the single-GPU step back to back.
set -euo pipefail
TAG=${1:?tag}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 780 python3 -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread \
    > "$O/tests.log" 2>&1
timeout -k 10 150 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-feed --no-c5"
SMASH_BENCH_SHARDED=1 timeout -k 10 240 python3 -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29551 "$R/bench.py" \
    $ARGS > "$O/sharded_w1.json" 2> "$O/sharded_w1.log"
timeout -k 10 200 python3 "$R/bench.py" $ARGS > "$O/single.json" 2> "$O/single.log"
exit 0
