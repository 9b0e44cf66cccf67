#!/bin/bash
# tools/r04_measure.sh TAG -- tools/measure_round.sh TAG (bench line, kernel
# trace, FETCH_SIZE pass, randbench calibration), then the multi-GPU step at
# world 1 and the single-GPU step back to back on the same box.
set -euo pipefail
TAG=${1:?tag}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
"$R/tools/measure_round.sh" "$TAG"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-feed --no-c5"
SMASH_BENCH_SHARDED=1 timeout -k 10 300 python3 -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29551 "$R/bench.py" \
    $ARGS > "$O/sharded_w1.json" 2> "$O/sharded_w1.log"
timeout -k 10 300 python3 "$R/bench.py" $ARGS > "$O/single.json" 2> "$O/single.log"
exit 0
