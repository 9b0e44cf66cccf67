#!/bin/bash
# tools/r04_sharded.sh TAG -- the single-GPU step and the multi-GPU step
# (dist.ShardedCounter at world 1: RCCL collectives to itself) on the same
# box, back to back, then a kernel trace of the sharded step for its
# breakdown (tools/step_breakdown.py).  Each step has its own time limit.
set -euo pipefail
TAG=${1:?tag}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-feed --no-c5"
timeout -k 10 400 python3 "$R/bench.py" $ARGS > "$O/single.json" 2> "$O/single.log"
SMASH_BENCH_SHARDED=1 timeout -k 10 400 python3 -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29551 "$R/bench.py" \
    $ARGS > "$O/sharded_w1.json" 2> "$O/sharded_w1.log"
timeout -k 10 400 python3 "$R/bench.py" $ARGS > "$O/single2.json" 2> "$O/single2.log"
if [ "${PROF:-1}" = "1" ]; then
  SMASH_BENCH_SHARDED=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29552 \
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv \
      -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-feed --no-c5 \
      > "$O/prof.log" 2>&1
  T=$(ls "$O"/prof/*/run_kernel_trace.csv 2>/dev/null | head -1 || true)
  [ -n "$T" ] && python3 "$R/tools/step_breakdown.py" "$T" 4 4 > "$O/step_breakdown.txt" || true
fi
exit 0
