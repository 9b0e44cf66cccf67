#!/bin/bash
# tools/r03_sharded.sh TAG -- the multi-GPU step (dist.ShardedCounter:
# all_to_all key de-dup, all_gather tails, all_reduce counts over RCCL) at
# world 1 on one GPU (SMASH_BENCH_SHARDED=1 under torchrun): the per-rank
# rate of bench.py --gpus N > 1, next to the single-GPU step's.
set -euo pipefail
TAG=${1:?tag}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for A2 in 1 0; do   # batch b + 2's search after b's export (smash_phase_search_ahead) or not
  SMASH_BENCH_AHEAD2=$A2 SMASH_BENCH_SHARDED=1 timeout -k 10 600 python3 -m torch.distributed.run \
      --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2953$A2 "$R/bench.py" \
      --steps 5 --warmup 1 --no-cpu-baseline --no-feed --no-c5 \
      > "$O/sharded_w1_ahead2_$A2.json" 2> "$O/sharded_w1_ahead2_$A2.log"
done
