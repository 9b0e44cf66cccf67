#!/bin/bash
# round-6 session 3: (1) U rebuild with 16 k-entry tiles in passes 1 and 2:
# parity tests, C5 prepare A/B (and the round-5 code, libsmashgpu_u0.so);
# (2) search streams at their own priority (SMASH_SEARCH_PRIO: a hardware
# queue from another pool) -- single-GPU and world-1 sharded steps
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r06u
mkdir -p "$O"
cd "$R"
python3 -c "import torch; print('stream priority range', torch.cuda.Stream.priority_range())" > "$O/prio.txt" 2>&1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_mappability.py -m gpu -v -k "prepare" \
    --timeout 200 --timeout-method thread > "$O/tests_mid.log" 2>&1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -v -k "c5_prepare" \
    --timeout 300 --timeout-method thread > "$O/tests_hg19.log" 2>&1
ROUNDS=2 timeout -k 10 300 python3 -u tools/c5_ab.py nt1024: p2_512:SMASH_UPART_NT2=512 \
    nt512:SMASH_UPART_NT=512,SMASH_UPART_NT2=512 > "$O/c5ab.log" 2>&1
ROUNDS=2 SMASH_LIB=$R/smash-paper_amd/lib/libsmashgpu_u0.so timeout -k 10 200 python3 -u \
    tools/c5_ab.py u0: > "$O/c5ab_u0.log" 2>&1
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-feed --no-c5 --no-sub"
port=29560
for pr in none high low; do
  SMASH_SEARCH_PRIO=$pr timeout -k 10 300 python3 "$R/bench.py" $ARGS > "$O/single_$pr.json" 2> "$O/single_$pr.log"
  port=$((port + 1))
  SMASH_SEARCH_PRIO=$pr SMASH_BENCH_SHARDED=1 timeout -k 10 300 python3 -m torch.distributed.run \
      --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port "$R/bench.py" \
      $ARGS > "$O/sharded_$pr.json" 2> "$O/sharded_$pr.log"
done
