#!/bin/bash
# tools/r05_rows.sh TAG -- dense hit rows (HitRows): the pipeline parity
# tests (per-pair hit lists, post paths, C2 / C3 / idx8 / the multi-GPU
# driver vs the oracle), then the C3 step on HEAD's build and on the previous
# one (lib/libsmashgpu_base.so), alternating, on one box.
set -euo pipefail
TAG=${1:?tag}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -v \
    --timeout 600 --timeout-method thread -k "not production and not mem_hg19 and not c5" \
    > "$O/tests.log" 2>&1
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-feed --no-c5"
for k in 1 2; do
  SMASH_LIB="$R/smash-paper_amd/lib/libsmashgpu_base.so" timeout -k 10 240 python3 "$R/bench.py" $ARGS \
      > "$O/base$k.json" 2> "$O/base$k.log"
  timeout -k 10 240 python3 "$R/bench.py" $ARGS > "$O/new$k.json" 2> "$O/new$k.log"
done
