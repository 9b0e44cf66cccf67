#!/bin/bash
# tools/r06_shard.sh TAG -- the world-1 multi-GPU step against the single-GPU
# step with its kernel trace (tools/r04_sharded.sh), and a kernel profile of
# one index build (tools/r06_idxprof.sh)
set -euo pipefail
TAG=${1:?tag}
R=$(cd "$(dirname "$0")/.." && pwd)
bash "$R/tools/r04_sharded.sh" "$TAG"
bash "$R/tools/r06_idxprof.sh" "$TAG/idx"
