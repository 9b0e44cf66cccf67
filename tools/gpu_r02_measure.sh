#!/bin/bash
# round-2 committed measurements: tools/measure_round.sh (bench, kernel trace,
# FETCH_SIZE + calibration), then the SQ counter passes (tools/profile_pmc.sh)
set -uo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r02m}
bash $R/tools/measure_round.sh $TAG || exit 1
tail -3 $R/gpurun_out/$TAG/bench.log
bash $R/tools/profile_pmc.sh c3 gpurun_out/$TAG/sq
