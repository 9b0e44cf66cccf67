#!/bin/bash
# tools/r05_run.sh TAG [tests|bench|both] -- the whole -m gpu suite and
# smoke(), then the default bench line (C3 + C5 + CPU baseline + ingest).
set -euo pipefail
TAG=${1:?tag}
WHAT=${2:-both}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
if [ "$WHAT" != bench ]; then
  timeout -k 10 1050 python3 -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread \
      > "$O/tests.log" 2>&1
  timeout -k 10 150 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
fi
if [ "$WHAT" != tests ]; then
  timeout -k 10 420 python3 bench.py > "$O/bench.json" 2> "$O/bench.log"
fi
exit 0
