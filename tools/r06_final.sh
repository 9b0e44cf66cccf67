#!/bin/bash
# tools/r06_final.sh TAG -- the closing checks of round 6 on one box: the whole
# -m gpu suite, smoke(), then the default bench line with the driver's
# arguments (C3 + CPU baseline + file-fed + C2 + MEM + C5)
set -uo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/${1:?tag}
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread \
    > "$O/tests.log" 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.log"
exit $rc
