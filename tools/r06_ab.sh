#!/bin/bash
# tools/r06_ab.sh TAG "LIB1 LIB2 ..." -- A/B of library builds on one box:
# first the parity tests $TESTS (default: production batch + idx8, which run
# the GEO search) on the tree's own lib, then the C3 step (5 timed steps, no
# side lines) once per library per round, $ROUNDS rounds (default 2),
# alternating.  LIBn: a file name under smash-paper_amd/lib ("-" = the tree's
# libsmashgpu.so).  Each GPU step has its own time limit; the chain stops at a
# crash or time limit.
set -euo pipefail
TAG=${1:?tag}
LIBS=${2:?libs}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
if [ "${TESTS:-production or idx8}" != "none" ]; then
  rc=0
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -v \
      --timeout 400 --timeout-method thread -k "${TESTS:-production or idx8}" > "$O/tests.log" 2>&1 || rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-feed --no-c5 --no-sub ${BENCH_ARGS:-}"
for k in $(seq 1 "${ROUNDS:-2}"); do
  for L in $LIBS; do
    n=${L#libsmashgpu}; n=${n%.so}; n=${n#_}; [ "$L" = "-" ] && n=head
    lib=$R/smash-paper_amd/lib/${L}
    [ "$L" = "-" ] && lib=$R/smash-paper_amd/lib/libsmashgpu.so
    SMASH_LIB="$lib" timeout -k 10 240 python3 "$R/bench.py" $ARGS > "$O/${n:-head}$k.json" 2> "$O/${n:-head}$k.log"
  done
done
python3 - "$O" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
        r = d["roofline"]
        print("%-14s %.4e reads/s  %.2f ms/step  k_mam %.2f / %.2f ms  non-search %.2f" % (
            os.path.basename(f), d["value"], d["ms_per_step"], r["avg_kernel_ms"],
            r["active_ms_per_launch"], r["non_search_ms_per_step"]))
    except Exception as e:
        print(f, "?", e)
PY
