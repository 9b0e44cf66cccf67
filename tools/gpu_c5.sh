#!/bin/bash
# C5 scan: the mappability tests, the C5 bench line, one SQ counter pass on k_mapscan
set -uo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/${1:-c5}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread \
    $R/tests/test_gpu_mappability.py "$R/tests/test_gpu_configs.py::test_c5_mappability_scan_full_genome" \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python3 -u $R/bench.py --config c5 --steps 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.log || exit 1
tail -2 $O/bench.log
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_ANY \
    --kernel-include-regex k_mapscan -d $O/pmc -o pmc --output-format csv \
    -- python3 $R/bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc.log 2>&1 || exit 1
python3 - $O <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float); n = set()
for r in csv.DictReader(open(sys.argv[1] + "/pmc/pmc_counter_collection.csv")):
    tot[r["Counter_Name"]] += float(r["Counter_Value"]); n.add(r["Dispatch_Id"])
print(len(n), "dispatches", {c: "%.4g" % v for c, v in sorted(tot.items())})
PY
