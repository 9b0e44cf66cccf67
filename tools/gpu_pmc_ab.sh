#!/bin/bash
# tools/gpu_pmc_ab.sh OUT LIB_A LIB_B -- SQ counters of k_mam_sm (sweep.py
# runs, one rocprofv3 --pmc pass per library)
set -uo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for k in A B; do
  L=$2; [ $k = B ] && L=$3
  SMASH_LIB=$R/$L timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH \
      SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS --kernel-include-regex k_mam_sm \
      -d $O/$k -o pmc --output-format csv -- python3 $R/tools/sweep.py --steps 2 base > $O/$k.log 2>&1 || exit 1
done
python3 - "$O" <<'PY'
import csv, sys, collections
for k in "AB":
    tot = collections.defaultdict(float); n = set()
    for r in csv.DictReader(open(f"{sys.argv[1]}/{k}/pmc_counter_collection.csv")):
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n.add(r["Dispatch_Id"])
    print(k, len(n), "dispatches", {c: "%.4g" % (v / len(n)) for c, v in sorted(tot.items())})
PY
