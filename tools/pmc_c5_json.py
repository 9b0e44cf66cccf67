"""tools/pmc_c5_json.py MEASURE_DIR PROFILE_DIR -- profiles/pmc_c5.json: the HBM
bytes of one C5 rep (smash_mappability_prepare: k_upart1-3, k_nsdir; the scan:
k_tilebins, k_mapscan, k_mapfix) from the FETCH_SIZE and WRITE_SIZE passes of
`bench.py --config c5 --steps 1` (tools/r06_run.sh part 4).  The last rep's
dispatches are the ones from the last k_upart1 on.  Every pass of the rep is a
wide coalesced stream, for which gfx950's FETCH_SIZE reports half the bytes
(MI355X_MICROARCH.md, HBM/rocprofv3 section): fetched = 2 x FETCH_SIZE;
WRITE_SIZE is exact for 16-byte streaming stores.  bench.py reports the sum as
c5.roofline.traffic."""
import csv
import glob
import json
import os
import re
import sys


def per_kernel(mdir, counter):
    f = glob.glob(os.path.join(mdir, "pmc_c5_%s" % counter, "**", "*counter_collection.csv"),
                  recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))
    names = [re.search(r"\b(k_\w+)", r["Kernel_Name"]).group(1) for r in rows]
    last = max(i for i, n in enumerate(names) if n == "k_upart1")
    out = {}
    for n, r in zip(names[last:], rows[last:]):
        out[n] = out.get(n, 0.0) + float(r["Counter_Value"]) * 1024
    return out, os.path.relpath(f, mdir)


def main(mdir, pdir):
    fe, fsrc = per_kernel(mdir, "FETCH_SIZE")
    wr, wsrc = per_kernel(mdir, "WRITE_SIZE")
    fetched = {k: 2 * v for k, v in fe.items()}
    total = sum(fetched.values()) + sum(wr.values())
    out = {"c5_bytes_per_rep": int(total),
           "fetched_bytes": {k: int(v) for k, v in sorted(fetched.items())},
           "written_bytes": {k: int(v) for k, v in sorted(wr.items())},
           "method": "2 x FETCH_SIZE (streaming reads: gfx950 counts half) + WRITE_SIZE, per "
                     "kernel of the last rep",
           "source": "%s/pmc_c5_{FETCH_SIZE,WRITE_SIZE}.csv (rocprofv3 --pmc, tools/r06_run.sh "
                     "part 4)" % pdir}
    json.dump(out, open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                     "profiles", "pmc_c5.json"), "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(*sys.argv[1:])
