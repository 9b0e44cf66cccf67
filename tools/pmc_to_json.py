"""tools/pmc_to_json.py MEASURE_DIR PROFILE_DIR [CONFIG] -- profiles/pmc_<config>.json
from a tools/measure_round.sh output directory.

FETCH_SIZE (kB) of the k_mam_sm dispatch is converted to bytes with the
randbench calibration of the same call (dependent random 16-byte probes, one
per 64-B line: FETCH_SIZE must count 64 B per probe; the measured ratio
rescales the kernel's figure), as MI355X_MICROARCH.md's HBM/rocprofv3 section
prescribes for gfx950.  bench.py reports the result as roofline.traffic.
"""
import csv
import json
import os
import sys


def fetch(path, match):
    vals = {}
    for r in csv.DictReader(open(path)):
        if match in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE":
            vals[int(r["Dispatch_Id"])] = (float(r["Counter_Value"]), r["Kernel_Name"])
    d = max(vals)
    return vals[d]


def main(mdir, pdir, config="c3"):
    kb, name = fetch(os.path.join(mdir, "pmc", "pmc_counter_collection.csv"), "k_mam_sm")
    ckb, _ = fetch(os.path.join(mdir, "calib", "pmc_counter_collection.csv"), "k_chase")
    loads = 16777216                       # tools/randbench calib: 262144 threads x 64
    per_probe = ckb * 1024 / loads
    scale = 64.0 / per_probe
    bench = json.load(open(os.path.join(mdir, "bench.json")))
    # the counted dispatch is the step's last batch: P - (nb - 1) * B pairs
    cfg = bench["config"]
    P, B, nb = cfg["pairs_per_rank"], cfg["batch_pairs"], cfg["batches_per_step"]
    reads_last = 2 * (P - (nb - 1) * B)
    out = {
        "k_mam_bytes_per_launch": int(round(kb * 1024 * scale)),
        "k_mam_bytes_per_read": round(kb * 1024 * scale / reads_last, 1),
        "reads_counted_dispatch": reads_last,
        "kernel": name.split("(")[0].replace("void smash::sm::", ""),
        "reads_per_launch": bench["roofline"]["reads_per_launch"],
        "fetch_size_kb": kb,
        "calibration": {
            "loads": loads, "fetch_size_kb": ckb,
            "bytes_counted_per_random_16B_probe": round(per_probe, 2),
            "note": "randbench calib: dependent random 16-byte loads over 64 GiB, one per "
                    "line; FETCH_SIZE counts 64 B per probe, so FETCH_SIZE is used as HBM "
                    "bytes (scaled by 64/counted)"},
        "source": os.path.join(pdir, "pmc_fetch_size_k_mam_sm.csv")
                  + " (rocprofv3 --pmc FETCH_SIZE, tools/measure_round.sh)",
    }
    json.dump(out, open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                     "profiles", "pmc_%s.json" % config), "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(*sys.argv[1:])
