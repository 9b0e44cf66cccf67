"""tools/pmc_mem_json.py MEASURE_DIR PROFILE_DIR -- profiles/pmc_c3mem.json from
a FETCH_SIZE pass over `bench.py --config c3mem` (tools/r06_run.sh).

One MEM launch (smash_match_batch SMASH_MODE_MEM) is k_mem, then the wave
jobs k_job_slots / k_mem_jobs / k_mem_fix; FETCH_SIZE (kB) of every dispatch
of those kernels is summed and divided by the launches profiled (the bench's
warm-up launch and its timed ones), then rescaled with the randbench
calibration of the same box (64 B counted per random 16-byte probe, as
tools/pmc_to_json.py and MI355X_MICROARCH.md's HBM section prescribe).
bench.py reports the result as c3mem.roofline.traffic.
"""
import csv
import re
import json
import os
import sys


def main(mdir, pdir, reads=2_000_000):
    per_kernel, launches = {}, 0
    for r in csv.DictReader(open(os.path.join(mdir, "pmc_mem", "pmc_counter_collection.csv"))):
        if r["Counter_Name"] != "FETCH_SIZE":
            continue
        mk = re.search(r"\b(k_mem\w*|k_job\w*)", r["Kernel_Name"])
        if not mk:
            continue
        k = mk.group(1)
        per_kernel[k] = per_kernel.get(k, 0.0) + float(r["Counter_Value"])
        launches += k == "k_mem"
    ckb = None
    for r in csv.DictReader(open(os.path.join(mdir, "calib", "pmc_counter_collection.csv"))):
        if "k_chase" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE":
            ckb = float(r["Counter_Value"])
    loads = 16777216                       # tools/randbench calib: 262144 threads x 64
    per_probe = ckb * 1024 / loads
    scale = 64.0 / per_probe
    kb = sum(per_kernel.values()) / max(launches, 1)
    out = {
        "mem_bytes_per_launch": int(round(kb * 1024 * scale)),
        "mem_bytes_per_read": round(kb * 1024 * scale / reads, 1),
        "reads_per_launch": reads, "launches_profiled": launches,
        "fetch_size_kb_per_launch": {k: round(v / max(launches, 1), 1)
                                     for k, v in sorted(per_kernel.items())},
        "calibration": {"loads": loads, "fetch_size_kb": ckb,
                        "bytes_counted_per_random_16B_probe": round(per_probe, 2)},
        "note": "FETCH_SIZE rescaled with the random 16-byte probe calibration; k_mem_jobs streams SA "
                "ranges in rank order, and on gfx950 FETCH_SIZE reports half the bytes of wide "
                "coalesced streaming reads (MI355X_MICROARCH.md), so the HBM bytes of those "
                "reads may be up to 2x the figure; below the algorithmic line count, repeat "
                "families' SA ranges are shared by many reads of a launch (cache hits)",
        "source": os.path.join(pdir, "pmc_fetch_size_mem.csv")
                  + " (rocprofv3 --pmc FETCH_SIZE over bench.py --config c3mem, tools/r06_run.sh)",
    }
    json.dump(out, open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                     "profiles", "pmc_c3mem.json"), "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(*sys.argv[1:])
