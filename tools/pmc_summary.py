"""tools/pmc_summary.py DIR -- sum rocprofv3 --pmc counters per kernel dispatch.

Reads DIR/p*/pmc_counter_collection.csv (tools/profile_pmc.sh) and prints one
line per counter for the last dispatch of each kernel name, with its duration.
"""
import csv
import glob
import sys
from collections import defaultdict


def main(d):
    for f in sorted(glob.glob(f"{d}/p*/pmc_counter_collection.csv")):
        last = {}
        vals = defaultdict(float)
        meta = {}
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].split("(")[0]
            disp = int(row["Dispatch_Id"])
            if last.get(k, -1) < disp:
                last[k] = disp
                for key in [x for x in vals if x[0] == k]:
                    del vals[key]
            if disp == last[k]:
                vals[(k, row["Counter_Name"])] += float(row["Counter_Value"])
                meta[k] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"]),
                           row["Grid_Size"], row["VGPR_Count"])
        for (k, c), v in sorted(vals.items()):
            ns, grid, vgpr = meta[k]
            print(f"{f.split('/')[-2]} {k[-30:]:>30} {c:24s} {v:.4e}  (dur {ns/1e6:.1f} ms, grid {grid}, vgpr {vgpr})")


if __name__ == "__main__":
    main(sys.argv[1])
