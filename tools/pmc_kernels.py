"""tools/pmc_kernels.py CSV... -- per kernel (short name) of rocprofv3 --pmc
runs: dispatches, mean duration (rocprofv3 serialises the dispatches of a
--pmc pass: isolated figures) and the mean of every counter per dispatch
(FETCH_SIZE / WRITE_SIZE in KB as rocprofv3 reports them; SQ counters raw)."""
import csv
import sys
from collections import defaultdict

from step_breakdown import short


def main(paths):
    disp = defaultdict(dict)   # kernel -> dispatch -> (dur, {counter: value})
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = short(r["Kernel_Name"])
            d = disp[k].setdefault((p, r["Dispatch_Id"]),
                                   [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6, {}])
            d[1][r["Counter_Name"]] = d[1].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    names = sorted({c for k in disp for d in disp[k].values() for c in d[1]})
    print("%-32s %5s %9s " % ("kernel", "n", "ms") + " ".join("%14s" % c for c in names))
    for k, ds in sorted(disp.items(), key=lambda x: -sum(d[0] for d in x[1].values())):
        n = len(ds)
        ms = sum(d[0] for d in ds.values()) / n
        row = []
        for c in names:
            v = [d[1][c] for d in ds.values() if c in d[1]]
            row.append("%14.4g" % (sum(v) / len(v)) if v else "%14s" % "-")
        print("%-32s %5d %9.3f " % (k[:32], n, ms) + " ".join(row))


if __name__ == "__main__":
    main(sys.argv[1:])
