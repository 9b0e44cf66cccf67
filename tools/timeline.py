"""tools/timeline.py TRACE.csv [first_search] [n_searches] -- the kernels of
a `rocprofv3 --kernel-trace` run around a stretch of k_mam_sm launches, in
start order, in ms from the first of them: start, end, duration, stream and
queue, so the gaps between consecutive searches can be read kernel by kernel
(which kernel ran when, beside or between the searches)."""
import csv
import sys

from step_breakdown import short


def main(trace, first=8, count=3):
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    mi = [i for i, r in enumerate(rows) if "k_mam_sm" in r["Kernel_Name"]]
    a = mi[int(first)]
    b = mi[min(len(mi) - 1, int(first) + int(count))]
    t0 = int(rows[a]["Start_Timestamp"])
    t_end = int(rows[b]["End_Timestamp"])
    print("%9s %9s %8s  %-6s %-5s %s" % ("start", "end", "ms", "stream", "queue", "kernel"))
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e < t0 or s > t_end:
            continue
        print("%9.3f %9.3f %8.3f  %-6s %-5s %s" % ((s - t0) / 1e6, (e - t0) / 1e6, (e - s) / 1e6,
                                                  r["Stream_Id"], r["Queue_Id"],
                                                  short(r["Kernel_Name"])))


if __name__ == "__main__":
    main(*sys.argv[1:])
