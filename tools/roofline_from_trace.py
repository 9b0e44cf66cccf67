"""tools/roofline_from_trace.py TRACE.csv BENCH.json [skip] -- recompute the
bench line's roofline.frac from a committed rocprofv3 kernel trace of the
same command: reads_per_launch x bytes_per_read / the trace's average
k_mam_sm duration (skipping the first `skip` launches = the warm-up steps'),
against the 8 TB/s HBM peak.  Prints both figures so they can be compared."""
import csv
import json
import sys


def main(trace, bench, skip=None):
    b = json.load(open(bench))
    r = b["roofline"]
    rows = [x for x in csv.DictReader(open(trace)) if "k_mam_sm" in x["Kernel_Name"]]
    if skip is None:
        skip = len(rows) - r["launches"] if len(rows) > r["launches"] else 0
    iv = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"])) for x in rows[int(skip):])
    d = [(e - s) / 1e6 for s, e in iv]
    avg = sum(d) / len(d)

    def frac(ms):
        a = r["reads_per_launch"] * r["bytes_per_read"] / (ms / 1e3) / 1e9
        return a, a / r["peak"]
    ach, f = frac(avg)
    print("trace: %d launches, avg %.3f ms -> %.1f GB/s = %.4f of %.0f GB/s" %
          (len(d), avg, ach, f, r["peak"]))
    # launches on the two search streams can overlap (a batch's search starts
    # under the previous one's tail): those that overlap no other launch, and
    # the union of all launches per launch (the overlap counted once)
    alone = [(e - s) / 1e6 for k, (s, e) in enumerate(iv)
             if all(e2 <= s or s2 >= e for j, (s2, e2) in enumerate(iv) if j != k)]
    if alone:
        a_ms = sum(alone) / len(alone)
        print("trace, %d launches overlapping no other: avg %.3f ms -> %.1f GB/s = %.4f"
              % ((len(alone), a_ms) + frac(a_ms)))
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    tot += ce - cs
    u_ms = tot / 1e6 / len(iv)
    print("trace, union of the launches / launches: %.3f ms -> %.1f GB/s = %.4f"
          % ((u_ms,) + frac(u_ms)))
    print("bench: %d launches, avg %.3f ms -> %.1f GB/s = %.4f" %
          (r["launches"], r["avg_kernel_ms"], r["achieved"], r["frac"]))


if __name__ == "__main__":
    main(*sys.argv[1:])
