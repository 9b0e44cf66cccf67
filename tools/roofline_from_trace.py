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
    d = [(int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e6 for x in rows[int(skip):]]
    avg = sum(d) / len(d)
    ach = r["reads_per_launch"] * r["bytes_per_read"] / (avg / 1e3) / 1e9
    print("trace: %d launches, avg %.3f ms -> %.1f GB/s = %.4f of %.0f GB/s" %
          (len(d), avg, ach, ach / r["peak"], r["peak"]))
    print("bench: %d launches, avg %.3f ms -> %.1f GB/s = %.4f" %
          (r["launches"], r["avg_kernel_ms"], r["achieved"], r["frac"]))


if __name__ == "__main__":
    main(*sys.argv[1:])
