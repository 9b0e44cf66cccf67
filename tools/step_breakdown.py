"""tools/step_breakdown.py TRACE.csv [warmup_launches] [launches_per_step] --
the timed steps of a `rocprofv3 --kernel-trace` bench run, kernel by kernel:
count, total / average / min duration per step, and the step time not
covered by any k_mam_sm launch (the post stage the search does not hide)."""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    if "onesweep" in n:
        return "radix_sort_onesweep_" + ("iteration" if "iteration" in n else "global_offsets")
    if "nccl" in n.lower() or "rccl" in n.lower():
        return "rccl_" + (re.search(r"(AllToAll|SendRecv|AllGather|AllReduce|Send|Recv)", n) or
                          re.search(r"(\w+)", n)).group(1)
    for k, v in (("scan_config", "rocprim_scan"), ("partition", "rocprim_partition"),
                 ("copyBuffer", "copyBuffer"), ("fillBuffer", "fillBuffer")):
        if k in n:
            return v
    m = re.search(r"(k_\w+(<[^>]*>)?)", n)
    return m.group(1) if m else n[:50]


def main(trace, warm=4, per_step=4):
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    mi = [i for i, r in enumerate(rows) if "k_mam_sm" in r["Kernel_Name"]]
    first, last = mi[int(warm)], mi[-1]
    t0 = int(rows[first]["Start_Timestamp"])
    # the step ends with the last batch's k_emit_bin (or k_bin) after the last search
    ends = [i for i in range(last, len(rows)) if short(rows[i]["Kernel_Name"]) in
            ("k_emit_bin", "k_emit_bin_lds", "k_bin", "k_tail_lps", "k_tail") and
            not any("copyBuffer" in rows[j]["Kernel_Name"] for j in range(last, i))]
    if not ends:   # (the sharded step: collectives' copies follow the last search)
        ends = [i for i in range(last, len(rows)) if short(rows[i]["Kernel_Name"]) in
                ("k_emit_bin", "k_emit_bin_lds", "k_bin")]
    end_i = max(ends)
    rs = rows[first:end_i + 1]
    t1 = max(int(r["End_Timestamp"]) for r in rs)
    steps = (len(mi) - int(warm)) / int(per_step)
    agg = defaultdict(lambda: [0, 0.0, 1e18])
    for r in rs:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        a = agg[short(r["Kernel_Name"])]
        a[0] += 1
        a[1] += d
        a[2] = min(a[2], d)
    print("%d timed steps, %.2f ms per step (first search start to last bin end)"
          % (steps, (t1 - t0) / 1e6 / steps))
    print("%-45s %6s %10s %9s %9s" % ("kernel", "calls", "ms/step", "avg ms", "min ms"))
    for k, (c, tot, mn) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print("%-45s %6d %10.2f %9.3f %9.3f" % (k, c, tot / steps, tot / c, mn))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rs
                if "k_mam_sm" in r["Kernel_Name"])
    u, (cs, ce) = 0, iv[0]
    for a, b in iv[1:]:
        if a > ce:
            u += ce - cs
            cs, ce = a, b
        else:
            ce = max(ce, b)
    u += ce - cs
    print("search union %.2f ms per step; not covered by a search: %.2f ms per step"
          % (u / 1e6 / steps, (t1 - t0 - u) / 1e6 / steps))
    # what runs in the uncovered time: per kernel, its overlap with the gaps
    # between search launches (kernels on other streams may overlap each other)
    merged, (cs, ce) = [], iv[0]
    for a, b in iv[1:]:
        if a > ce:
            merged.append((cs, ce))
            cs, ce = a, b
        else:
            ce = max(ce, b)
    merged.append((cs, ce))
    gaps = [(merged[i][1], merged[i + 1][0]) for i in range(len(merged) - 1)]
    gaps.append((merged[-1][1], t1))
    gap_k = defaultdict(float)
    busy = []
    for r in rs:
        if "k_mam_sm" in r["Kernel_Name"]:
            continue
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        for g0, g1 in gaps:
            o0, o1 = max(a, g0), min(b, g1)
            if o1 > o0:
                gap_k[short(r["Kernel_Name"])] += o1 - o0
                busy.append((o0, o1))
    busy.sort()
    bu = 0
    if busy:
        (cs, ce) = busy[0]
        for a, b in busy[1:]:
            if a > ce:
                bu += ce - cs
                cs, ce = a, b
            else:
                ce = max(ce, b)
        bu += ce - cs
    gap_total = sum(g1 - g0 for g0, g1 in gaps)
    print("uncovered time: %.2f ms per step in kernels, %.2f ms per step idle"
          % (bu / 1e6 / steps, (gap_total - bu) / 1e6 / steps))
    for k, t in sorted(gap_k.items(), key=lambda x: -x[1]):
        if t / 1e6 / steps >= 0.05:
            print("  %-43s %10.2f ms/step uncovered" % (k, t / 1e6 / steps))


if __name__ == "__main__":
    main(*sys.argv[1:])
