"""tools/prof_top.py DB [N] -- per-kernel summary (calls, total ms, average
us, share) of a rocprofv3 --kernel-trace --stats run written as its rocpd
SQLite database (durations there in us); kernel names cut at the first '('."""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
rows = db.execute("select name, total_calls, total_duration, average, percentage "
                  "from top_kernels limit ?", (n,)).fetchall()
print("%-60s %7s %11s %11s %6s" % ("kernel", "calls", "total ms", "avg us", "%"))
for name, calls, tot, avg, pct in rows:
    short = name.replace("(anonymous namespace)::", "").replace("smash::", "")
    if short.startswith("void "):
        short = short[5:]
    short = short.split("(")[0]
    if "rocprim" in short:
        short = "rocprim::" + ("radix_sort" if "radix_sort" in name else "partition" if "partition" in name
                               else "scan" if "scan" in name else "other")
    print("%-60s %7d %11.3f %11.1f %6.2f" % (short[-60:], calls, tot / 1e3, avg, pct))
