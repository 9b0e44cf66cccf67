"""tools/isa_regions.py KERNEL.s MAM_SM_HPP -- static VALU / SALU of the
k_mam_sm loop attributed to its source regions (consume states, decide
blocks), through inlined-at chains: an instruction counts for the outermost
mam_sm.hpp line inside the kernel body.  Diagnostic tooling."""
import re
import sys
from collections import Counter

src = open(sys.argv[2]).read().split("\n")
marks = []
for i, l in enumerate(src, 1):
    m = re.search(r"case (S_[A-Z]+)|if \(a == (A_[A-Z_]+)\)|(// ---------------- decide)|(for \(;;\) \{)", l)
    if m:
        marks.append((i, next(g for g in m.groups() if g)))
body0 = next(i for i, n in marks if n.startswith("for"))
def region(line):
    r = "loop-top"
    for i, n in marks:
        if i <= line:
            r = n
    return r

valu, salu = Counter(), Counter()
cur = None
for line in open(sys.argv[1]):
    if ".loc\t" in line and "mam_sm.hpp" in line:
        # the chain: file:line entries in the comment, innermost first
        chain = [int(x) for x in re.findall(r"mam_sm\.hpp:(\d+):\d+", line)]
        outer = [x for x in chain if x >= body0]
        cur = outer[-1] if outer else (chain[-1] if chain else None)
        continue
    t = line.strip()
    if cur is None:
        continue
    if t.startswith("v_"):
        valu[region(cur)] += 1
    elif t.startswith("s_") and not t.startswith(("s_waitcnt", "s_nop", "s_cbranch", "s_branch")):
        salu[region(cur)] += 1
tot = sum(valu.values())
print("total VALU %d SALU %d" % (tot, sum(salu.values())))
for r, c in sorted(valu.items(), key=lambda x: -x[1]):
    print("%-28s VALU %5d  SALU %5d" % (r, c, salu[r]))
