"""tagged mapout (reduced, from make_golden.sh) -> positions.txt.

Golden-generation helper: runs the oracle's smashMEM restatement
(oracle/smash_oracle.c:orc_smash_pair + the global de-dup set) over the
REFERENCE's own tagged SAM, then applies the awk/perl extraction of
smash_mapping.sh:29.  Records of one name are grouped like samtools sort -n
(fixed-width names: plain sort order), pysam fields per SURVEY.md §8c.

usage: oracle_positions.py ref.fa tagged.txt chrom_sizes.txt > positions.txt
"""
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import oracle as O  # noqa: E402

CIG = re.compile(r"(\d+)([SM=])")


def parse_hit(f, tid_of):
    """pysam 0.8 view of one mapped record of the reduced tagged file."""
    h = O.OrcHit()
    h.tid = tid_of[f[2]]
    h.rc = 1 if int(f[1]) & 16 else 0
    h.pos = int(f[3]) - 1
    ops = CIG.findall(f[5])
    rlen = sum(int(n) for n, _ in ops)
    lead = int(ops[0][0]) if ops[0][1] == "S" else 0
    trail = int(ops[-1][0]) if ops[-1][1] == "S" else 0
    h.qstart, h.qend = lead, rlen - trail
    tags = dict((t.split(":")[0], t.split(":")[2]) for t in f[9:])
    h.hi = int(tags["HI"])
    h.L0 = int(tags["L0"])
    h.R0 = int(tags["R0"])
    return h


def main():
    ref_fa, tagged, chrom_sizes = sys.argv[1:4]
    names = []
    with open(ref_fa) as fh:
        for line in fh:
            if line.startswith(">"):
                names.append(line[1:].split()[0])
    tid_of = {n: i for i, n in enumerate(names)}
    groups = {}
    order = []
    with open(tagged) as fh:
        for line in fh:
            f = line.rstrip("\n").split("\t")
            name, flag = f[0], int(f[1])
            if name not in groups:
                groups[name] = ([], [])
                order.append(name)
            if flag & 4:
                continue
            (groups[name][0] if flag & 64 else groups[name][1]).append(parse_hit(f, tid_of))
    rx = re.compile(r"^chr(\d+|[XY]) \d+$")
    seen = set()
    out = sys.stdout
    for name in sorted(order):
        h1, h2 = groups[name]
        h1.sort(key=lambda h: h.hi)
        h2.sort(key=lambda h: h.hi)
        kept = O.smash_pair(h1, h2)
        if kept is None:
            continue
        key = tuple(kept)
        if key in seen:
            continue
        seen.add(key)
        for tid, pos in kept:
            line = "%s %d" % (names[tid], pos)
            if rx.match(line):
                out.write(line + "\n")


if __name__ == "__main__":
    main()
