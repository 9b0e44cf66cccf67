"""tools/smashmem_edge.py -- a hand-made, name-sorted, mappability-tagged SAM
(test DATA for tools/make_golden_smashmem.sh) that walks smashMEM.py's
branches (smashMEM.py:76-92,154-228):
the excess filter at qlen - max(L0, R0) = 3 / 4, the read-2 hit window
(same tid and |pos1 - pos2| < 10000, strict), the key in HI order (not file
order), r1 and r2 hits not separated in the key, first-wins de-dup, pairs with
nothing kept, unmapped mates, reverse strands with soft clips on both ends,
merged CIGARs with M gaps (qlen counts them), small contigs.
usage: python3 tools/smashmem_edge.py > smashmem_edge.sam"""
import sys

HEAD = ["@HD\tVN:1.0\tSO:unsorted", "@PG\tID:longMEM\tPN:longMEM\tVN:0.5",
        "@SQ\tSN:chr1\tLN:120000", "@SQ\tSN:chr1_gl000191_random\tLN:40000",
        "@SQ\tSN:chr2\tLN:90000", "@SQ\tSN:chrM\tLN:16571", "@SQ\tSN:chrX\tLN:60000"]
L = 100
SEQ = ("ACGT" * 25)[:L]
QUAL = "I" * L


def rec(name, mate, chrom=None, pos=0, cigar=None, hi=0, nh=1, L0=0, R0=0, rev=False):
    """one record; chrom None: the unmapped line -nomap prints"""
    flag = (64 if mate == 1 else 128) | 1
    if chrom is None:
        return "\t".join([name, str(flag | 4), "*", "0", "0", "*", "*", "0", "0", SEQ, QUAL])
    flag |= (16 if rev else 0) | (256 if hi else 0)
    return "\t".join([name, str(flag), chrom, str(pos), "50", cigar, "*", "0", "0", SEQ, QUAL,
                      "XM:i:1", "XU:i:30", "XE:i:40", "XS:A:+", "NH:i:%d" % nh, "HI:i:%d" % hi,
                      "L0:i:%d" % L0, "R0:i:%d" % R0])


def main():
    out = list(HEAD)
    n = [0]

    def pair(r1, r2):
        name = "e%06d" % n[0]
        n[0] += 1
        for m, hits in ((1, r1), (2, r2)):
            if not hits:
                out.append(rec(name, m))
            for h in hits:
                out.append(rec(name, m, **h))
    H = lambda chrom, pos, cigar, hi, **k: dict(chrom=chrom, pos=pos, cigar=cigar, hi=hi, **k)
    # excess filter: qlen 30, max(L0, R0) 27 -> 3 (dropped), 26 -> 4 (kept)
    pair([H("chr1", 1000, "30=70S", 0, L0=27, R0=5), H("chr1", 5000, "30S30=40S", 1, L0=3, R0=26)],
         [H("chr2", 700, "50S50=", 0, L0=10, R0=10)])
    # read-2 window: 9999 away (dropped), 10000 away (kept), same pos on another chrom (kept)
    pair([H("chr1", 20000, "40=60S", 0)],
         [H("chr1", 29999, "40S40=20S", 0), H("chr1", 30000, "60S40=", 1), H("chr2", 20000, "40=60S", 2)])
    # key in HI order, records in file order HI 2, 0, 1; a reverse hit with clips on both ends
    pair([H("chr2", 300, "20S30=50S", 2), H("chr1", 40000, "30=70S", 0, rev=True),
          H("chrX", 9, "70S30=", 1)], [])
    # the same key again, its hits in another file order: a duplicate
    pair([H("chr1", 40000, "30=70S", 0, rev=True), H("chrX", 9, "70S30=", 1),
          H("chr2", 300, "20S30=50S", 2)], [])
    # the same (tid, pos) list split r1 / r2 differently: the key does not
    # separate the mates, so this is a duplicate of the pair above too
    pair([H("chr1", 40000, "30=70S", 0, rev=True), H("chrX", 9, "70S30=", 1)],
         [H("chr2", 300, "20S30=50S", 0)])
    # nothing survives the filters: neither counted nor a key
    pair([H("chr1", 60000, "25=75S", 0, L0=22, R0=22)], [])
    # read 1 unmapped, read 2 mapped (key from read 2 alone), twice: 2nd a dupe
    pair([], [H("chr2", 80000, "35S35=30S", 0)])
    pair([], [H("chr2", 80000, "35S35=30S", 0)])
    # a merged diagonal (M gap counted in qlen: 10S + 20= 5M 20= + 45S -> 45)
    pair([H("chr1", 90000, "10S20=5M20=45S", 0, L0=40, R0=30)], [H("chr1", 110000, "45=55S", 0)])
    # small contigs (filters apply; the extraction step drops them later)
    pair([H("chrM", 100, "40=60S", 0), H("chr1_gl000191_random", 200, "60S40=", 1)], [])
    # read 2 near a read-1 hit that the excess filter dropped: not a window hit
    pair([H("chr1", 70000, "30=70S", 0, L0=28, R0=0), H("chrX", 500, "30S30=40S", 1)],
         [H("chr1", 70100, "50S50=", 0)])
    # a reverse read-2 hit inside the window of a reverse read-1 hit
    pair([H("chr2", 50000, "50=50S", 0, rev=True)], [H("chr2", 41000, "50S50=", 0, rev=True)])
    # both mates unmapped
    pair([], [])
    sys.stdout.write("\n".join(out) + "\n")


if __name__ == "__main__":
    main()
