"""tools/golden_queries.py -- query files derived from a committed
fastqs_to_sam golden (tests/golden/s*_fastqs_to_sam.sam.gz), written the same
way by tools/make_golden_r02.sh (to run the reference on them) and by the
tests (to run ours): FASTQ with Illumina '1:N:0' / '2:N:0' comments, FASTA
with ' 1' / ' 2' comments, or the first n SAM records.

  python tools/golden_queries.py SAM_GZ fastq|fasta|sam OUT [N_RECORDS]
"""
import gzip
import sys


def records(sam_gz, n=None):
    out = []
    for line in gzip.open(sam_gz):
        f = line.rstrip(b"\n").split(b"\t")
        out.append(f)
        if n is not None and len(out) >= n:
            break
    return out


def write(sam_gz, kind, path, n=None):
    recs = records(sam_gz, n)
    with open(path, "wb") as o:
        for f in recs:
            mate = b"1" if int(f[1]) & 64 else b"2"
            if kind == "fastq":
                o.write(b"@%s %s:N:0\n%s\n+\n%s\n" % (f[0], mate, f[9], f[10]))
            elif kind == "fasta":
                o.write(b">%s %s\n%s\n" % (f[0], mate, f[9]))
            elif kind == "sam":
                o.write(b"\t".join(f) + b"\n")
            else:
                raise ValueError(kind)
    return len(recs)


if __name__ == "__main__":
    write(sys.argv[1], sys.argv[2], sys.argv[3],
          int(sys.argv[4]) if len(sys.argv) > 4 else None)
