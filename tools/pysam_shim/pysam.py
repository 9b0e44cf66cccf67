"""tools/pysam_shim/pysam.py -- a SAM-text stand-in for the part of pysam
0.8 that the reference's smashMEM.py calls (test tooling: golden generation
in the dev container only; never imported by the product).

smashMEM.py (smashMEM.py:9-56,154-230) uses pysam.Samfile(path, 'rb') as an
iterator with reset() / getrname(tid) / close(), and these read fields:
qname, is_read1, is_read2, is_reverse, is_unmapped, qlen, qstart, qend,
rlen, pos, tid, opt(tag).  Here the file is SAM TEXT (the 'rb' mode is
ignored) and the fields follow pysam 0.8's AlignedRead semantics as
SURVEY.md section 8c restates them:
  pos    = POS - 1                   tid = index of RNAME among the @SQ lines
  rlen   = len(SEQ)                  qstart = leading soft clip
  qend   = rlen - trailing soft clip qlen = qend - qstart (M gap bases included)
  opt(t) = the tag's value: int for type i, the text for Z and A.
The accessors are restated, not pysam's code: this pins smashMEM.py's own
control flow (grouping, filters, hit window, key, first-wins) to its text.
"""
import re

_CIG = re.compile(r"(\d+)([MIDNSHP=X])")


class AlignedRead(object):
    __slots__ = ("qname", "flag", "tid", "pos", "rlen", "qstart", "qend", "_tags")

    def __init__(self, f, tid_of):
        self.qname = f[0]
        self.flag = int(f[1])
        self.tid = tid_of.get(f[2], -1) if f[2] != "*" else -1
        self.pos = int(f[3]) - 1
        self.rlen = len(f[9]) if f[9] != "*" else 0
        ops = _CIG.findall(f[5]) if f[5] != "*" else []
        lead = int(ops[0][0]) if ops and ops[0][1] == "S" else 0
        trail = int(ops[-1][0]) if len(ops) > 1 and ops[-1][1] == "S" else 0
        self.qstart = lead
        self.qend = self.rlen - trail
        self._tags = {}
        for t in f[11:]:
            name, typ, val = t.split(":", 2)
            self._tags[name] = int(val) if typ == "i" else val

    is_read1 = property(lambda self: bool(self.flag & 64))
    is_read2 = property(lambda self: bool(self.flag & 128))
    is_reverse = property(lambda self: bool(self.flag & 16))
    is_unmapped = property(lambda self: bool(self.flag & 4))
    qlen = property(lambda self: self.qend - self.qstart)

    def opt(self, tag):
        return self._tags[tag]


class Samfile(object):
    def __init__(self, path, mode="r"):
        self._names = []
        self._body = []
        with open(path) as fh:
            for line in fh:
                line = line.rstrip("\n")
                if line.startswith("@"):
                    if line.startswith("@SQ"):
                        sn = [x for x in line.split("\t") if x.startswith("SN:")][0]
                        self._names.append(sn[3:])
                    continue
                if line:
                    self._body.append(line)
        self._tid = {n: i for i, n in enumerate(self._names)}
        self._i = 0

    def __iter__(self):
        return self

    def __next__(self):
        if self._i >= len(self._body):
            raise StopIteration
        rec = AlignedRead(self._body[self._i].split("\t"), self._tid)
        self._i += 1
        return rec

    next = __next__

    def reset(self):
        self._i = 0

    def getrname(self, tid):
        return self._names[tid]

    def close(self):
        pass
