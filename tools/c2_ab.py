"""tools/c2_ab.py BATCH... -- the C2 line (bench.c2_line: 1 M x 100 bp, 100 k
bins, 20 timed runs) on one hg19 index, once per batch size (pairs per
search launch), in one process"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("smash-paper_amd", "tools", "tools/sm_emu", "oracle", ""):
    sys.path.insert(0, os.path.join(ROOT, p))
import bench  # noqa: E402


class A:
    no_cpu_baseline = True


def main():
    import torch
    import smashgpu as S
    import synth
    contigs = synth.make_genome("hg19")
    T, sp, sz, names = S.text_from_contigs(contigs)
    dix = S.Index.create(T, sp, sz, names, device=0)
    dev = torch.device("cuda", 0)
    for b in [int(x) for x in sys.argv[1:]] * 2:
        r = bench.c2_line(A(), dix, contigs, dev, None, None, batch=b)
        print("[c2_ab] batch %7d: %.4e reads/s, %.3f ms per step" % (b, r["value"], r["ms_per_step"]),
              flush=True)


if __name__ == "__main__":
    main()
