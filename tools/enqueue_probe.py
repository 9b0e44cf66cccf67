"""tools/enqueue_probe.py -- does the host block while it queues a resident
run?  Times smash_count_batches' return (the host finished queueing every
batch) against the device finishing the run, at the bench's C3 batch size.
Diagnostic tooling."""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "smash-paper_amd"), os.path.join(ROOT, "tools"), ROOT):
    sys.path.insert(0, p)
import bench  # noqa: E402


def main():
    import torch
    import smashgpu as S
    import synth
    import readgen
    cfg = dict(bench.CONFIGS["c3"])
    contigs = synth.make_genome(cfg["genome"])
    T, sp, sz, names = S.text_from_contigs(contigs)
    dix = S.Index.create(T, sp, sz, names, device=0)
    starts = bench.bin_starts_for(cfg, contigs, tempfile.mkdtemp())
    cs = bench.chrom_sizes_for(cfg, contigs)
    P, B, L = 12_000_000, cfg["batch"], cfg["read_len"]
    d_reads = readgen.Generator(dix, contigs, L, seed=3).generate(P)
    pipe = S.Pipeline(dix, cs, starts, L, B, dedup_capacity=P)
    counts = torch.zeros(len(starts), dtype=torch.int64, device="cuda")
    for rep in range(3):
        pipe.reset(); counts.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pipe.count_batches(d_reads, P, B, counts)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print("[probe] %d pairs in %d-pair batches: host queued in %.1f ms, device done at %.1f ms"
              % (P, B, (t1 - t0) * 1e3, (t2 - t0) * 1e3), flush=True)


if __name__ == "__main__":
    main()
