"""tools/tail_probe.py -- does a k_mam_sm launch pay a tail?  Times
smash_map_batch (MAM, the search alone) on the first n reads of one set of
hg19-shaped SMASH reads for several n: with a fixed per-launch tail (the
slowest reads still running when the work queue empties), the time per read
falls as n grows.  Diagnostic tooling (GPU)."""
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
    L = cfg["read_len"]
    pairs = 4_000_000
    d_reads = readgen.Generator(dix, contigs, L, seed=cfg["seed"] * 1000).generate(pairs)
    cap = L - 20 + 1
    n_max = 2 * pairs
    d_out = torch.empty(n_max * cap, dtype=torch.int64, device="cuda")
    d_n = torch.empty(n_max, dtype=torch.int32, device="cuda")
    print("[tail] ready: %d reads" % n_max, flush=True)
    for n in (250_000, 500_000, 1_000_000, 2_000_000, 4_000_000, 8_000_000):
        S.map_batch(dix, d_reads, n, L, d_out, cap, d_n)
        torch.cuda.synchronize()
        reps = max(2, 8_000_000 // n)
        t = time.perf_counter()
        for _ in range(reps):
            S.map_batch(dix, d_reads, n, L, d_out, cap, d_n)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / reps
        print("[tail] n %8d reads: %.3f ms per launch, %.3f ns per read" % (n, dt * 1e3, dt / n * 1e9),
              flush=True)


if __name__ == "__main__":
    main()
