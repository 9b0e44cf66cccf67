"""tools/dist_phases.py [--world 8] [--per-rank 1000000] [--batches 3] -- the
multi-GPU step's phases per batch at W ranks, run as W threads of one
process on ONE device (tests/thread_ranks.py: the real dist.ShardedCounter
step, only the transport replaced by device copies), with
SMASH_DIST_TIMING=1 (each phase closed by a device synchronisation, so the
step's overlap is gone and the ranks share one GPU: the phase split, not the
8-GPU step time).  Prints the phase seconds per batch (max over ranks) and
the exchange volume per key: header words, hit words and the flag byte that
cross to other ranks.  Diagnostic tooling only."""
import argparse
import json
import os
import sys

os.environ["SMASH_DIST_TIMING"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("smash-paper_amd", "tools", "tests", ""):
    sys.path.insert(0, os.path.join(ROOT, p))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--per-rank", type=int, default=1_000_000)
    ap.add_argument("--batches", type=int, default=3)
    a = ap.parse_args()
    import tempfile
    import time

    import torch
    import bench
    import readgen
    import smashgpu as S
    import synth
    import thread_ranks as TR
    from dist import ShardedCounter

    cfg = dict(bench.CONFIGS["c3"])
    contigs = synth.make_genome(cfg["genome"])
    T, sp, sz, names = S.text_from_contigs(contigs)
    dix = S.Index.create(T, sp, sz, names)
    starts = bench.bin_starts_for(cfg, contigs, tempfile.mkdtemp())
    cs = bench.chrom_sizes_for(cfg, contigs)
    W, B, nb = a.world, a.per_rank, a.batches
    n = W * B * nb
    d_reads = readgen.Generator(dix, contigs, cfg["read_len"], seed=44).generate(n)
    print("[phases] %d ranks x %d pairs x %d batches, hg19, 150 bp" % (W, B, nb), flush=True)
    pipes, counts = TR.make_pipes(dix, W, cs, starts, cfg["read_len"], B, n + n // 8 + (1 << 20))
    scs = [None] * W

    def body(r, comm):
        sc = ShardedCounter(pipes[r], r, W, d_reads.device, comm=comm)
        scs[r] = sc
        sc.reset()
        for b in range(nb):
            lo = b * W * B + r * B
            sc.step(d_reads[2 * lo:2 * (lo + B)], B, b * W * B, counts[r])

    t0 = time.perf_counter()
    TR._run_threads(W, body)
    el = time.perf_counter() - t0
    phases = sorted({k for sc in scs for k in sc.timing})
    per = {k: round(max(sc.timing.get(k, 0.0) for sc in scs) / nb * 1e3, 3) for k in phases}
    keys = sum(sc.sent["keys"] for sc in scs)
    words = sum(sc.sent["words"] for sc in scs)
    rk = sum(sc.sent["remote_keys"] for sc in scs)
    rw = sum(sc.sent["remote_words"] for sc in scs)
    hdr_w = S.Pipeline.hdr_words
    out = {"world": W, "pairs_per_rank_per_batch": B, "batches": nb, "wall_s": round(el, 2),
           "phase_ms_per_batch_max_over_ranks": per,
           "keys_exported": keys, "words_per_key": round(words / max(keys, 1), 3),
           "remote_key_share": round(rk / max(keys, 1), 4),
           "bytes_per_key_on_links": round((rw * 8 + rk * (8 * hdr_w + 1)) / max(rk, 1), 2),
           "link_bytes_per_rank_per_batch": int((rw * 8 + rk * (8 * hdr_w + 1)) / (W * nb)),
           "note": "W threads on one GPU, device-copy transport, phases synchronised: the "
                   "split of a batch's time, not the 8-GPU step"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
