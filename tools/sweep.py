"""tools/sweep.py [--config c3] SETTING... -- A/B timing of the search kernel
under several environment settings in ONE process (the genome, the device
index and the reads are built once).

Each SETTING is a comma-separated list of VAR=VALUE (or "base" for none); for
each, the pipeline runs --steps timed steps and prints the k_mam_sm
milliseconds per launch, the step time and whether the bin counts equal the
first setting's (every setting must give identical counts).

  python tools/sweep.py base SMASH_SM_BLOCKS_PER_CU=4 SMASH_SM_BLOCKS_PER_CU=5
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "smash-paper_amd"), os.path.join(ROOT, "tools"), ROOT):
    sys.path.insert(0, p)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--pairs", type=int, default=2_000_000,
                    help="one batch of this many pairs (the A/B logs of round 2 use 2 M)")
    ap.add_argument("--batch", type=int, default=0,
                    help="run the --pairs as count_batches of this many pairs (the bench's "
                         "C3 step: --pairs 25000000 --batch 6250000)")
    ap.add_argument("--resident", action="store_true",
                    help="count_batches(resident=True) as bench.py's C3 step")
    ap.add_argument("settings", nargs="+")
    a = ap.parse_args()
    import tempfile

    import torch
    import smashgpu as S
    import synth
    cfg = dict(bench.CONFIGS[a.config])
    contigs = synth.make_genome(cfg["genome"])
    T, sp, sz, names = S.text_from_contigs(contigs)
    dix = S.Index.create(T, sp, sz, names, device=0)
    starts = bench.bin_starts_for(cfg, contigs, tempfile.mkdtemp())
    cs = bench.chrom_sizes_for(cfg, contigs)
    P, L = a.pairs, cfg["read_len"]           # one batch of the config's reads
    import readgen
    d_reads = readgen.Generator(dix, contigs, L, seed=cfg["seed"] * 1000).generate(P)
    B = a.batch or P
    pipe = S.Pipeline(dix, cs, starts, L, B, dedup_capacity=P + P // 8 + (1 << 20))
    counts = torch.zeros(len(starts), dtype=torch.int64, device="cuda")
    ref = None
    print("[sweep] ready: %d pairs x %d bp" % (P, L), flush=True)
    for setting in a.settings:
        env = {} if setting == "base" else dict(kv.split("=", 1) for kv in setting.split(","))
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        fresh = ("SMASH_POST", "SMASH_BIN", "SMASH_FUSED", "SMASH_KEY", "SMASH_GATE",
                 "SMASH_ONE", "SMASH_PRIO", "SMASH_PREP_ALL")   # read at create
        if any(k.startswith(fresh) for k in env) or pipe is None:
            pipe = None                      # read at create: a fresh pipeline
            pipe = S.Pipeline(dix, cs, starts, L, B, dedup_capacity=P + P // 8 + (1 << 20))

        def run():
            pipe.reset(); counts.zero_()
            if a.batch:
                pipe.count_batches(d_reads, P, B, counts, resident=a.resident)
            else:
                pipe.count_batch(d_reads, P, counts)
        run()   # warm-up
        torch.cuda.synchronize()
        pipe.profile(True)
        t = time.perf_counter()
        for _ in range(a.steps):
            run()
        torch.cuda.synchronize()
        el = (time.perf_counter() - t) / a.steps
        ms, launches, _ = pipe.profile_read()
        pipe.profile(False)
        c = counts.cpu().numpy().copy()
        if ref is None:
            ref = c
        st = pipe.stats()
        print("[sweep] %-50s k_mam %.2f ms  step %.2f ms  %.3e reads/s  same_counts %s err %d"
              % (setting, ms / max(launches, 1), el * 1e3, 2 * P / el,
                 bool(np.array_equal(c, ref)), st.error), flush=True)
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        if any(k.startswith(fresh) for k in env):
            pipe = None


if __name__ == "__main__":
    main()
