"""tools/c5_waves.py -- A/B of k_mapscan's register budget on one index in
one process: SMASH_MAPSCAN_WAVES = 0 (the compiler's choice), 4, 5, 6 waves
per SIMD (W:SUB also sets SMASH_MAPSCAN_SUB), each scanned `reps` times (C5: hg19, k = 36, 50 000 bins); every
variant's map.bin must equal the index build's and its counts the first
variant's.  Prints one JSON line per variant."""
import json
import os
import sys
import types

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "smash-paper_amd"), os.path.join(R, "tools")]


def main():
    import torch
    import bench
    import smashgpu as S
    import synth
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    variants = sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "4", "5", "6", "0"]
    contigs = synth.make_genome("hg19")
    T, sp, sz, names = S.text_from_contigs(contigs)
    dix = S.Index.create(T, sp, sz, names, device=0)
    dev = torch.device("cuda", 0)
    args = types.SimpleNamespace(no_cpu_baseline=True)
    ref = None
    for v in variants:
        w, _, sub = v.partition(":")   # "5n:2": SMASH_MAPSCAN_SUB=2
        os.environ["SMASH_MAPSCAN_WAVES"] = w
        os.environ["SMASH_MAPSCAN_SUB"] = sub
        r = bench.c5_scan(args, dix, contigs, "50000", 1, 0, dev, None, None, reps=reps)
        key = (r["unique_kmers"], r["map_identical_to_index_build"])
        ref = ref or key
        print(json.dumps({"waves": v, "ms_per_scan": round(r["ms_per_scan"], 3),
                          "avg_kernel_ms": r["roofline"]["avg_kernel_ms"],
                          "frac": r["roofline"]["frac"], "unique": r["unique_kmers"],
                          "map_identical": r["map_identical_to_index_build"],
                          "same_as_first": key == ref}), flush=True)


if __name__ == "__main__":
    main()
