"""tools/c5_ab.py VARIANT... -- the C5 line (bench.c5_scan: U rebuilt from SA
+ L8, then the map.bin scan, hg19) on one index, once per variant per round
(2 rounds), in one process.  A variant is "name:ENV=VAL,ENV=VAL" (no "=":
the environment as it is), e.g. s25: s24:SMASH_UPART_S1=24"""
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
    for rnd in range(int(os.environ.get("ROUNDS", "2"))):
        for v in sys.argv[1:]:
            name, _, envs = v.partition(":")
            keys = []
            for kv in filter(None, envs.split(",")):
                k, _, val = kv.partition("=")
                os.environ[k] = val
                keys.append(k)
            r = bench.c5_scan(A(), dix, contigs, "50000", 1, 0, dev, None, None, reps=5)
            for k in keys:
                del os.environ[k]
            print("[c5_ab] %-10s round %d: prepare %.3f ms, scan %.3f ms, %.4e bases/s, map ok %s"
                  % (name, rnd, r["prepare_ms"], r["scan_ms"], r["value"],
                     r["map_identical_to_index_build"]), flush=True)
            print("[c5_ab]   per rep (device prepare, scan ms): %s; host (prepare, scan call ms): %s"
                  % (r["reps_ms"], r["reps_host_ms"]), flush=True)


if __name__ == "__main__":
    main()
