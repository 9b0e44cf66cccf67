"""tools/calib_cpu.py -- the CPU baseline's calibration (dev container only:
runs the compiled reference, oracle/_ref): the oracle's restatement, which
bench.py times on the GPU box as `cpu_baseline` (kind "port"), next to the
REFERENCE's own mummer on the same reads, BASELINE config C1's genome
(tools/synth.py "chr21", 32-bit index), at 1 and 8 cores.

  reference  mummer -verbose -rcref -qthreads Q -nomap -samin -samout (the
             smash_mapping.sh:19 line; Q = max(2, cores): -qthreads 1
             deadlocks), pinned with taskset to
             `cores` CPUs; reads/s = reads / (wall - wall of a 2-pair run),
             i.e. the index load and start-up taken out
  oracle     orc_map_only (the search alone, longSA::MAM restated) and
             orc_run_pairs (the whole chain: search, resolve, tag, smashMEM,
             varbin), `cores` threads, inside one pinned process

usage: python3 tools/calib_cpu.py [n_pairs] > profiles/rNN/cpu_calibration.log
"""
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [HERE, os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import oracle as O  # noqa: E402
import synth  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref")


def wall(cmd, cpus, cwd):
    t = time.perf_counter()
    subprocess.run(["taskset", "-c", cpus] + cmd, cwd=cwd, check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    return time.perf_counter() - t


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    W = "/tmp/calib_c1"
    os.makedirs(W, exist_ok=True)
    g = synth.make_genome("chr21")
    fa = os.path.join(W, "chr21.fa")
    if not os.path.exists(os.path.join(W, "chr21.fa.bin", "rc1.i4.index.sa.bin")):
        synth.write_fasta(fa, g)
        subprocess.run([os.path.join(REF, "mummer"), "-rcref", "chr21.fa", "dummy"], cwd=W,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    r1, r2 = synth.make_reads(g, n, 100, seed=1)
    for tag, k in (("big", n), ("tiny", 2)):
        synth.write_fastq(os.path.join(W, "r1.fq"), r1[:k], 1)
        synth.write_fastq(os.path.join(W, "r2.fq"), r2[:k], 2)
        with open(os.path.join(W, tag + ".sam"), "w") as f:
            subprocess.run([os.path.join(REF, "fastqs_to_sam"), "r1.fq", "r2.fq", "1"], cwd=W,
                           stdout=f, check=True)
    reads = np.empty((2 * n, 100), np.uint8)
    reads[0::2], reads[1::2] = r1, r2
    reads = np.frombuffer(O.lower_read(reads.tobytes()), np.uint8).reshape(2 * n, 100).copy()
    t = time.perf_counter()
    T, sp, sz, names = O.text_from_fasta(fa)
    oix = O.Index(T, sp, sz, names)
    oix.accel()
    print("# C1 genome %d bp, N = %d; oracle index (own suffix sort + accelerators) %.1f s; "
          "%d pairs = %d reads of 100 bp (SMASH reads, seed 1)"
          % (sum(len(s) for _, s in g), oix.N, time.perf_counter() - t, n, 2 * n))
    mp = oix.mappability()
    cs = {"chr21": 2781598825}
    starts = np.array([int(l.split("\t")[2]) for l in
                       open(os.path.join(ROOT, "data", "bins", "50000", "bins.txt"))], np.int64)
    print("cores\tref_mummer_reads_s\toracle_map_only_reads_s\toracle_whole_chain_reads_s\t"
          "ratio_map_only_vs_ref")
    for cores in (1, 8):
        cpus = "0" if cores == 1 else "0-%d" % (cores - 1)
        q = str(max(2, cores))
        cmd = lambda sam: [os.path.join(REF, "mummer"), "-verbose", "-rcref", "-qthreads", q,
                           "-nomap", "-samin", "-samout", "chr21.fa", sam]
        subprocess.run(["rm", "-rf", os.path.join(W, "mapout")])
        t0 = wall(cmd("tiny.sam"), cpus, W)
        subprocess.run(["rm", "-rf", os.path.join(W, "mapout")])
        t1 = wall(cmd("big.sam"), cpus, W)
        ref = 2 * n / max(t1 - t0, 1e-9)
        os.sched_setaffinity(0, set(range(cores)))
        t = time.perf_counter()
        O.map_only(oix, reads, threads=cores)
        om = 2 * n / (time.perf_counter() - t)
        op = O.Pipeline(oix, mp, cs, starts)
        t = time.perf_counter()
        assert op.run(reads, threads=cores) == 0
        oc = 2 * n / (time.perf_counter() - t)
        os.sched_setaffinity(0, set(range(os.cpu_count())))
        print("%d\t%.0f\t%.0f\t%.0f\t%.2f" % (cores, ref, om, oc, om / ref), flush=True)
        print("# reference: %.2f s for %d reads, %.2f s start-up (2-pair run), -qthreads %s"
              % (t1, 2 * n, t0, q), flush=True)


if __name__ == "__main__":
    main()
