#!/usr/bin/env python
"""bench.py -- reads/s mapped + binned on MI355X (BASELINE.json metric).

Workload (default --config c3, BASELINE.json configs[2], the 1-GPU
configuration its metric is quoted on: "hg19, 50M synthetic 150 bp reads,
1xMI355X, sample_bins/50000"): the hg19-shaped synthetic genome
(tools/synth.py: hg19 contig lengths, N runs over the assembly gaps,
repeats; 3.1 Gbp, doubled text N = 6.19e9, 64-bit SA/ISA) is indexed ON THE
DEVICE and kept resident in HBM; each rank's 25 M synthetic 150 bp SMASH
read pairs (50 M reads, 7.5 GB; generated on the device by tools/readgen.hip)
are resident in HBM before the timed region.  One step = one complete run of
the hot path over those 50 M reads, as the reference scripts run one sample:
13 batches of <= 2 M pairs through MAM search -> resolve -> mappability tag
-> smashMEM filters -> global first-wins pair de-dup (one 25 M-key set for
the whole run) -> varbin adjacent de-dup (carried across batches) -> bin
counts; with N ranks each rank runs its own 25 M pairs (400 M reads at N = 8
is BASELINE config C4) plus the de-dup all_to_all, the tail all_gather and
the RCCL all_reduce of the count vector.  value = reads processed by all
ranks / max-over-ranks wall time of the K timed steps.

Also reported: `roofline` of the dominant kernel (k_mam_sm: algorithmic bytes
= 64 B x the line transitions of the kernel's own probe sequence, counted by
running the kernel source on the host (tools/sm_emu) over the downloaded index
for a sample of the same reads, over the HIP-event-timed kernel duration),
`cpu_baseline` (the C oracle of the whole chain and of the search alone, on
all the host CPUs the box grants (its cgroup quota = nproc), rank 0, N = 1,
bounded sample of the same
reads; the device's counts on that sample must be identical) and `c5`
(BASELINE config C5 on the same resident index: the map.bin self-scan of
every forward base with unique-36-mer counts, bases/s, its roofline and a CPU
baseline).
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in ("smash-paper_amd", "tools", "tools/sm_emu", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, _p))

import numpy as np  # noqa: E402

METRIC = ("reads/sec mapped+binned (hg19, 150 bp) at 1/2/4/8 MI355X; "
          "bit-exact bin counts")

CONFIGS = {
    # BASELINE.json configs[2]: hg19, 50 M x 150 bp, sample_bins/50000 (the
    # metric's config); configs[3] (C4) is this at N = 8: 400 M reads
    "c3": dict(genome="hg19", read_len=150, pairs=25_000_000, batch=12_500_000, bins="50000",
               seed=3, workload="C3 hg19-shaped, 50 M x 150 bp SMASH reads per rank "
                                "(25 M pairs, one run in batches), sample_bins/50000"),
    # configs[1]: hg19 1M x 100 bp, sample_bins/100000 (synthesized 2-way split)
    "c2": dict(genome="hg19", read_len=100, pairs=500_000, batch=500_000, bins="100000", seed=2,
               workload="C2 hg19-shaped 1M x 100 bp SMASH reads, sample_bins/100000"),
    # configs[0]-like plumbing on the chr21-sized genome (bins split 10-way)
    "c1": dict(genome="chr21", read_len=100, pairs=5_000, batch=5_000, bins="500000", seed=1,
               workload="C1 chr21-sized genome, 10 k x 100 bp, sample_bins/500000"),
    # configs[4]: whole-genome mappability self-scan (every 36-mer), C5
    "c5": dict(genome="hg19", bins="50000", k=36,
               workload="C5 hg19-shaped mappability self-scan (map.bin + unique 36-mer "
                        "counts per chromosome and per 50 k bin)"),
    # -maxmatch (longSA::findMEM) on C3's reads: the search mode north_star
    # names beside MAM, timed alone (not on the SMASH path)
    "c3mem": dict(genome="hg19", read_len=150, pairs=1_000_000, bins="50000", seed=3, cap=512,
                  workload="MEM (memsam -maxmatch, longSA::findMEM) of C3's 150 bp SMASH reads "
                           "on hg19, 2 M reads per launch"),
    # quick functional run
    "mid": dict(genome="mid", read_len=150, pairs=200_000, batch=200_000, bins="synthetic",
                seed=2, workload="3.2 Mbp synthetic genome, 150 bp (functional check)"),
}


def host_cores():
    """The host CPUs this process may use: the cgroup CPU quota when one is
    set (the GPU box: 16 of the node's os.cpu_count() = 256, what `nproc`
    reports there), else the affinity mask.  Returns (cores, note)."""
    cpus = os.cpu_count() or 1
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = max(1, -(-int(q) // int(p)))
            return n, "cgroup cpu.max %s/%s = %d CPUs (nproc); os.cpu_count() = %d" % (q, p, n, cpus)
    except (OSError, ValueError):
        pass
    try:
        n = len(os.sched_getaffinity(0))
        return n, "affinity %d CPUs; os.cpu_count() = %d" % (n, cpus)
    except AttributeError:
        return cpus, "os.cpu_count() = %d" % cpus


def log(*a):
    print("[bench %s]" % time.strftime("%H:%M:%S"), *a, file=sys.stderr, flush=True)


def chrom_sizes_of(contigs):
    out, n = {}, 0
    for name, s in contigs:
        if "_" in name:
            continue
        out[name] = n
        n += len(s)
    return out


def bin_starts_for(cfg, contigs, tmpdir):
    import synth
    src = os.path.join(ROOT, "data", "bins", "50000", "bins.txt")
    if cfg["bins"] == "50000":
        path = src
    elif cfg["bins"] in ("100000", "500000"):
        path = os.path.join(tmpdir, "bins_%s.txt" % cfg["bins"])
        synth.split_bins(src, 2 if cfg["bins"] == "100000" else 10, path)
    else:
        path = os.path.join(tmpdir, "bins_syn.txt")
        synth.make_bins(contigs, 64, path)
    return np.array([int(l.split("\t")[2]) for l in open(path)], np.int64)


def chrom_sizes_for(cfg, contigs):
    cs = chrom_sizes_of(contigs)
    if cfg["genome"] == "chr21":    # hg19 offset so that hg19 bins apply (§8d C1)
        cs = {"chr21": 2781598825}
    return cs


def make_reads(contigs, cfg, n_pairs, seed):
    import smashgpu as S
    import synth
    r1, r2 = synth.make_reads(contigs, n_pairs, cfg["read_len"], seed=seed)
    reads = np.empty((2 * n_pairs, cfg["read_len"]), np.uint8)
    reads[0::2] = r1
    reads[1::2] = r2
    return S.prepare_reads(reads)


def kmer_codes(reads, K):
    """Distinct 2-bit codes of the all-ACGT K-mers of the reads (host)."""
    lut = np.full(256, -1, np.int64)
    for i, ch in enumerate(b"acgt"):
        lut[ch] = i
    a = lut[np.asarray(reads, np.uint8)]
    if a.shape[1] < K:
        return np.zeros(0, np.uint64)
    w = np.lib.stride_tricks.sliding_window_view(a, K, axis=1)
    ok = (w >= 0).all(axis=2)
    code = np.zeros(w.shape[:2], np.uint64)
    for k in range(K):
        code = (code << np.uint64(2)) | np.where(w[:, :, k] >= 0, w[:, :, k], 0).astype(np.uint64)
    return np.unique(code[ok])


def host_index(S, O, dix, T, sp, sz, names, sample_reads=None):
    """Download the device index into the oracle's host layout (cpu leg).
    The k-mer table (4^K x 16 B, 69 GB at K = 16) is not copied: a lazily
    committed zero array gets only the entries of sample_reads' k-mers
    (what the host emulation of the kernel looks up)."""
    i = dix.info
    N = i.N
    # SA / ISA as the device holds them: with packed index words (hg19) the
    # oracle reads their element bits (pos_mask), the emulation of k_mam_sm
    # their hints too
    SA, ISA = dix.download_sa_isa(plain=False)
    L8 = S.download(i.d_lcp8, N)
    ovf = S.download(i.d_lcp_ovf, 16 * i.n_lcp_overflow, np.uint64).reshape(-1, 2)
    mp = S.download(i.d_map, i.map_bytes)
    oix = O.Index(T, sp, sz, names, SA=SA, ISA=ISA, L8=L8, ovf=ovf,
                  pos_mask=dix.pos_mask if i.pos_bits else None)
    U = S.download(i.d_uniq, N + 64)
    KT = np.zeros(2 << (2 * i.kmer_k), np.uint64)          # calloc: pages on first touch
    if sample_reads is not None:
        import torch
        codes = kmer_codes(sample_reads, i.kmer_k)
        if len(codes):
            kt_dev = S.device_view(i.d_kmer, 16 << (2 * i.kmer_k), torch.int64).view(-1, 2)
            idx = torch.from_numpy(codes.astype(np.int64)).to(kt_dev.device)
            got = kt_dev.index_select(0, idx).cpu().numpy().view(np.uint64)
            KT.reshape(-1, 2)[codes.astype(np.int64)] = got
    # (the window filter's presence bits ride in the k-mer entries: KT is
    # the device layout, which the emulation reads as is; no bitmap)
    it = np.array([(i.in_text[c >> 6] >> (c & 63)) & 1 for c in range(256)], np.uint8)
    oix.accel(U, KT, i.kmer_k, np.zeros(1, np.uint64), i.bitmap_b, it, KTF=KT)
    return oix, mp


def add_sample_kmers(S, dix, oix, reads):
    """copy the device k-mer entries of `reads`' k-mers into the host table
    host_index left lazily committed (oix holds that array, not a copy), so
    the host emulation and the oracle's k-mer descents can run on them"""
    import torch
    K = dix.info.kmer_k
    codes = kmer_codes(reads, K)
    if len(codes):
        kt_dev = S.device_view(dix.info.d_kmer, 16 << (2 * K), torch.int64).view(-1, 2)
        idx = torch.from_numpy(codes.astype(np.int64)).to(kt_dev.device)
        oix._KT.reshape(-1, 2)[codes.astype(np.int64)] = \
            kt_dev.index_select(0, idx).cpu().numpy().view(np.uint64)


def search_lines(S, dix, oix, sample):
    """k_mam_sm's probe sequence over `sample` on the host (tools/sm_emu, the
    kernel's own source, one lane): (emulator, iterations per read, lines)"""
    import sm_emu
    add_sample_kmers(S, dix, oix, sample)
    emu = sm_emu.Emu(oix, copy=False, packed=bool(dix.info.pos_bits))
    _, emu_it = emu.map(sample)
    return emu, emu_it, sum(v[1] for v in emu.counters.values())


def c2_line(args, dix, contigs, dev, oix, mp, steps=20, warmup=3, batch=None):
    """BASELINE configs[1] (C2) on the resident hg19 index: 1 M x 100 bp SMASH
    reads (500 k pairs, one batch) through the whole chain into
    sample_bins/100000; the GEO 100 search kernel (mam.hip run_sm).  Roofline
    from the emulated probe sequence of a sample of its reads; the oracle runs
    the whole C2 workload on the host's cores (cpu_baseline) and its counts
    must equal the device's."""
    import torch
    import smashgpu as S
    import readgen
    cfg = CONFIGS["c2"]
    starts = bin_starts_for(cfg, contigs, tempfile.mkdtemp())
    cs = chrom_sizes_for(cfg, contigs)
    P, L = cfg["pairs"], cfg["read_len"]
    d_reads = S.to_rows(readgen.Generator(dix, contigs, L, seed=cfg["seed"] * 1000).generate(P), L)
    # (batch: the pairs per search launch; smaller batches let a launch's
    # tail overlap the next one's start on the other search stream)
    B = batch or int(os.environ.get("SMASH_C2_BATCH", "0")) or P
    pipe = S.Pipeline(dix, cs, starts, L, B, dedup_capacity=P + P // 8 + (1 << 20),
                      read_stride=d_reads.shape[1])
    counts = torch.zeros(len(starts), dtype=torch.int64, device=dev)

    def step():
        counts.zero_()
        pipe.reset()
        pipe.count_batches(d_reads, P, B, counts, resident=True)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    ref = counts.cpu().numpy().copy()
    pipe.profile(True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t1
    mam_ms, launches, mam_reads = pipe.profile_read()
    pipe.profile(False)
    st = pipe.stats()
    dev_counts = counts.cpu().numpy()
    value = 2 * P * steps / el
    avg_ms = mam_ms / max(launches, 1)
    res = {"metric": "reads/sec mapped+binned (hg19, 100 bp, C2)", "value": value,
           "unit": "reads/s", "ms_per_step": 1000.0 * el / steps, "steps": steps,
           "warmup": warmup, "workload": cfg["workload"], "pairs": P, "read_len": L,
           "bins": int(len(starts)), "batch_pairs": B,
           "search_kernel": "k_mam_sm GEO 100" if dix.info.pos_bits else "k_mam_sm",
           "deterministic_counts": bool(np.array_equal(dev_counts, ref)),
           "stats": st.as_dict(), "roofline": None, "cpu_baseline": None}
    log("C2: %d steps %.3f s -> %.3e reads/s, %.3f ms per step, k_mam %.3f ms per launch"
        % (steps, el, value, 1000.0 * el / steps, avg_ms))
    if oix is not None:
        import oracle as O
        ns = min(4000, 2 * P)
        sample = d_reads[:ns, :L].contiguous().cpu().numpy()
        emu, emu_it, lines = search_lines(S, dix, oix, sample)
        b_read = 64.0 * lines / ns
        rpl = mam_reads / max(launches, 1)
        achieved = rpl * b_read / (avg_ms / 1e3) / 1e9
        res["roofline"] = {
            "bound": "hbm", "kernel": "k_mam_sm", "achieved": round(achieved, 2), "peak": 8000.0,
            "unit": "GB/s", "frac": round(achieved / 8000.0, 5), "traffic": None,
            "bytes_per_read": round(b_read, 1), "avg_kernel_ms": round(avg_ms, 3),
            "reads_per_launch": int(rpl),
            "lines_per_read": {k: round(v[1] / ns, 3) for k, v in emu.counters.items()},
            "loop_iterations_per_read": round(float(emu_it.mean()), 1),
            "requests_per_read": round(emu.requests[0] / ns, 2),
            "bytes_method": "64 B x line transitions of the kernel's probe sequence (tools/sm_emu "
                            "on the downloaded index, %d reads)" % ns}
        if not args.no_cpu_baseline:
            # the whole C2 workload through the oracle's chain (~8 s on 16
            # threads): its counts against the device's
            threads, note = host_cores()
            h = d_reads[:2 * P, :L].contiguous().cpu().numpy()
            op = O.Pipeline(oix, mp, cs, starts)
            t3 = time.perf_counter()
            err = op.run(h, threads=threads)
            dt = time.perf_counter() - t3
            exact = bool(err == 0 and np.array_equal(dev_counts.astype(np.uint64), op.counts))
            res["cpu_baseline"] = {
                "value": 2 * P / dt, "unit": "reads/s", "cores": threads, "kind": "port",
                "sample": "the whole C2 workload, %d pairs (%d reads), whole chain "
                          "(oracle/smash_oracle.c orc_run_pairs, %d threads), %.1f s"
                          % (P, 2 * P, threads, dt),
                "cores_note": note}
            res["bin_counts_identical_to_oracle"] = exact
            log("C2 cpu baseline: %.3e reads/s on %d threads; counts == oracle: %s"
                % (2 * P / dt, threads, exact))
    pipe.close()
    del d_reads
    torch.cuda.empty_cache()
    return res


def c5_scan(args, dix, contigs, cfg_bins, world, rank, dev, dist, oix=None, reps=3):
    """C5 on the resident index: map.bin bytes of every forward base (longSA::
    show) + unique 36-mer counts per contig and per bin, bases split into
    `world` contiguous ranges, counts all-reduced.  Returns (json, per-rep s)."""
    import torch
    import smashgpu as S
    starts = bin_starts_for(dict(bins=cfg_bins), contigs, tempfile.mkdtemp())
    cs = chrom_sizes_of(contigs)
    off = np.array([cs.get(c, -1) if ("_" not in c and c != "chrM") else -1
                    for c in dix.contigs], np.int64)
    total = int(sum(dix.contig_sizes))
    g0, g1 = total * rank // world, total * (rank + 1) // world
    k = 36
    d_bins = torch.from_numpy(starts).to(dev)
    bc = torch.zeros(len(starts), dtype=torch.int64, device=dev)
    cc = torch.zeros(len(dix.contigs), dtype=torch.int64, device=dev)
    out = torch.empty(2 * (g1 - g0), dtype=torch.uint8, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3 * reps)]
    # C5 from the index arrays (SA, ISA, LCP bytes + overflow): each rep first
    # rebuilds, from SA + the LCP bytes, the per-position unique lengths U and
    # their directory over the text window the rank's bases read
    # (smash_mappability_prepare: longSA.cpp:628-641's m[r] in rank order,
    # scattered to SA[r] by three streaming partition passes), then scans
    # (k_mapscan, k_mapfix).  U is poisoned in that window first, so the scan
    # can only see what the timed rebuild wrote.
    lo, hi = S.mappability_window(dix, g0, g1)
    N = dix.info.N
    U = S.device_view(dix.info.d_uniq, N + 64, torch.uint8)
    U[lo:hi].fill_(0x55)

    host_ms = []   # per timed rep: host time in the prepare call, in the scan call

    def step(i, timed):
        bc.zero_()
        cc.zero_()
        if timed:
            ev[3 * i].record()
        h0 = time.perf_counter()
        S.mappability_prepare(dix, g0, g1)
        h1 = time.perf_counter()
        if timed:
            ev[3 * i + 1].record()
        S.mappability_scan(dix, g0, g1, k, out, off, d_bins, len(starts), bc, cc)
        h2 = time.perf_counter()
        if timed:
            ev[3 * i + 2].record()
            host_ms.append((round(1e3 * (h1 - h0), 2), round(1e3 * (h2 - h1), 2)))
        if world > 1:
            dist.all_reduce(bc)
            dist.all_reduce(cc)

    step(0, False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    for i in range(reps):
        step(i, True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t1
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    prep_ms = sum(ev[3 * i].elapsed_time(ev[3 * i + 1]) for i in range(reps)) / reps
    scan_ms = sum(ev[3 * i + 1].elapsed_time(ev[3 * i + 2]) for i in range(reps)) / reps
    kms = prep_ms + scan_ms
    S.mappability_release(dix)
    # the scan reproduces the index build's map.bin (compared on the device)
    dmap = S.device_view(dix.info.d_map, dix.info.map_bytes, torch.uint8)
    same_map = bool(torch.equal(out, dmap[2 + 2 * g0:2 + 2 * g1]))
    n_uniq = int(cc.sum().item())
    value = total * reps / el
    # the bytes the step streams: the rebuild reads all of SA (idx_bytes per
    # rank) and the LCP bytes (1 B), and per position of the window writes +
    # reads a u32 entry twice (passes 1 -> 2 -> 3) and writes U (1 B); the
    # directory reads U once (1 B); the scan reads U at the forward and at the
    # reverse-complement position (1 B each) and writes the 2 map.bin bytes
    nw = hi - lo
    prep_bytes = N * (dix.info.idx_bytes + 1) + nw * (4 + 8 + 5 + 1)
    scan_bytes = (g1 - g0) * 4
    achieved = (prep_bytes + scan_bytes) / (kms / 1e3) / 1e9
    res = {"metric": "bases/sec mappability self-scan (hg19, every 36-mer; map.bin + unique "
                     "counts, C5) from the index arrays",
           "value": value, "unit": "bases/s", "ms_per_scan": 1000.0 * el / reps,
           "scaling": "strong", "bases": total, "k": k, "bins": int(len(starts)),
           "prepare_ms": round(prep_ms, 3), "scan_ms": round(scan_ms, 3),
           "reps_ms": [[round(ev[3 * i].elapsed_time(ev[3 * i + 1]), 2),
                        round(ev[3 * i + 1].elapsed_time(ev[3 * i + 2]), 2)] for i in range(reps)],
           "reps_host_ms": host_ms,
           "window_positions": int(nw),
           "roofline": {"bound": "hbm", "kernel": "smash_mappability_prepare (k_upart1-3, "
                                                  "k_nsdir) + k_mapscan + k_mapfix",
                        "achieved": round(achieved, 2),
                        "peak": 8000.0, "unit": "GB/s", "frac": round(achieved / 8000.0, 5),
                        "traffic": None,
                        "bytes_per_base": round((prep_bytes + scan_bytes) / (g1 - g0), 2),
                        "bytes_method": "streamed bytes of the rebuild of U from SA + LCP "
                                        "(SA %d B + LCP 1 B per rank; 4 + 8 + 5 + 1 B per "
                                        "window position) + the scan (4 B per base); SURVEY "
                                        "section 8d's gather model (ISA + 2 random LCP lines, "
                                        "146 B per base) prices the same output at %.0f GB/s"
                                        % (dix.info.idx_bytes,
                                           146.0 * (g1 - g0) / (kms / 1e3) / 1e9),
                        "avg_kernel_ms": round(kms, 3)},
           "map_identical_to_index_build": same_map, "unique_kmers": n_uniq,
           "cpu_baseline": None}
    pmc = os.path.join(ROOT, "profiles", "pmc_c5.json")
    if os.path.exists(pmc) and world == 1:
        try:
            j = json.load(open(pmc))
            res["roofline"]["traffic"] = j["c5_bytes_per_rep"]
            res["roofline"]["traffic_vs_model"] = round(j["c5_bytes_per_rep"] /
                                                        max(prep_bytes + scan_bytes, 1), 3)
            res["roofline"]["traffic_source"] = os.path.relpath(pmc, ROOT)
        except Exception:   # noqa: BLE001
            pass
    log("C5: %d reps %.3f s -> %.3e bases/s; prepare %.2f ms + scan %.2f ms; unique %d-mers %d; "
        "map == build: %s" % (reps, el, value, prep_ms, scan_ms, k, n_uniq, same_map))
    if oix is not None and rank == 0 and world == 1 and not args.no_cpu_baseline:
        # oracle/smash_oracle.c orc_mappability_range on every host thread,
        # contiguous sub-windows of one window in the middle of the genome
        from concurrent.futures import ThreadPoolExecutor
        threads, note = host_cores()
        n0 = 1 << 18
        t3 = time.perf_counter()
        oix.mappability_range(g0, g0 + n0, k)
        rate1 = n0 / (time.perf_counter() - t3)
        n1 = int(min(g1 - g0, max(n0, rate1 * threads * args.cpu_seconds / 3)))
        a = (g1 - g0 - n1) // 2 + g0
        cuts = [a + n1 * j // threads for j in range(threads + 1)]
        t3 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            parts = list(ex.map(lambda j: oix.mappability_range(cuts[j], cuts[j + 1], k)[0],
                                range(threads)))
        dt = time.perf_counter() - t3
        got = np.concatenate(parts)
        dev_part = out[2 * (a - g0):2 * (a - g0 + n1)].cpu().numpy()
        exact = bool(np.array_equal(got, dev_part))
        res["cpu_baseline"] = {
            "value": n1 / dt, "unit": "bases/s", "cores": threads, "kind": "port",
            "sample": "%d consecutive forward bases from %d (oracle/smash_oracle.c "
                      "orc_mappability_range, %d threads), %.1f s" % (n1, a, threads, dt),
            "cores_note": note,
            "map_identical_to_device": exact}
        log("C5 cpu baseline: %.3e bases/s on %d threads; identical: %s"
            % (n1 / dt, threads, exact))
    return res


def bench_c5(args, cfg, world, rank, local, dist):
    """--config c5: the C5 scan as the headline line."""
    import torch
    import smashgpu as S
    import synth
    dev = torch.device("cuda", local)
    contigs = synth.make_genome(cfg["genome"])
    T, sp, sz, names = S.text_from_contigs(contigs)
    dix = S.Index.create(T, sp, sz, names, device=local)
    log("device index: %.1f s, %.1f GB in HBM" % (dix.info.build_seconds,
                                                  dix.info.device_bytes / 1e9))
    oix = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import oracle as O
        oix, _ = host_index(S, O, dix, T, sp, sz, names)
    r = c5_scan(args, dix, contigs, cfg["bins"], world, rank, dev, dist, oix, reps=args.steps)
    out_j = {"metric": r.pop("metric"), "value": r.pop("value"), "unit": "bases/s",
             "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
             "ms_per_step": r.pop("ms_per_scan"), "higher_is_better": True,
             "scaling": r.pop("scaling"), "vs_baseline": None, "dtype": "u8/u64 (integer)",
             "data": "synthetic (tools/synth.py hg19-shaped genome)",
             "config": {"workload": cfg["workload"], "genome": cfg["genome"],
                   "index_words": "packed (SA / ISA hints, DESIGN section 3)"
                                  if dix.info.pos_bits else "plain",
                        "bases": r.pop("bases"), "k": r.pop("k"), "bins": r.pop("bins"),
                        "parallelism": "%d contiguous base ranges, all_reduce counts" % world}}
    out_j.update(r)
    if rank == 0:
        print(json.dumps(out_j), flush=True)
    if world > 1:
        dist.destroy_process_group()


def mem_line(args, cfg, dix, d_reads, n, dev, oix, world=1, rank=0, dist=None, steps=None,
             warmup=None, cpu_seconds=None):
    """MEM (-maxmatch) of n C3-style reads (d_reads: dense [n, L] on the
    device; csrc/mem.hip, smash_match_batch SMASH_MODE_MEM), every launch over
    all of them; roofline from the line transitions of mem.hip's own probe
    sequence (oracle orc_mem_dev: the k-mer table from the root, 8-byte
    singleton compares, counted) on a sample, `traffic` from the FETCH_SIZE
    pass in profiles/pmc_c3mem.json; CPU baseline the reference's probe
    sequence (orc_mem, the oracle) on the host's cores; the device's records
    of a sample equal the oracle's, in emission order.  oix: the host copy
    of the index (rank 0), or None."""
    import torch
    import smashgpu as S
    import oracle as O
    steps = args.steps if steps is None else steps
    warmup = args.warmup if warmup is None else warmup
    cpu_seconds = args.cpu_seconds if cpu_seconds is None else cpu_seconds
    L, cap = cfg["read_len"], cfg["cap"]
    out = torch.zeros(n * cap * 2, dtype=torch.int64, device=dev)
    nn = torch.zeros(n, dtype=torch.int32, device=dev)

    def launch():
        S.match_batch(dix, d_reads, n, L, out, cap, nn, mode="MEM")

    log("MEM: %d reads, cap %d; warm-up launch" % (n, cap))
    for _ in range(max(1, warmup)):
        t0 = time.perf_counter()
        launch()
        torch.cuda.synchronize()
        log("MEM: warm-up launch %.3f s" % (time.perf_counter() - t0))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * steps)]
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    for i in range(steps):
        ev[2 * i].record()
        launch()
        ev[2 * i + 1].record()
        ev[2 * i + 1].synchronize()   # (a progress line per launch; the next is queued after)
        log("MEM: launch %d done" % i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t1
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    kms = sum(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(steps)) / steps
    counts = nn.cpu().numpy()
    value = n * world * steps / el
    log("MEM: %d reads x %d launches in %.3f s -> %.3e reads/s; %.1f ms per launch; %.1f MEMs "
        "per read (max %d, cap %d)" % (n, steps, el, value, kms, counts.mean(), counts.max(), cap))
    res = {"metric": "reads/sec MEM search (memsam -maxmatch, hg19, 150 bp)", "value": value,
           "unit": "reads/s", "n_gpus": world, "steps": steps, "warmup": warmup,
           "ms_per_step": 1000.0 * el / steps, "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u8/u64 (integer)",
           "data": "synthetic (tools/synth.py hg19-shaped genome; SMASH reads generated on the "
                   "device, tools/readgen.hip, seeded)",
           "config": {"workload": cfg["workload"], "genome": cfg["genome"], "reads": n,
                      "read_len": L, "cap_per_read": cap,
                      "kernel": "k_mem + k_mem_jobs (csrc/mem.hip)",
                      "parallelism": "dp%d: read shards" % world},
           "mems_per_read": round(float(counts.mean()), 2), "mems_max": int(counts.max()),
           "records_cut": int((counts > cap).sum()), "roofline": None, "cpu_baseline": None}
    if oix is not None:
        t2 = time.time()
        ns = 2000
        sample = d_reads[:ns].cpu().numpy()
        add_sample_kmers(S, dix, oix, sample)
        _, per, ctr = O.mem_batch(oix, sample, threads=host_cores()[0], device_probes=True,
                                  count=True)
        log("MEM: oracle probe sequence over %d reads: %.1f s" % (ns, time.time() - t2))
        lines = {"text": ctr.ref_lines / ns, "sa": ctr.sa_lines / ns, "isa": ctr.isa_lines / ns,
                 "lcp": ctr.lcp_lines / ns, "kmer": ctr.kt_lines / ns}
        b_read = 64.0 * sum(lines.values())
        achieved = n * b_read / (kms / 1e3) / 1e9
        res["roofline"] = {
            "bound": "hbm", "kernel": "k_mem + k_mem_jobs", "achieved": round(achieved, 2),
            "peak": 8000.0, "unit": "GB/s", "frac": round(achieved / 8000.0, 5), "traffic": None,
            "bytes_per_read": round(b_read, 1), "avg_kernel_ms": round(kms, 3),
            "lines_per_read": {k: round(v, 2) for k, v in lines.items()},
            "lines_G_per_s": round(n * sum(lines.values()) / (kms / 1e3) / 1e9, 2),
            "bytes_method": "64 B x line transitions of mem.hip's probe sequence (oracle "
                            "orc_mem_dev on the downloaded index, %d reads)" % ns}
        pmc = os.path.join(ROOT, "profiles", "pmc_c3mem.json")
        if os.path.exists(pmc):
            try:
                j = json.load(open(pmc))
                res["roofline"]["traffic"] = j["mem_bytes_per_read"] * n
                res["roofline"]["traffic_bytes_per_read"] = j["mem_bytes_per_read"]
                res["roofline"]["traffic_source"] = os.path.relpath(pmc, ROOT)
            except Exception:   # noqa: BLE001
                pass
        # the device's records == the oracle's, in emission order
        # (reads whose MEMs exceed cap -- a repeat family's millions -- keep
        # exact counts and cut records: their counts are compared)
        o = out.view(n, 2 * cap)[:200].cpu().numpy().view(np.uint64)
        same = all(S.unpack_records(o[i], counts[i], cap) == oix.search(sample[i].tobytes(),
                                                                         mode="MEM")
                   for i in range(200) if counts[i] <= cap)
        res["records_identical_to_oracle"] = bool(same)
        res["counts_identical_to_oracle"] = bool((per == counts[:ns]).all())
        if not args.no_cpu_baseline:
            threads, note = host_cores()
            t3 = time.perf_counter()
            O.mem_batch(oix, sample[:64 * threads], threads=threads)
            dt0 = time.perf_counter() - t3
            m = int(min(n, max(64 * threads, 64 * threads * cpu_seconds / max(dt0, 1e-3))))
            h = d_reads[:m].cpu().numpy()
            t3 = time.perf_counter()
            O.mem_batch(oix, h, threads=threads)
            dt = time.perf_counter() - t3
            res["cpu_baseline"] = {"value": m / dt, "unit": "reads/s", "cores": threads,
                                   "kind": "port",
                                   "sample": "%d reads of the same reads, longSA::findMEM "
                                             "restated (oracle orc_mem, %d threads), %.1f s"
                                             % (m, threads, dt),
                                   "cores_note": note}
            log("MEM cpu baseline: %.3e reads/s on %d threads" % (m / dt, threads))
    del out, nn
    torch.cuda.empty_cache()
    return res


def bench_mem(args, cfg, world, rank, local, dist):
    """--config c3mem: the MEM line (mem_line) as the headline, on reads of
    its own (cfg pairs, seeded as C3's)."""
    import torch
    import smashgpu as S
    import synth
    import readgen
    import oracle as O
    dev = torch.device("cuda", local)
    contigs = synth.make_genome(cfg["genome"])
    T, sp, sz, names = S.text_from_contigs(contigs)
    dix = S.Index.create(T, sp, sz, names, device=local)
    log("device index: %.1f s" % dix.info.build_seconds)
    P = cfg["pairs"]
    d_reads = readgen.Generator(dix, contigs, cfg["read_len"],
                                seed=cfg["seed"] * 1000 + rank).generate(P)
    oix = None
    if rank == 0:
        t2 = time.time()
        oix, _ = host_index(S, O, dix, T, sp, sz, names,
                            sample_reads=d_reads[:2000].cpu().numpy())
        log("host copy of the index: %.1f s" % (time.time() - t2))
    res = mem_line(args, cfg, dix, d_reads, 2 * P, dev, oix, world, rank, dist)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def fit_batch(B, P, L, free, min_len=20, headroom=12 << 30, nbins=50_000, max_batch=None):
    """the largest batch ceil(P / k) <= B (k = 1, 2, ...) whose pipeline
    buffers leave `headroom` of the free HBM: two search sets' match rows and
    the hit rows (slots u64 per mate each, slots = L - min_len + 1), ~130 B
    of other per-pair state, the key set (~170 B per key of capacity), and
    k_emit_bin_lds's per-block counts (256 x 4 B per bin, up to 311 296
    bins); the headroom is for the file-fed buffers (2 x 2 B x 160 B) and the
    multi-GPU exchange buffers.  Never above max_batch (the library's
    smash_pipeline_max_batch: max_pairs * 2 * slots < 2^32)."""
    slots = L - min_len + 1
    cap = P + P // 8 + (1 << 20)
    fixed = cap * 170 + (256 * 4 * nbins if nbins <= 4 * 77824 else 0)

    def need(b):
        return b * (3 * 2 * slots * 8 + 130) + fixed
    k = max(1, -(-P // B))
    while max_batch and -(-P // k) > max_batch:
        k += 1
    while -(-P // k) > 1_000_000 and need(-(-P // k)) + headroom > free:
        k += 1
    b = -(-P // k)
    log("batch %d pairs (%d per step): %.1f GB of pipeline buffers, %.1f GB of HBM free"
        % (b, k, need(b) / 1e9, free / 1e9))
    return b


def drop_cache(paths):
    """flush the files and drop their pages from the page cache
    (posix_fadvise DONTNEED after fsync), so the file-fed run reads them
    from disk, not from the memory the writer just filled"""
    for q in paths:
        fd = os.open(q, os.O_RDONLY)
        try:
            os.fsync(fd)
            os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
        finally:
            os.close(fd)


def feed_bench(S, pipe, starts, L, d_reads, P, B, dev, tmpdir, n_plain=None, n_gz=4000000,
               gz_lanes=16):
    """The file-fed rate (smash_count_fastq, csrc/feed.hip): the same reads
    written as FASTQ (names in sort -n order) to local disk, then counted from
    the files through the bench's own pipeline (its batches of B pairs) with
    parse / H2D / compute overlapped: plain as ONE file pair of all P pairs
    (the C3 run; the parallel reader indexes it by byte range), gzip as
    `gz_lanes` lane files per mate (SMASH passes lane lists; gzip inflates one
    thread per file).  Counts must equal the device-resident run's on the same
    pairs.  Also the pinned H2D copy rate."""
    import shutil
    import torch
    import readgen
    res = {}
    n_plain = min(P, n_plain or P)
    rec = 2 * (2 * L + 21)                 # bytes per pair on disk
    free = shutil.disk_usage(tmpdir).free
    if n_plain * rec * 1.2 > free:         # (a box with little scratch space: fewer pairs)
        n_plain = int(free / 1.2 / rec)
    n_gz = min(n_plain, n_gz)

    def resident(n):
        pipe.reset()
        c = torch.zeros(len(starts), dtype=torch.int64, device=dev)
        pipe.count_batches(d_reads, n, B, c)
        return c.cpu().numpy()

    # warm-up: the first call pins the feed's slots (3 x 2 B L bytes) and
    # allocates its device buffers, which the pipeline keeps for later calls
    # (a service's steady state; the first call's wall time is reported)
    h = d_reads[:2 * min(P, 10000), :L].contiguous().cpu().numpy()
    w1, w2 = readgen.write_fastq_lanes(h, os.path.join(tmpdir, "warm"), 1)
    c = torch.zeros(len(starts), dtype=torch.int64, device=dev)
    pipe.reset()
    t0 = time.perf_counter()
    pipe.count_fastq(w1, w2, c, sort_names=False)
    res["first_call_setup_s"] = round(time.perf_counter() - t0, 3)
    for q in w1 + w2:
        os.remove(q)

    for kind, n, lanes in (("plain", n_plain, 1), ("gz", n_gz, gz_lanes)):
        t0 = time.perf_counter()
        h = d_reads[:2 * n, :L].contiguous().cpu().numpy()
        p1, p2 = readgen.write_fastq_lanes(h, os.path.join(tmpdir, kind), lanes, gz=kind == "gz")
        del h
        wr = time.perf_counter() - t0
        drop_cache(p1 + p2)
        nbytes = sum(os.path.getsize(q) for q in p1 + p2)
        exp = resident(n)
        pipe.reset()
        c = torch.zeros(len(starts), dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        fs = pipe.count_fastq(p1, p2, c, sort_names=False)
        same = bool(np.array_equal(c.cpu().numpy(), exp))
        res[kind] = {"reads_per_s": round(2 * fs["pairs"] / fs["wall_s"], 1),
                     "pairs": int(fs["pairs"]), "batches": int(fs["batches"]),
                     "files_per_mate": lanes, "parallel_reader": bool(fs["parallel"]),
                     "wall_s": round(fs["wall_s"], 3), "index_s": round(fs["index_s"], 3),
                     "ingest_s": round(fs["ingest_s"], 3),
                     "device_waited_s": round(fs["wait_s"], 3), "file_bytes": int(nbytes),
                     "page_cache": "dropped after writing (fsync + posix_fadvise DONTNEED)",
                     "counts_identical_to_resident": same}
        if kind == "gz":
            # the multi-GPU driver's rank-local reader (smashgpu.FastqShards)
            # on the same lanes at world 1: its scan (every file inflated
            # once) and the packs of the run's batches
            drop_cache(p1 + p2)
            t2 = time.perf_counter()
            sh = S.FastqShards(p1, p2, 0, 1, lambda b: [b])
            buf = np.empty((2 * min(B, sh.n), L), np.uint8)
            for k0 in range(0, sh.n, B):
                sh.pack(k0, min(sh.n, k0 + B), buf)
            ss = sh.stats()
            sh.close()
            res["gz_shard_reader"] = {
                "reads_per_s": round(2 * n / (time.perf_counter() - t2), 1),
                "scan_s": round(ss["scan_s"], 3), "pack_s": round(ss["pack_s"], 3),
                "scan_bytes": int(ss["scan_bytes"]), "pack_bytes": int(ss["pack_bytes"]),
                "note": "host only (no device); at W ranks each scans ~1/W of the files and "
                        "packs only its own batches"}
        log("file-fed %s: %d pairs in %d file(s) per mate, %.3f s -> %.3e reads/s (index %.3f s, "
            "ingest %.3f s, device waited %.3f s, %.1f GB, written in %.1f s, parallel reader %s); "
            "counts == resident: %s"
            % (kind, fs["pairs"], lanes, fs["wall_s"], 2 * fs["pairs"] / fs["wall_s"],
               fs["index_s"], fs["ingest_s"], fs["wait_s"], nbytes / 1e9, wr,
               bool(fs["parallel"]), same))
        for q in p1 + p2:
            os.remove(q)
    # the pinned host -> device copy rate of one batch of reads
    hp = torch.from_numpy(d_reads[:2 * min(P, 1000000)].cpu().numpy()).pin_memory()   # (rows)
    dd = torch.empty_like(hp, device=dev)
    dd.copy_(hp, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        dd.copy_(hp, non_blocking=True)
    torch.cuda.synchronize()
    gbs = 5 * hp.numel() / (time.perf_counter() - t0) / 1e9
    res["h2d_pinned_GBps"] = round(gbs, 2)
    res["h2d_reads_per_s"] = round(gbs * 1e9 / d_reads.shape[1], 1)
    res["method"] = ("smash_count_fastq (csrc/feed.hip) through the bench's pipeline: plain "
                     "strict 4-line FASTQ read by the parallel reader (csrc/fastq_par.hpp: files "
                     "mapped, records indexed by byte range, checked and packed on all host "
                     "threads); gzip lanes by the per-file streaming producer (worker threads "
                     "inflate and index files in pair order, batches packed as they land); "
                     "3 pinned slots, 2 device buffers, H2D on its own stream; batches of %d "
                     "pairs; FASTQ on local disk, names in sort -n order, page cache dropped "
                     "before each read" % B)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--pairs", type=int, default=0, help="pairs per rank per step")
    ap.add_argument("--batch", type=int, default=0, help="pairs per device batch")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 scan on the same index")
    ap.add_argument("--no-feed", action="store_true", help="skip the file-fed measurement")
    ap.add_argument("--no-sub", action="store_true",
                    help="skip the C2 and MEM lines on the same index (c3, one GPU)")
    ap.add_argument("--feed-pairs", type=int, default=0,
                    help="pairs of the file-fed run (0: all the rank's pairs, the C3 run)")
    args = ap.parse_args()
    cfg = dict(CONFIGS[args.config])
    if args.pairs:
        cfg["pairs"] = args.pairs
    if args.batch:
        cfg["batch"] = args.batch

    import torch
    import smashgpu as S
    import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # SMASH_BENCH_SHARDED=1 (under torchrun, any world size): the multi-GPU
    # step (dist.ShardedCounter, collectives over RCCL) even at world 1 --
    # the per-rank rate of the N > 1 path, measurable on one GPU
    sharded = world > 1 or os.environ.get("SMASH_BENCH_SHARDED", "0") == "1"
    if sharded:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if args.config == "c5":
        return bench_c5(args, cfg, world, rank, local, dist)
    if args.config == "c3mem":
        return bench_mem(args, cfg, world, rank, local, dist)

    t0 = time.time()
    contigs = synth.make_genome(cfg["genome"])
    T, sp, sz, names = S.text_from_contigs(contigs)
    log("genome %s: %.3f Gbp, N=%d (%.1fs)" % (cfg["genome"], sum(len(s) for _, s in contigs) / 1e9,
                                               len(T), time.time() - t0))
    dix = S.Index.create(T, sp, sz, names, device=local)
    log("device index: %.1f s, %.1f GB in HBM, idx_bytes=%d, lcp overflow %d"
        % (dix.info.build_seconds, dix.info.device_bytes / 1e9, dix.info.idx_bytes,
           dix.info.n_lcp_overflow))
    tmpdir = tempfile.mkdtemp()
    starts = bin_starts_for(cfg, contigs, tmpdir)
    cs = chrom_sizes_for(cfg, contigs)
    P, L, B = cfg["pairs"], cfg["read_len"], min(cfg["batch"], cfg["pairs"])
    # the rank's reads, generated on the device (tools/readgen.hip), resident
    import readgen
    gen = readgen.Generator(dix, contigs, L, seed=cfg["seed"] * 1000 + rank)
    d_reads = gen.generate(P)
    # the device's native read layout: each mate in a 16-byte aligned,
    # zero-padded row (smash_read_stride: 160 B at 150 bp), which the search
    # copies straight into LDS (no record build); SMASH_BENCH_ROWS=0: dense
    # [2P, L] mates, searched through k_prep's records (A/B)
    rows = os.environ.get("SMASH_BENCH_ROWS", "1") != "0"
    if rows:
        d_reads = S.to_rows(d_reads, L)
    torch.cuda.synchronize()
    log("reads: %d pairs x %d bp per rank in HBM (%.1f GB, rows of %d B), batches of %d "
        "(%.1fs since start)" % (P, L, d_reads.numel() / 1e9, d_reads.shape[1], B,
                                 time.time() - t0))
    # the batch: the config's (C3: 12.5 M pairs, 2 per step) when the
    # pipeline's buffers leave 12 GB of what the index and the reads leave of
    # HBM, else P / 3, P / 4, ... (at hg19 with 150 bp reads: P / 3 = 8.33 M;
    # profiles/r04/sched: 3.50-3.52e8 reads/s vs 3.47-3.48e8 at 6.25 M and
    # 3.56-3.60e8 at 12.5 M, which leaves only ~4 GB)
    if not args.batch:
        free = torch.cuda.mem_get_info(dev)[0]
        if sharded:   # every rank must run the same batches: the least free HBM decides
            f = torch.tensor([free], dtype=torch.int64, device=dev)
            dist.all_reduce(f, op=dist.ReduceOp.MIN)
            free = int(f.item())
        # (one GPU: 6 GB beside the pipeline hold the file-fed buffers of
        # 6.25 M-pair feed batches, or the world-1 exchange; N > 1 GPUs: 12 GB
        # for the exchange with the other ranks)
        B = fit_batch(B, P, L, free, headroom=(12 << 30) if world > 1 else (6 << 30),
                      nbins=len(starts), max_batch=S.pipeline_max_batch(L))
    # the key set: every key of the run (single GPU), or the keys this rank
    # owns ((hash >> 1) % world of all ranks' keys: ~P as well)
    pipe = S.Pipeline(dix, cs, starts, L, B, dedup_capacity=P + P // 8 + (1 << 20),
                      read_stride=d_reads.shape[1] if rows else 0)
    counts = torch.zeros(len(starts), dtype=torch.int64, device=dev)
    nb = (P + B - 1) // B

    if sharded:
        from dist import ShardedCounter
        # the per-batch key counts are host integers: exchanged over gloo
        # they need no device synchronisation
        sc = ShardedCounter(pipe, rank, world, dev, count_group=dist.new_group(backend="gloo"),
                            plan_pairs=P * world)
        # the reads are resident and complete: the phase searches wait on no
        # input event, so a look-ahead search (the next batch's, or the next
        # run's first ones) starts once its set's post stage is done instead
        # of behind everything queued for the current batch
        pipe.reads_resident(True)

    resident = os.environ.get("SMASH_BENCH_RESIDENT", "1") != "0"   # (A/B)
    ahead2 = os.environ.get("SMASH_BENCH_AHEAD2", "1") != "0"       # (A/B, sharded step)

    # SMASH_BENCH_CROSS=0 (A/B, sharded step): no look-ahead across runs
    cross = os.environ.get("SMASH_BENCH_CROSS", "1") != "0"

    def step(i, last=0):
        """one run over the rank's P pairs: a fresh key set / adjacent-dup
        state (a new smashMEM.py + varbin.py invocation), carried across
        the batches.  i: the run's index among `last` runs issued back to
        back (the sharded step searches run i + 1's first batches under run
        i's last exchange when i + 1 < last)"""
        counts.zero_()
        if not sharded:
            pipe.reset()
            # the batches in order; each batch's search starts under the
            # previous one's tail, and (the reads are resident: no input
            # event, smash_count_batches_ready) this run's first searches
            # under the previous run's post stage
            pipe.count_batches(d_reads, P, B, counts, resident=resident)
        else:
            # (cross: the previous run's last batch already issued this run's
            # first searches -- back-to-back runs over the resident reads, as
            # the single-GPU chain overlaps them; never across the warm-up /
            # timed boundary, and the last timed run issues none)
            sc.reset(keep_search=cross and i > 0)
            for b in range(nb):
                b0, b1 = b * B, min(P, (b + 1) * B)
                n0, n1 = b1, min(P, b1 + B)   # the next batch, searched under this one's exchange
                m0, m1 = n1, min(P, n1 + B)   # and the one after, once this one's export is done
                if b + 1 == nb and cross and i + 1 < last:
                    n0, n1 = 0, min(P, B)          # the next run's first batches
                    m0, m1 = n1, min(P, n1 + B)
                    if m0 == 0 or nb == 1:
                        m1 = m0                    # (one batch per run: no second)
                if not ahead2:
                    m1 = m0
                sc.step(d_reads[2 * b0:2 * b1], b1 - b0, b0 * world, counts,
                        d_reads[2 * n0:2 * n1] if n1 > n0 else None, n1 - n0,
                        next2_reads=d_reads[2 * m0:2 * m1] if m1 > m0 else None,
                        next2_pairs=m1 - m0)
            dist.all_reduce(counts)

    for i in range(args.warmup):
        step(i, args.warmup)
    torch.cuda.synchronize()
    ref_counts = counts.cpu().numpy().copy()
    st0 = pipe.stats()
    if st0.error:
        raise SystemExit("pipeline data error: %s" % S.ERRORS.get(st0.error, st0.error))
    pipe.profile(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for i in range(args.steps):
        step(i, args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t1
    if sharded and sc.timing:
        log("sharded step phases (s, synchronised): %s"
            % ", ".join("%s %.3f" % kv for kv in sc.timing.items()))
    mam_ms, launches, mam_reads = pipe.profile_read()
    active_ms = pipe.profile_active()
    launch_iv = pipe.profile_intervals()
    pipe.profile(False)
    st = pipe.stats()
    if st.error:
        raise SystemExit("pipeline data error: %s" % S.ERRORS.get(st.error, st.error))
    same = bool(np.array_equal(counts.cpu().numpy(), ref_counts)) if args.warmup else True
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    total_reads = 2 * P * world * args.steps
    value = total_reads / el
    log("timed %d steps: %.3f s -> %.3e reads/s; k_mam %.2f ms/launch, %.2f ms active per launch "
        "(%d launches); stats %s; deterministic=%s"
        % (args.steps, el, value, mam_ms / max(launches, 1), active_ms / max(launches, 1),
           launches, st.as_dict(), same))

    out = {
        "metric": METRIC, "value": value, "unit": "reads/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": 1000.0 * el / args.steps, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8/u64 (integer)",
        "data": "synthetic (tools/synth.py hg19-shaped genome; SMASH reads generated on the "
                "device, tools/readgen.hip, seeded)",
        "config": {"workload": cfg["workload"], "genome": cfg["genome"],
                   "index_words": "packed (SA / ISA hints, DESIGN section 3)"
                                  if dix.info.pos_bits else "plain",
                   "genome_bp": int(sum(len(s) for _, s in contigs)),
                   "text_N": int(dix.info.N), "pairs_per_rank": P, "read_len": L,
                   "reads_per_step": 2 * P * world, "batch_pairs": B, "batches_per_step": nb,
                   "bins": int(len(starts)),
                   "parallelism": "dp%d: pair shards, all_to_all key de-dup, "
                                  "all_gather tails, all_reduce counts" % world
                   if sharded else "single GPU",
                   "index_build_s": round(dix.info.build_seconds, 2),
                   "index_hbm_gb": round(dix.info.device_bytes / 1e9, 2)},
    }

    # ---- roofline + cpu baseline (rank 0) -------------------------------------
    avg_ms = mam_ms / max(launches, 1)
    act_ms = active_ms / max(launches, 1)
    reads_per_launch = mam_reads / max(launches, 1)
    roof = None
    cpu = None
    oix = None
    if rank == 0:
        import oracle as O
        t2 = time.time()
        ns = min(4000, 2 * P)
        sample = d_reads[:ns, :L].contiguous().cpu().numpy()
        oix, mp = host_index(S, O, dix, T, sp, sz, names, sample_reads=sample)
        log("host copy of the index for the oracle: %.1fs" % (time.time() - t2))
        # algorithmic bytes per read: 64 B x the 64-byte line transitions of
        # k_mam_sm's own probe sequence, counted by running the kernel's code
        # on the host (tools/sm_emu: the same source, one lane) over this
        # index and a sample of the same reads
        emu, emu_it, lines = search_lines(S, dix, oix, sample)
        b_read = 64.0 * lines / ns
        # achieved = the bytes of one launch / the average launch duration
        # (HIP events around each k_mam_sm on its own stream; rocprofv3's
        # kernel-trace average of the same command must agree).  Consecutive
        # batches' searches overlap on the two search streams, so a launch's
        # duration includes its share of the GPU with the neighbour; the union
        # of the launches' intervals is reported beside it, not used for frac
        achieved = reads_per_launch * b_read / (avg_ms / 1e3) / 1e9
        roof = {"bound": "hbm", "kernel": "k_mam_sm", "achieved": round(achieved, 2),
                "peak": 8000.0, "unit": "GB/s", "frac": round(achieved / 8000.0, 5),
                "traffic": None, "bytes_per_read": round(b_read, 1),
                "avg_kernel_ms": round(avg_ms, 3),
                "active_ms_per_launch": round(act_ms, 3),
                # the step's time split: the union of the search launches'
                # intervals and the rest (the post stage and record builds
                # the searches do not cover; DESIGN.md §3 schedule table)
                "search_union_ms_per_step": round(active_ms / args.steps, 3),
                "non_search_ms_per_step": round(1000.0 * el / args.steps - active_ms / args.steps, 3),
                "frac_over_active_time": round(mam_reads * b_read / (active_ms / 1e3) / 1e9 / 8000.0, 5),
                "timing": "achieved = reads_per_launch x bytes_per_read / avg_kernel_ms (HIP events "
                          "around each k_mam_sm launch on its stream); launches overlap by %.1f%% "
                          "of the time at least one ran (active_ms_per_launch)" % (
                              100.0 * (mam_ms - active_ms) / max(active_ms, 1e-9)),
                "reads_per_launch": int(reads_per_launch),
                # every timed launch's [start, end] (ms from the first start;
                # HIP events on its stream): avg_kernel_ms is their mean
                # duration, so frac can be recomputed from this line alone
                "launch_intervals_ms": [[round(a, 3), round(b, 3)] for a, b in launch_iv],
                "launches": int(launches),
                "lines_per_read": {k: round(v[1] / ns, 3) for k, v in emu.counters.items()},
                "probes_per_read": {k: round(v[0] / ns, 3) for k, v in emu.counters.items()},
                "loop_iterations_per_read": round(float(emu_it.mean()), 1),
                # the memory requests the kernel issues (every 16-byte load, the
                # binary search's speculative SA elements included): with the
                # lines they bring, the figures of the request-rate ceiling
                # (tools/randbench req)
                "requests_per_read": round(emu.requests[0] / ns, 2),
                "speculative_requests_per_read": round(emu.requests[1] / ns, 2),
                "requests_G_per_s": round(reads_per_launch * emu.requests[0] / ns / (avg_ms / 1e3) / 1e9, 2),
                "lines_G_per_s": round(reads_per_launch * lines / ns / (avg_ms / 1e3) / 1e9, 2),
                "bytes_method": "64 B x line transitions of the kernel's probe sequence "
                                "(tools/sm_emu on the downloaded index, %d reads)" % ns}
        pmc = os.path.join(ROOT, "profiles", "pmc_%s.json" % args.config)
        if os.path.exists(pmc):
            try:
                j = json.load(open(pmc))
                roof["traffic"] = j.get("k_mam_bytes_per_read", 0) * reads_per_launch or \
                    j.get("k_mam_bytes_per_launch")
                roof["traffic_source"] = os.path.relpath(pmc, ROOT)
            except Exception:
                pass
        if world == 1 and not args.no_cpu_baseline:
            threads, note = host_cores()
            op = O.Pipeline(oix, mp, cs, starts)
            # calibrate, then a bounded sample of ~cpu_seconds of the same reads
            n0 = min(P, 64 * threads)
            h0 = d_reads[:2 * n0, :L].contiguous().cpu().numpy()
            t3 = time.perf_counter()
            op.run(h0, threads=threads)
            dt0 = time.perf_counter() - t3
            n1 = int(min(P, max(n0, n0 * args.cpu_seconds / max(dt0, 1e-3))))
            h1 = d_reads[:2 * n1, :L].contiguous().cpu().numpy()
            op = O.Pipeline(oix, mp, cs, starts)
            t3 = time.perf_counter()
            err = op.run(h1, threads=threads)
            dt = time.perf_counter() - t3
            # the search alone (longSA::MAM, no resolve/tag/filter/bin), ~5 s
            nm = int(min(len(h1), max(2 * n0, 5.0 * 2 * n1 / max(dt, 1e-3))))
            t3 = time.perf_counter()
            O.map_only(oix, h1[:nm], threads=threads)
            dtm = time.perf_counter() - t3
            # device on the same sample must give the same counts
            pipe.reset()
            c2 = torch.zeros(len(starts), dtype=torch.int64, device=dev)
            pipe.count_batches(d_reads, n1, B, c2)
            dev_counts = c2.cpu().numpy().astype(np.uint64)
            exact = bool(err == 0 and np.array_equal(dev_counts, op.counts))
            cpu = {"value": 2 * n1 / dt, "unit": "reads/s", "cores": threads,
                   "kind": "port",
                   "sample": "%d pairs (%d reads) of the same reads, whole chain "
                             "(oracle/smash_oracle.c orc_run_pairs, %d threads), %.1f s"
                             % (n1, 2 * n1, threads, dt),
                   "mapping_only_reads_per_s": round(nm / dtm, 1),
                   "mapping_only_sample": "%d reads, longSA::MAM restated (orc_map_only), "
                                          "%.1f s" % (nm, dtm),
                   "end_to_end_reads_per_s": round(2 * n1 / dt, 1),
                   "cores_note": note,
                   "port_vs_reference": "the port maps 1.64x the reference binary's rate on "
                                        "1 core, 1.04x on 8 (profiles/r03/"
                                        "cpu_calibration_c1.log): an upper bound on the "
                                        "reference CPU path",
                   "index_load_s": round(time.time() - t2 - dt - dtm - dt0, 1),
                   "bin_counts_identical_to_device": exact}
            log("cpu baseline: %.3e reads/s end to end, %.3e mapping only, on %d threads; "
                "device==oracle counts: %s" % (cpu["value"], nm / dtm, threads, exact))
    out["roofline"] = roof
    out["cpu_baseline"] = cpu
    # the side measurements must not cost the line: a failure is recorded in
    # its object (and the log) instead
    if rank == 0 and world == 1 and not args.no_feed:
        # the file-fed batches: at most 6.25 M pairs (2 x 2 B x 160 B of
        # device buffers beside the pipeline)
        os.environ.setdefault("SMASH_FEED_BATCH", str(min(B, 6_250_000)))
        try:
            out["host_boundary"] = feed_bench(S, pipe, starts, L, d_reads, P, B, dev, tmpdir,
                                              n_plain=args.feed_pairs)
        except Exception as e:   # noqa: BLE001
            log("file-fed measurement failed: %r" % (e,))
            out["host_boundary"] = {"error": repr(e)}
    out["deterministic_counts"] = same
    out["stats_last_step"] = st.as_dict()
    # the other hg19 lines on the same resident index (BASELINE configs[1]
    # C2, the MEM mode north_star names, configs[4] C5): each needs HBM of
    # its own, so the C3 pipeline and its file-fed buffers go first
    subs = cfg["genome"] == "hg19" and args.config == "c3"
    if subs and world == 1 and not args.no_sub:
        pipe.close()
        torch.cuda.empty_cache()
        try:
            out["c2"] = c2_line(args, dix, contigs, dev, oix, mp if oix is not None else None)
        except Exception as e:   # noqa: BLE001
            log("C2 line failed: %r" % (e,))
            out["c2"] = {"error": repr(e)}
        try:
            mcfg = CONFIGS["c3mem"]
            nm = 2 * mcfg["pairs"]
            # the first 2 M of C3's own reads, dense (k_mem reads [n, L])
            dm = d_reads[:nm, :L].contiguous()
            out["c3mem"] = mem_line(args, mcfg, dix, dm, nm, dev, oix, steps=2, warmup=1,
                                    cpu_seconds=min(10.0, args.cpu_seconds))
            del dm
        except Exception as e:   # noqa: BLE001
            log("MEM line failed: %r" % (e,))
            out["c3mem"] = {"error": repr(e)}
    if cfg["genome"] == "hg19" and not args.no_c5:
        # the scan needs ~12 GB of its own (its map.bin output and the
        # comparison)
        pipe.close()
        torch.cuda.empty_cache()
        out["c5"] = c5_scan(args, dix, contigs, "50000", world, rank, dev, dist, oix)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if sharded:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
