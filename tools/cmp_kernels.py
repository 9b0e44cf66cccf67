"""tools/cmp_kernels.py CONFIG [PAIRS] -- run smash_map_batch on the bench
workload with the direct per-lane kernel and with the state-machine kernel
(bounds-checked: SMASH_SM_CHECK=1) and report every read whose packed matches
differ.  GPU debugging aid: no pipeline kernels run, so a wrong match list
cannot turn into a fault downstream.  Writes gpurun_out/cmp_<config>.json.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in ("smash-paper_amd", "tools", "oracle", ""):
    sys.path.insert(0, os.path.join(ROOT, _p))

import numpy as np  # noqa: E402


def main():
    cfg_name = sys.argv[1] if len(sys.argv) > 1 else "mid"
    import bench
    import smashgpu as S
    import synth
    import torch
    cfg = dict(bench.CONFIGS[cfg_name])
    if len(sys.argv) > 2:
        cfg["pairs"] = int(sys.argv[2])
    t0 = time.time()
    contigs = synth.make_genome(cfg["genome"])
    T, sp, sz, names = S.text_from_contigs(contigs)
    dix = S.Index.create(T, sp, sz, names)
    print("index %.1fs idx_bytes %d" % (time.time() - t0, dix.info.idx_bytes), flush=True)
    reads = bench.make_reads(contigs, cfg, cfg["pairs"], cfg["seed"] * 1000)
    n, L = reads.shape
    d = torch.from_numpy(reads).cuda()
    cap = 64
    res = {}
    for kern in ("direct", "sm"):
        os.environ["SMASH_MAM_KERNEL"] = kern
        if kern == "sm":
            os.environ["SMASH_SM_CHECK"] = "1"
        out = torch.zeros(n * cap, dtype=torch.int64, device="cuda")
        nout = torch.zeros(n, dtype=torch.int32, device="cuda")
        t = time.time()
        try:
            S.map_batch(dix, d, n, L, out, cap, nout)
            torch.cuda.synchronize()
        except S.SmashError as e:
            print("%s: %s" % (kern, e), flush=True)
            res["error_" + kern] = str(e)
        print("%s: %.3fs" % (kern, time.time() - t), flush=True)
        res[kern] = (out.view(n, cap).cpu().numpy(), nout.cpu().numpy())
    os.environ.pop("SMASH_SM_CHECK", None)
    (o1, n1), (o2, n2) = res["direct"], res["sm"]
    diff = np.nonzero((n1 != n2) | np.any(o1 != o2, axis=1))[0]
    rep = {"config": cfg_name, "reads": int(n), "differ": int(len(diff)),
           "error": res.get("error_sm"), "first": []}
    for i in diff[:20]:
        k1, k2 = min(int(n1[i]), cap), min(int(n2[i]), cap)
        rep["first"].append({"read": int(i), "seq": reads[i].tobytes().decode("latin1"),
                             "direct": S.unpack_matches(o1[i], k1),
                             "sm": S.unpack_matches(o2[i], k2)})
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(rep, open(os.path.join(ROOT, "gpurun_out", "cmp_%s.json" % cfg_name), "w"), indent=1)
    print("reads %d differ %d error %s" % (n, len(diff), rep["error"]))


if __name__ == "__main__":
    main()
