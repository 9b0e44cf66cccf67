"""tools/index_time.py [SETTING ...] -- the device index build of the hg19-shaped
genome (bench.py's), timed once per setting in ONE process (the genome is made
once), alternating; SETTING: VAR=VALUE[,VAR=VALUE] or "base".  Prints the
build seconds and the LCP step's (SMASH_VERBOSE)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("smash-paper_amd", "tools"):
    sys.path.insert(0, os.path.join(ROOT, p))


def main():
    import smashgpu as S
    import synth
    os.environ["SMASH_VERBOSE"] = "1"
    contigs = synth.make_genome("hg19")
    T, sp, sz, names = S.text_from_contigs(contigs)
    for setting in sys.argv[1:] or ["base"]:
        env = {} if setting == "base" else dict(kv.split("=", 1) for kv in setting.split(","))
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        t = time.time()
        dix = S.Index.create(T, sp, sz, names, device=0)
        print("[index_time] %-24s build %.2f s (wall %.2f s)" % (setting, dix.info.build_seconds,
                                                               time.time() - t), flush=True)
        del dix
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


if __name__ == "__main__":
    main()
