#!/bin/bash
# tools/isa_lines.sh [KERNEL_SUBSTR] [TOP] -- static instructions of one
# k_mam_sm instantiation attributed to source lines (-g line tables), the top
# TOP lines.  In the state-machine regime nearly every state body runs each
# wave iteration, so this is a cost map of the loop.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
K=${1:-_ZN5smash2sm8k_mam_smImLi64ELb1ELb0EE}
TOP=${2:-30}
T=$(mktemp -d)
cd "$T"
/opt/rocm/bin/hipcc -O3 -g -std=c++17 --offload-arch=gfx950 -I"$R/include" -c \
  "$R/smash-paper_amd/csrc/mam.hip" --save-temps -o mam.o 2>/dev/null
/opt/rocm/lib/llvm/bin/llvm-objdump -d -l --no-show-raw-insn ./*gfx950.out > dis.txt
python3 - "$K" "$TOP" "$R/smash-paper_amd/csrc/mam_sm.hpp" <<'PY'
import collections, re, sys
k, top, src = sys.argv[1], int(sys.argv[2]), open(sys.argv[3]).read().split("\n")
infn, cur, cnt = False, None, collections.Counter()
for l in open("dis.txt"):
    if re.match(r"^[0-9a-f]+ <", l):
        infn = k in l
        continue
    if not infn:
        continue
    m = re.match(r"^; (/\S+):(\d+)", l)
    if m:
        cur = (m.group(1).split("/")[-1], int(m.group(2)))
        continue
    m = re.match(r"^\s+([a-z_0-9]+)\s", l)
    if m and cur:
        cnt[cur] += 1
print("total", sum(cnt.values()))
for (f, ln), c in cnt.most_common(top):
    txt = src[ln - 1].strip()[:90] if f == "mam_sm.hpp" else ""
    print("%5d  %s:%d  %s" % (c, f, ln, txt))
PY
rm -rf "$T"
