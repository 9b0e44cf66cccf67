#!/bin/bash
# round-6 session 3: C5 prepare variants under rocprofv3 (one process each:
# its kernel stats), and the round-5 U rebuild (libsmashgpu_u0.so) on the
# same box
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r06s
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for v in "nt512:" "nt1024:SMASH_UPART_NT=1024" "e256:SMASH_UPART_E2MB=256,SMASH_UPART_NT=1024"; do
  n=${v%%:*}
  ROUNDS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/prof_$n" -o run \
      --output-format csv -- python3 -u "$R/tools/c5_ab.py" "$v" > "$O/c5_$n.log" 2>&1
done
ROUNDS=2 SMASH_LIB=$R/smash-paper_amd/lib/libsmashgpu_u0.so timeout -k 10 200 python3 -u \
    "$R/tools/c5_ab.py" u0: > "$O/c5ab_u0.log" 2>&1
ROUNDS=2 timeout -k 10 200 python3 -u "$R/tools/c5_ab.py" nt512: nt1024:SMASH_UPART_NT=1024 \
    e256:SMASH_UPART_E2MB=256,SMASH_UPART_NT=1024 > "$O/c5ab.log" 2>&1
