#!/bin/bash
# tools/ab.sh OUT LIB_A [LIB_B] -- A/B timing of two builds of libsmashgpu.so on
# the same box: tools/sweep.py runs once per library (SMASH_LIB), A, B, A, B,
# each in its own process (genome + index + reads rebuilt per process).
# Extra sweep settings for the B runs can follow in SWEEP_B.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/$1; A=$R/$2; B=${3:+$R/$3}
mkdir -p "$O"
for k in 1 2; do
  timeout -k 10 300 env SMASH_LIB="$A" python3 "$R/tools/sweep.py" --steps 5 base > "$O/a$k.log" 2>&1
  if [ -n "$B" ]; then
    timeout -k 10 300 env SMASH_LIB="$B" python3 "$R/tools/sweep.py" --steps 5 base ${SWEEP_B:-} > "$O/b$k.log" 2>&1
  else
    timeout -k 10 300 python3 "$R/tools/sweep.py" --steps 5 base ${SWEEP_B:-} > "$O/b$k.log" 2>&1
  fi
done
grep -h "sweep\] [a-zA-Z]" "$O"/a*.log "$O"/b*.log
