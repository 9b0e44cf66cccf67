#!/bin/bash
# tools/isa_stats.sh [KERNEL_REGEX] -- static instruction mix of the k_mam_sm
# loop as compiled for gfx950 (VALU / SALU / VMEM / LDS / branch / spill
# lanes).  In the state-machine regime a wave executes nearly the whole loop
# body every iteration, so the static counts track per-iteration cost.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
K=${1:-'k_mam_smImLi64ELb1ELb0EE'}
T=$(mktemp -d)
cd "$T"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I"$R/include" -c \
  "$R/smash-paper_amd/csrc/mam.hip" --save-temps -o mam.o 2>/dev/null
S=$(ls "$T"/*gfx950*.s)
awk -v pat="^_ZN5smash2sm8${K}EvNS0_3CtxIT_EE:" '$0 ~ pat {p=1} p {print} p && /s_endpgm/ {exit}' "$S" > k.s
awk '
  /^[ \t]+v_writelane|^[ \t]+v_readlane/ {spill++}
  /^[ \t]+v_/ {valu++}
  /^[ \t]+s_/ && !/s_waitcnt|s_nop|s_cbranch|s_branch/ {salu++}
  /^[ \t]+s_cbranch|^[ \t]+s_branch/ {br++}
  /^[ \t]+(global|flat|buffer|scratch)_/ {vmem++}
  /^[ \t]+ds_/ {lds++}
  END {printf "VALU %d (spill-lane ops %d)  SALU %d  branches %d  VMEM %d  LDS %d\n", valu, spill, salu, br, vmem, lds}
' k.s
grep -E "VGPRs:|SGPRs Spill|Occupancy" <(/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I"$R/include" -c "$R/smash-paper_amd/csrc/mam.hip" -o /dev/null -Rpass-analysis=kernel-resource-usage 2>&1 | grep -A8 "$K" ) | sed 's/.*remark: *//' | head -3
rm -rf "$T"
