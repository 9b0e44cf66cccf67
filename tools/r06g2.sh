#!/bin/bash
# round-6 session 3: the search kernel built with other LLVM scheduling
# strategies (max-ilp, iterative-ilp) vs the default, C3 step A/B, 2 rounds
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
ROUNDS=2 TESTS=none bash "$R/tools/r06_ab.sh" r06g2 '- libsmashgpu_ilp.so libsmashgpu_iter.so'
