#!/bin/bash
# tools/r05_measure.sh TAG [PART] -- the round-5 measurement set, in two box
# calls (each under gpurun's 20-minute limit):
# PART 1:
#   1. the MEM hg19 parity test (-m gpu -k mem_hg19)                   -> tests.log
#   2. bench.py --config c3mem (the MEM line)                          -> c3mem.json/.log
#   3. bench.py default line (C3 + CPU baseline + file-fed + C5)       -> bench.json/.log
# PART 2:
#   4. rocprofv3 --kernel-trace --stats of a 3-step C3 bench           -> prof/
#   5. rocprofv3 --pmc FETCH_SIZE on k_mam_sm (one step)               -> pmc/
#   6. FETCH_SIZE of the post-stage kernels, WRITE_SIZE of all (one
#      step)                                                            -> pmc_post/, pmc_wr/
#   7. FETCH_SIZE calibration for random 16-byte probes (randbench)    -> calib/
#   8. rocprofv3 --kernel-trace --stats of the C5 line                 -> prof_c5/
# Each GPU step has its own time limit; the chain stops at the first failure
# (a failed test lets the measurements go on; a crash or time limit not).
set -euo pipefail
TAG=${1:?tag}
PART=${2:-1}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
ARGS="--no-cpu-baseline --no-feed --no-c5"
if [ "$PART" = 1 ]; then
  cd "$R"
  rc=0
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -v --timeout 500 \
      --timeout-method thread -k "${TESTS:-mem_hg19}" > "$O/tests.log" 2>&1 || rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 python3 "$R/bench.py" --config c3mem --steps 3 > "$O/c3mem.json" 2> "$O/c3mem.log"
  timeout -k 10 420 python3 "$R/bench.py" > "$O/bench.json" 2> "$O/bench.log"
  exit $rc
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 $ARGS > "$O/prof.json" 2> "$O/prof.log"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_mam_sm -d "$O/pmc" -o pmc \
    --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 $ARGS > "$O/pmc.log" 2>&1
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_post|k_dedup|k_emit|k_scan' \
    -d "$O/pmc_post" -o pmc --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 \
    $ARGS > "$O/pmc_post.log" 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'k_mam_sm|k_post|k_dedup|k_emit|k_scan' \
    -d "$O/pmc_wr" -o pmc --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 \
    $ARGS > "$O/pmc_wr.log" 2>&1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d "$O/calib" -o pmc --output-format csv \
    -- "$R/tools/randbench" calib > "$O/calib.log" 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/prof_c5" -o run --output-format csv \
    -- python3 "$R/bench.py" --config c5 --steps 5 --warmup 1 --no-cpu-baseline \
    > "$O/prof_c5.json" 2> "$O/prof_c5.log"
exit 0
