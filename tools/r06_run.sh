#!/bin/bash
# tools/r06_run.sh TAG [PART] -- round-6 measurement calls (each under gpurun's
# 20-minute limit; every GPU step has its own time limit, the chain stops at a
# crash or time limit, a failed test lets the measurements go on).
# PART 1: parity tests ($TESTS) + the default bench line (C3 + CPU baseline +
#   file-fed + C2 + MEM + C5)                              -> tests.log, bench.json/.log
# PART 2: FETCH_SIZE of the MEM kernels + randbench calib  -> pmc_mem/, calib/
# PART 3: rocprofv3 kernel trace of a 3-step C3 bench, FETCH_SIZE of k_mam_sm
#   and of the post stage, WRITE_SIZE, calib, C5 trace     -> prof/, pmc*/, calib/, prof_c5/
set -euo pipefail
TAG=${1:?tag}
PART=${2:-1}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
ARGS="--no-cpu-baseline --no-feed --no-c5 --no-sub"
if [ "$PART" = 1 ]; then
  cd "$R"
  rc=0
  if [ -n "${TESTS:-}" ]; then
    timeout -k 10 700 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -v --timeout 500 \
        --timeout-method thread -k "$TESTS" > "$O/tests.log" 2>&1 || rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  fi
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 python3 "$R/bench.py" ${BENCH_ARGS:-} > "$O/bench.json" 2> "$O/bench.log"
  exit $rc
fi
cd /tmp && export TMPDIR=/tmp
if [ "$PART" = 2 ]; then
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_mem|k_job' -d "$O/pmc_mem" \
      -o pmc --output-format csv -- python3 "$R/bench.py" --config c3mem --steps 1 --warmup 0 \
      --no-cpu-baseline > "$O/pmc_mem.json" 2> "$O/pmc_mem.log"
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d "$O/calib" -o pmc --output-format csv \
      -- "$R/tools/randbench" calib > "$O/calib.log" 2>&1
  exit 0
fi
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
if [ "$PART" = 4 ]; then   # + the C5 and MEM counter passes
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 200 rocprofv3 --pmc $C --kernel-include-regex 'k_upart|k_nsdir|k_mapscan|k_mapfix|k_tilebins' \
        -d "$O/pmc_c5_$C" -o pmc --output-format csv -- python3 "$R/bench.py" --config c5 --steps 1 \
        --warmup 0 --no-cpu-baseline > "$O/pmc_c5_$C.json" 2> "$O/pmc_c5_$C.log"
  done
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_mem|k_job' -d "$O/pmc_mem" \
      -o pmc --output-format csv -- python3 "$R/bench.py" --config c3mem --steps 1 --warmup 0 \
      --no-cpu-baseline > "$O/pmc_mem.json" 2> "$O/pmc_mem.log"
fi
exit 0
