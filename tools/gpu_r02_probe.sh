#!/bin/bash
# does the host block while queueing a resident run? (enqueue_probe.py), and
# the HIP API + kernel timeline of the same run
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02probe}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 -u $R/tools/enqueue_probe.py > $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
grep probe $O/probe.log
timeout -k 10 500 rocprofv3 --kernel-trace --hip-trace -d $O/trace -o run --output-format csv \
    -- python3 $R/tools/enqueue_probe.py > $O/trace.log 2>&1 || exit 1
grep probe $O/trace.log
