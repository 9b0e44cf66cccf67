set -o pipefail
mkdir -p gpurun_out/r02_t2
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
( nproc; python3 -c "import os; print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; free -g ) > $R/gpurun_out/r02_t2/host.txt 2>&1
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread $R/tests/test_gpu_configs.py $R/tests/test_dropin.py > $R/gpurun_out/r02_t2/tests.log 2>&1
rc=$?
tail -5 $R/gpurun_out/r02_t2/tests.log
[ $rc -eq 0 ] && timeout -k 10 600 python3 -u $R/bench.py > $R/gpurun_out/r02_t2/bench.json 2> $R/gpurun_out/r02_t2/bench.log
rc2=$?
tail -3 $R/gpurun_out/r02_t2/bench.log
exit $(( rc | rc2 ))
