set -uo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ab1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread $R/tests/test_gpu_parity.py $R/tests/test_gpu_modes.py > $R/gpurun_out/ab1/tests.log 2>&1 || { tail -20 $R/gpurun_out/ab1/tests.log; exit 1; }
tail -1 $R/gpurun_out/ab1/tests.log
bash $R/tools/abn.sh ab1 ab/libA_head.so ab/libB_codes.so ab/libC_swar.so
