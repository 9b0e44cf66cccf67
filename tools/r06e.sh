set -euo pipefail
cd /root/repo
mkdir -p gpurun_out/r06e
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_phases.py tests/test_gpu_feed.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06e/parity.log 2>&1
TESTS='production or idx8 or hg19_counts' bash tools/r06_ab.sh r06e 'libsmashgpu_base.so -'
