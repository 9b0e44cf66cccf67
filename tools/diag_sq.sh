set -e
mkdir -p gpurun_out/diag
export TMPDIR=/tmp
timeout -k 10 300 env SMASH_SM_STATS=1 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/diag/stats.json 2> gpurun_out/diag/stats.log
bash tools/profile_pmc.sh c3 gpurun_out/diag/pmc
