#!/bin/bash
# A/B round 2 of this session: HEAD vs the SWAR/codes + A_ROOT build, the
# prefetch / U-scan width knobs in one process, one SQ counter pass per build,
# the request-rate ceilings (randbench req)
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
bash $R/tools/abn.sh ab2 ab/libA_head.so ab/libE_knobs.so || exit 1
timeout -k 10 600 python3 -u $R/tools/sweep.py --steps 5 base SMASH_SM_PF=0 SMASH_SM_U32=0 SMASH_SM_PF=0,SMASH_SM_U32=0 base > $O/sweep.log 2>&1 || exit 1
grep "sweep\]" $O/sweep.log
for L in libA_head libE_knobs; do
  SMASH_LIB=$R/ab/$L.so timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVES SQ_INSTS_LDS \
    --kernel-include-regex k_mam_sm -d $O/sq_$L -o pmc --output-format csv -- python3 $R/tools/sweep.py --steps 1 base > $O/sq_$L.log 2>&1 || exit 1
done
timeout -k 10 300 $R/tools/randbench req > $O/randbench_req.log 2>&1 || exit 1
cat $O/randbench_req.log
