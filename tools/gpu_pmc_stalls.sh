#!/bin/bash
# Stall/issue counters of the sweep kernel (separate --pmc passes, kernel-trace only).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; export TMPDIR=/tmp
W=${1:-c2}
mkdir -p gpurun_out/pmc_$W
K=${2:-persist_kernel}
# two dispatches (50 warm-up + 200 sweeps) of the workload only: tools/pmc_run.py
B="python3 $R/tools/pmc_run.py $W 50 200"
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES" \
         "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_VMEM" \
         "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM" \
         "GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INSTS_SMEM SQ_INST_CYCLES_SMEM SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P -d $R/gpurun_out/pmc_$W/p$i -o run --output-format csv -- $B > gpurun_out/pmc_${W}_p$i.log 2>&1; rc=$?; echo ${W}_p${i}_rc=$rc
  [ $rc -eq 0 ] || exit $rc
  python3 $R/tools/pmc_reduce.py $R/gpurun_out/pmc_$W/p$i $K && rm -rf $R/gpurun_out/pmc_$W/p$i
done
exit 0
