#!/bin/bash
# Verdict r3 #8 rehearsal on one card: c4 at 8 ranks gives each rank 125,000 customers (489 blocks,
# grid 490 of 504 persistent slots, instance persist_kernel<2,5,true>).  Two processes with 62,500
# customers each on this card put the same load per CU on the same instance (2 x 246 workgroups):
# the peer-exchange persistent kernel vs the fused exchange (CLV_PERSISTENT=0), 2,000 sweeps each.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
export CLV_P2P_WORKLOAD=c4 CLV_P2P_N=125000
timeout -k 10 240 python tools/p2p_onegpu.py 2 2000 > gpurun_out/r4b_c4r8_p2p.log 2>&1 || exit $?
grep '^{' gpurun_out/r4b_c4r8_p2p.log
CLV_PERSISTENT=0 timeout -k 10 240 python tools/p2p_onegpu.py 2 2000 > gpurun_out/r4b_c4r8_fx.log 2>&1 || exit $?
grep '^{' gpurun_out/r4b_c4r8_fx.log
