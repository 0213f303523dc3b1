# Scratch GPU session script (overwritten per experiment).
# Round 6: the persistent level-2 workgroup's coalesced poll, group size 4 / 8 / all (build/gc8,
# build/gc64) vs the lane-per-block poll (build/nocoal): wall us per sweep (persistent forced).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
L=$PWD/mcmc_clv_model_amd/libclvmcmc.so
for rep in 1 2; do for lib in $PWD/build/nocoal/libclvmcmc.so $L $PWD/build/gc8/libclvmcmc.so $PWD/build/gc64/libclvmcmc.so; do
  for W in c4_shard8; do
    CLV_PERSISTENT=1 CLV_LIB_PATH=$lib timeout -k 10 300 python tools/persist_breakdown.py $W 3000 > gpurun_out/c_wall.txt 2>&1 || { tail -5 gpurun_out/c_wall.txt; exit 1; }
    echo $W $lib $(grep "wall:" gpurun_out/c_wall.txt)
  done
done; done
