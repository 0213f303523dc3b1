# Scratch GPU session script (overwritten per experiment; the round-6 diagnostics ran from it).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
L=$PWD/mcmc_clv_model_amd
for rep in 1 2; do for lib in $L/libclvmcmc.so $PWD/build/l2alone/libclvmcmc.so; do for w in c4_shard8 c2; do
  CLV_PERSISTENT=1 CLV_LIB_PATH=$lib timeout -k 10 300 python tools/persist_breakdown.py $w 3000 > gpurun_out/b_wall.txt 2>&1 || exit $?
  echo $w $lib $(tail -1 gpurun_out/b_wall.txt)
done; done; done
timeout -k 10 600 python tools/persist_crossover.py > gpurun_out/b_crossover1.jsonl 2>&1 || exit $?
CROSSOVER_SET=2 timeout -k 10 600 python tools/persist_crossover.py > gpurun_out/b_crossover2.jsonl 2>&1 || exit $?
cat gpurun_out/b_crossover1.jsonl gpurun_out/b_crossover2.jsonl | grep -v Warn | cut -c1-200
