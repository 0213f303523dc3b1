# Scratch GPU session script (overwritten per experiment).
# Round 6: the driver's command with the clock settled by the sampler's own sweeps vs fp64 matmuls.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do for w in sampler matmul; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --settle-work $w > gpurun_out/drv_$w.log 2>&1 || { tail -20 gpurun_out/drv_$w.log; exit 1; }
  python - $w <<'PY'
import json,sys
l=json.loads(open(f"gpurun_out/drv_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print(sys.argv[1], "value=%.4e" % l["value"], "us/step=%.3f" % (l["ms_per_step"]*1e3), "clk", l["gpu_clock_ghz"], "kernel_us/sweep", l["roofline"]["sweep_kernel_us"], "cold", round(l["cold"]["ms_per_step"]*1e3,2), "c4", round(l["configs"]["c4"]["ms_per_step"]*1e3,2), l["configs"]["c4"]["gpu_clock_ghz"])
PY
done; done
