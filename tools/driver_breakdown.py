"""Where the driver's 20-sweep c2 step goes (bench.py --steps 20 --warmup 5): host time until
clv_run returns, then torch.cuda.synchronize(), next to the launch's event-timed duration; and the
same launch right after a long one (GPU clocks ramped) to separate the clock ramp from fixed costs.
Env: REPS, NSWEEPS, TIMING (1: events around the timed launch, as bench.py; 0: none), LABEL.
One JSON line per case into stdout, then a median line per case."""
import ctypes
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from bench import load_workload  # noqa: E402
from mcmc_clv_model_amd.sampler import HipSampler, build_problem  # noqa: E402


def main():
    reps = int(os.environ.get("REPS", "5"))
    n = int(os.environ.get("NSWEEPS", "20"))
    timing = os.environ.get("TIMING", "1") == "1"
    label = os.environ.get("LABEL", "")
    df, D, covs, chains, burnin, mcmc, thin, sink = load_workload("c2")
    p = build_problem(df, covs, D)
    s = HipSampler(p, mcmc=mcmc, burnin=burnin, thin=thin, chains=chains, seed=42, draw_sink=sink, device=0)
    s.run(5)
    s.synchronize()
    rows = {}
    cases = os.environ.get("CASES", "cold,after_long").split(",")
    # after_busy: 2,000 sweeps' worth of unrelated GPU work (fp64 matmuls) then the driver's 5
    # warm-up sweeps -- the GPU's clocks warm, the sampler's caches as cold as in "cold";
    # long_then_idle: 2,000 sweeps then 0.2 s idle then 5 sweeps -- the caches warm, the clocks
    # after the same idle gap as "cold"
    a = torch.randn(2048, 2048, dtype=torch.float64, device="cuda:0")
    for case in cases:
        for r in range(reps):
            if case == "after_long":
                s.run(2000)
            elif case == "after_busy":
                b = a
                t_end = time.perf_counter() + 0.021
                while time.perf_counter() < t_end:
                    b = torch.tanh(a @ b * 1e-3)
                    torch.cuda.synchronize()
                s.run(5)
            elif case == "long_then_idle":
                s.run(2000)
                s.synchronize()
                time.sleep(0.2)
                s.run(5)
            else:
                time.sleep(0.2)  # the driver's command: seconds of host work before the timed step
                s.run(5)
            s.synchronize()
            torch.cuda.synchronize()
            if timing:
                s.set_timing(True)
            t0 = time.perf_counter()
            s.run(n)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            hn = (ctypes.c_int64 * 8)()
            assert s._L.clv_debug_host_times(s.h, hn) == 0
            h = [x / 1e3 for x in hn]  # us
            host = dict(setdev=round(h[1] - h[0], 2), pre_launch=round(h[2] - h[1], 2), launch=round(h[3] - h[2], 2),
                        post_launch=round(h[4] - h[3], 2), wait=round(h[5] - h[4], 2), epilogue=round(h[6] - h[5], 2),
                        outside=round((t1 - t0) * 1e6 - (h[6] - h[0]), 2))
            kt = s.kernel_time() if timing else {"sweep_ms": float("nan")}
            if timing:
                s.set_timing(False)
            row = dict(label=label, case=case, rep=r, sweeps=n, run_us=round((t1 - t0) * 1e6, 2),
                       sync_us=round((t2 - t1) * 1e6, 2), wall_us=round((t2 - t0) * 1e6, 2),
                       kernel_us=round(kt["sweep_ms"] * 1e3, 2), us_per_step=round((t2 - t0) * 1e6 / n, 3),
                       host=host)
            rows.setdefault(case, []).append(row)
            print(json.dumps(row), flush=True)
    for case, rs in rows.items():
        med = {k: round(statistics.median(x[k] for x in rs), 2) for k in ("run_us", "sync_us", "wall_us", "kernel_us",
                                                                        "us_per_step")}
        med["host"] = {k: round(statistics.median(x["host"][k] for x in rs), 2) for k in rs[0]["host"]}
        print(json.dumps(dict(label=label, case=case, median=med,
                              env={k: v for k, v in os.environ.items() if k.startswith("CLV_")})), flush=True)
    s.close()


if __name__ == "__main__":
    main()
