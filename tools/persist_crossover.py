#!/usr/bin/env python
"""Persistent kernel vs launch-per-sweep at world size 1 as the resident grid fills the chip
(verdict r3 #8: c4 at 8 ranks is 125,000 customers per GPU).  Synthetic problems
(mcmc_clv_model_amd.data.synthetic_cbs), CLV_PERSISTENT=1 / 0 at create, 200 warm-up sweeps then
1,000 timed sweeps; one JSON line per (model, size, path) with the grid's workgroups per CU."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CASES = [(2, 2, 4, 20000), (2, 2, 4, 26000), (2, 2, 4, 30000),
         (2, 5, 1, 60000), (2, 5, 1, 90000), (2, 5, 1, 110000), (2, 5, 1, 125000),
         (3, 3, 4, 20000), (3, 3, 4, 26000)]
if os.environ.get("CROSSOVER_SET") == "2":  # chains vs covariates vs model, separated
    CASES = [(2, 5, 4, 20000), (2, 5, 4, 26000), (2, 2, 1, 60000), (2, 2, 1, 90000), (2, 2, 1, 110000),
             (2, 9, 1, 60000), (2, 9, 1, 90000), (3, 9, 1, 60000), (3, 3, 1, 90000), (3, 3, 1, 110000),
             (2, 2, 2, 60000), (2, 2, 4, 28000)]


def main():
    import torch
    from mcmc_clv_model_amd.data import synthetic_cbs
    from mcmc_clv_model_amd.sampler import HipSampler, build_problem
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    for D, K, chains, n in CASES:
        p = build_problem(synthetic_cbs(n, K, D, seed=7), [f"c{k}" for k in range(1, K)], D)
        for mode in ("1", "0"):
            os.environ["CLV_PERSISTENT"] = mode
            s = HipSampler(p, mcmc=5000, burnin=5000, thin=1, chains=chains, seed=42, draw_sink="summary")
            info = s.launch_info()
            s.run(200)
            s.synchronize()
            t0 = time.perf_counter()
            s.run(1000)
            s.synchronize()
            dt = (time.perf_counter() - t0) / 1000
            nb = -(-n // 256)
            print(json.dumps(dict(D=D, K=K, chains=chains, n=n, grid_wgs=chains * (nb + 1),
                                  wgs_per_cu=round(chains * (nb + 1) / n_cu, 3), requested=mode,
                                  persistent=info["persistent"], us_per_sweep=round(dt * 1e6, 3))), flush=True)
            s.close()
    os.environ.pop("CLV_PERSISTENT", None)


if __name__ == "__main__":
    main()
