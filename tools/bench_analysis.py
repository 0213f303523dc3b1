"""Measurement of the posterior-analysis kernels on the c2 workload's draws.

Runs the c2 sampler (4 chains x 23,570 CDNOW customers, burnin 10,000, mcmc 10,000, thin 10 =>
4,000 level-1 draws resident in HBM), then times the *_sampler entry points (draws read in place)
with the device synchronised around each call, and the oracle (the reference's own numpy code,
restated bitwise in oracle/analysis_cpu.py) on a bounded sample of the same draws on one core.
Prints one JSON line per analysis.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    import bench
    from mcmc_clv_model_amd.sampler import HipSampler, build_problem
    from oracle import analysis_cpu as oan
    df, D, covs, chains, burnin, mcmc, thin, sink = bench.load_workload("c2")
    p = build_problem(df, covs, D)
    s = HipSampler(p, mcmc=mcmc, burnin=burnin, thin=thin, chains=chains, seed=42, draw_sink="full")
    s.run(burnin + mcmc)
    nd = chains * s.n_draws
    n = s.n
    birth = np.zeros(n)
    times = np.arange(1.0, 79.0)

    def gpu(fn, reps=3):
        fn()
        s.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        s.synchronize()
        return (time.perf_counter() - t0) / reps

    l1, _, _ = s.read_draws()
    sample = 100  # draws per chain for the CPU leg (of s.n_draws)
    draws_cpu = dict(level_1=[l1[c, :sample] for c in range(chains)])
    frac = sample / s.n_draws

    def cpu(fn):
        t0 = time.perf_counter()
        fn()
        return (time.perf_counter() - t0) / frac  # scaled to all draws

    rows = [
        ("draw_future_transactions", lambda: s.predict(T_star=39.0, seed=1),
         lambda: oan.draw_future_transactions_bi(df, draws_cpu, 39.0, seed=1)),
        ("level1_summary (Table 4 statistics)", lambda: s.level1_summary(),
         lambda: oan.table4_stats(draws_cpu)),
        ("chain_total_loglik", lambda: s.chain_total_loglik(),
         lambda: oan.chain_total_loglik(draws_cpu["level_1"], df)),
        ("weekly tracking (78 weeks)", lambda: s.track(birth, times, seed=1),
         lambda: oan.weekly_tracking(dict(level_1=[l1[c, :10] for c in range(chains)]), birth, times) if False else None),
    ]
    for name, g, c in rows:
        tg = gpu(g)
        tc = None
        if name.startswith("weekly"):
            sub = dict(level_1=[l1[c2, :5] for c2 in range(chains)])
            t0 = time.perf_counter()
            oan.weekly_tracking(sub, birth, times)
            tc = (time.perf_counter() - t0) / (5 / s.n_draws)
        else:
            tc = cpu(c)
        print(json.dumps(dict(analysis=name, workload="c2 draws: 4 chains x 1000 draws x 23570 customers",
                              gpu_s=round(tg, 6), cpu_1core_s_extrapolated=round(tc, 3),
                              cpu_sample="oracle (reference numpy code) on 100 draws/chain (tracking: 5), scaled",
                              speedup=round(tc / tg, 1))))
    s.close()


if __name__ == "__main__":
    main()
