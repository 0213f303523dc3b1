"""Minimal driver for the PMC passes of tools/gpu_pmc_stalls.sh: one workload's sampler, a
`warm`-sweep call then a `timed`-sweep call (persistent kernel: exactly two dispatches), nothing
else -- bench.py's scaling legs and c1 leg would add thousands of dispatches to every pass.

    python3 tools/pmc_run.py c2 50 200        (c4stored: the c4 sampler with burn-in 0)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    w = sys.argv[1] if len(sys.argv) > 1 else "c2"
    warm = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    timed = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    import bench
    from mcmc_clv_model_amd.sampler import HipSampler, build_problem
    stored = w.endswith("stored")  # "<w>stored": burn-in 0, every sweep a stored sweep (bi:402-428)
    w = w[:-len("stored")] if stored else w
    df, D, covs, chains, burnin, mcmc, thin, sink = bench.load_workload(w)
    if stored:
        mcmc, burnin = mcmc + burnin, 0
    p = build_problem(df, covs, D)
    s = HipSampler(p, mcmc=max(mcmc, warm + timed), burnin=burnin, thin=thin, chains=chains, seed=42,
                   draw_sink=sink, device=0)
    s.run(warm)
    s.synchronize()
    s.run(timed)
    s.synchronize()
    info = s.launch_info()
    print(f"{w}: {warm}+{timed} sweeps, persistent={info['persistent']}", flush=True)


if __name__ == "__main__":
    main()
