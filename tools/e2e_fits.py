"""End-to-end drop-in fits on the GPU next to the reference's published runtimes.

Each fit is the reference driver's exact call — mcmc_draw_parameters(...) with its chains, seed,
trace and n_mh_steps — timed from the call to the returned dict of numpy arrays (upload, every
sweep, the D2H copy of all stored draws, the per-chain array split).  The published numbers are
the reference's own `outputs/excel/mcmc_runtimes.csv` (the authors' CPU, numpy, chains run one
after another), copied below as constants.

  abe_bi_M1  run_mcmc_abe.py:61-71   cdnow_abeCBS (2,357), M1, 4 chains, 10,000 + 4,000, thin 1
  abe_bi_M2  run_mcmc_abe.py:85-95   same, covariate first_sales_scaled
  c2 / c3    BASELINE configs[1-2]   full CDNOW (23,570), 4 chains, 10,000 + 10,000, thin 10
             (no published runtime: the `full_bi_*` rows ran on a `cdnow_cbs_full.csv` that is not
             in the reference, so they are not comparable)

Usage (GPU box): python tools/e2e_fits.py > gpurun_out/e2e.jsonl
"""
import contextlib
import io
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PUBLISHED_S = {"abe_bi_M1": 206.85397124290463, "abe_bi_M2": 208.458181142807}  # mcmc_runtimes.csv:2-3

FITS = [
    ("abe_bi_M1", "bi", "abe", [], dict(mcmc=4000, burnin=10000, thin=1, chains=4)),
    ("abe_bi_M2", "bi", "abe", ["first_sales_scaled"], dict(mcmc=4000, burnin=10000, thin=1, chains=4)),
    ("c2", "bi", "full", ["first_sales_scaled"], dict(mcmc=10000, burnin=10000, thin=10, chains=4)),
    ("c3", "tri", "full", ["gender_F", "age_scaled"], dict(mcmc=10000, burnin=10000, thin=10, chains=4)),
]


def main():
    import numpy as np
    from mcmc_clv_model_amd import mcmc_draw_parameters, mcmc_draw_parameters_rfm_m
    from tests.helpers import cdnow
    for name, kind, data, covs, kw in FITS:
        df = cdnow(data)
        fn = mcmc_draw_parameters if kind == "bi" else mcmc_draw_parameters_rfm_m
        walls = []
        for rep in range(2):  # first call includes the one-time library / device initialisation
            out = io.StringIO()
            t0 = time.perf_counter()
            with contextlib.redirect_stdout(out):
                d = fn(df, covs, seed=42, trace=1000, n_mh_steps=20, **kw)
            walls.append(time.perf_counter() - t0)
            assert all(np.isfinite(a).all() for a in d["level_1"])
            lines = out.getvalue().splitlines()
            rec_bytes, rec_ll = int(sum(a.nbytes for a in d["level_1"])), float(d["log_likelihood"])
            del d  # freeing the previous call's multi-GB result is not the next call's cost
        sweeps = kw["burnin"] + kw["mcmc"]
        n = len(df)
        rec = dict(fit=name, n_customers=n, covariates=covs, sweeps=sweeps, **kw, seed=42, trace=1000,
                   wall_s=round(walls[1], 4), wall_first_call_s=round(walls[0], 4),
                   customer_sweeps_per_s=kw["chains"] * n * sweeps / walls[1],
                   level1_bytes=rec_bytes, trace_lines=len(lines), log_likelihood=rec_ll)
        if name in PUBLISHED_S:
            rec["published_s"] = PUBLISHED_S[name]
            rec["speedup_vs_published"] = round(PUBLISHED_S[name] / walls[1], 1)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
