"""Driver counterpart of the reference's run scripts (src/models/*/run_mcmc_{abe,full}.py).

    python -m mcmc_clv_model_amd.run_mcmc --cbs cdnow_abeCBS.csv --model bi --covariates first_sales_scaled \
        --mcmc 4000 --burnin 10000 --thin 1 --chains 4 --seed 42 --out abe_bi_m2.pkl --runtimes mcmc_runtimes.csv

Reads the CBS CSV (run_mcmc_abe.py:42-43), adds the driver-side columns log_s
(trivariate/run_mcmc_full.py:60-67) and gender_F (trivariate/run_mcmc_full.py:100-105), runs the
sampler on the GPU, pickles the draws dict (run_mcmc_abe.py:76-77) and records the runtime in the
(model, runtime) CSV format of outputs/excel/mcmc_runtimes.csv (run_mcmc_abe.py:106-127).
"""
from __future__ import annotations

import argparse
import os
import pickle
import time

import pandas as pd

from .bivariate import mcmc_draw_parameters
from .data import add_driver_columns
from .trivariate import mcmc_draw_parameters_rfm_m


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--cbs", required=True, help="CBS CSV (columns x, t_x, T_cal, ...)")
    ap.add_argument("--model", choices=("bi", "tri"), default="bi")
    ap.add_argument("--covariates", nargs="*", default=[])
    ap.add_argument("--mcmc", type=int, default=4000)
    ap.add_argument("--burnin", type=int, default=10000)
    ap.add_argument("--thin", type=int, default=1)
    ap.add_argument("--chains", type=int, default=4)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--trace", type=int, default=1000)
    ap.add_argument("--n-mh-steps", type=int, default=20)
    ap.add_argument("--draw-sink", choices=("full", "summary", "none"), default="full")
    ap.add_argument("--out", help="pickle path for the draws dict")
    ap.add_argument("--runtimes", help="CSV of (model, runtime) rows to update")
    ap.add_argument("--name", help="model name in the runtimes CSV (default: <file stem>_<model>)")
    a = ap.parse_args(argv)

    cbs = add_driver_columns(pd.read_csv(a.cbs))
    fn = mcmc_draw_parameters if a.model == "bi" else mcmc_draw_parameters_rfm_m
    t0 = time.time()
    draws = fn(cbs, a.covariates, mcmc=a.mcmc, burnin=a.burnin, thin=a.thin, chains=a.chains, seed=a.seed,
               trace=a.trace, n_mh_steps=a.n_mh_steps, draw_sink=a.draw_sink)
    runtime = time.time() - t0
    print(f"Model runtime: {runtime:.2f} seconds")
    if a.out:
        with open(a.out, "wb") as f:
            pickle.dump(draws, f)
    if a.runtimes:
        name = a.name or f"{os.path.splitext(os.path.basename(a.cbs))[0]}_{a.model}"
        df = pd.read_csv(a.runtimes) if os.path.exists(a.runtimes) else pd.DataFrame(columns=["model", "runtime"])
        df = df[df.model != name]
        df = pd.concat([df, pd.DataFrame([{"model": name, "runtime": runtime}])], ignore_index=True)
        df.to_csv(a.runtimes, index=False)
    return draws


if __name__ == "__main__":
    main()
