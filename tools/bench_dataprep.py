"""Measurement of the data-preparation kernels at scale, with the reference's
own Python code timed on a bounded sample on one core (extrapolated linearly).

* generate_pareto_abe: 10M customers (c5 scale), CBS only; reference: the per-customer loop of
  bivariate/mcmc.py:150-162 on 20,000 customers (oracle: the reference function itself is not
  shipped to the GPU box, so the timed CPU leg is its restatement in this script's loop).
* elog2cbs: a 20M-event log from the generator (dates = t weeks after 1997-01-01); reference:
  pandas code of utils/elog2cbs2param.py restated (oracle-free: timed on 1M events).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402


def ref_generate_loop(n, lam, tau, T_cal, T_star_max, rng):
    """bivariate/mcmc.py:150-162 (the event loop that dominates the reference generator)."""
    rows = 0
    for i in range(n):
        lam_i, tau_i = float(lam[i]), float(tau[i])
        min_T = min(T_cal + T_star_max, tau_i)
        t_acc, ts = 0.0, [0.0]
        while t_acc < min_T:
            t_acc += rng.exponential(scale=1.0 / lam_i)
            ts.append(t_acc)
        ts = np.array(ts)
        ts = ts[ts <= tau_i]
        rows += int((ts <= T_cal + T_star_max).sum())
    return rows


def ref_elog2cbs(elog, units, T_cal, T_tot):
    """utils/elog2cbs2param.py:36-93, restated (same pandas calls)."""
    elog = elog.copy()
    elog = elog.groupby(["cust", "date"], as_index=False).agg({"sales": "sum"})
    elog = elog.sort_values(["cust", "date"])
    elog["first"] = elog.groupby("cust")["date"].transform("min")
    elog["t"] = (elog["date"] - elog["first"]) / np.timedelta64(1, units)
    elog["itt"] = elog.groupby("cust")["t"].diff().fillna(0)
    cal = elog[elog["date"] <= T_cal]
    out = cal.groupby("cust").agg(x=("date", lambda d: len(d) - 1), t_x=("t", "max"),
                                  litt=("itt", lambda x: np.log(x[x > 0]).sum()), sales=("sales", "sum"),
                                  sales_x=("sales", lambda s: s.iloc[1:].sum() if len(s) > 1 else 0),
                                  first=("first", "first")).reset_index()
    return out


def main():
    from mcmc_clv_model_amd.data import elog2cbs, generate_pareto_abe
    beta = np.array([[-0.5, -3.7], [0.1, 0.05]])
    gamma = np.array([[1.4, 0.2], [0.2, 2.5]])
    n = 10_000_000
    generate_pareto_abe(1000, 38.86, [39.0], beta, gamma, seed=1, return_elog=False)  # warm-up
    t0 = time.perf_counter()
    cbs, _ = generate_pareto_abe(n, 38.86, [39.0], beta, gamma, seed=1, return_elog=False)
    tg = time.perf_counter() - t0
    ns = 20_000
    rng = np.random.default_rng(1)
    t0 = time.perf_counter()
    ref_generate_loop(ns, cbs["lambda_true"].to_numpy()[:ns], cbs["tau_true"].to_numpy()[:ns], 38.86, 39.0, rng)
    tc = (time.perf_counter() - t0) * n / ns
    print(json.dumps(dict(dataprep="generate_pareto_abe", n_customers=n, gpu_s=round(tg, 3),
                          cpu_1core_s_extrapolated=round(tc, 1),
                          cpu_sample="reference event loop (bi:150-162) on 20,000 customers, scaled",
                          speedup=round(tc / tg, 1), note="GPU time includes the host copies of the CBS")))
    nc = 2_000_000
    c2, el = generate_pareto_abe(nc, 38.86, [39.0], beta, gamma, seed=2)
    el = el[el["cust"] <= nc]
    base = np.datetime64("1997-01-01", "ns")
    elog = pd.DataFrame(dict(cust=el["cust"].astype(np.int64).to_numpy(),
                             date=base + (el["t"].to_numpy() * 7 * 86400e9).astype("timedelta64[ns]"),
                             sales=np.round(np.abs(np.random.default_rng(3).normal(30, 10, len(el))), 2)))
    kw = dict(units="W", T_cal="1997-09-30", T_tot="1998-06-30")
    elog2cbs(elog.iloc[:10000], **kw)  # warm-up
    t0 = time.perf_counter()
    elog2cbs(elog, **kw)
    tg = time.perf_counter() - t0
    m = 1_000_000
    sub = elog[elog["cust"] <= elog["cust"].iloc[m]]
    t0 = time.perf_counter()
    ref_elog2cbs(sub, "W", pd.Timestamp("1997-09-30"), pd.Timestamp("1998-06-30"))
    tc = (time.perf_counter() - t0) * len(elog) / len(sub)
    print(json.dumps(dict(dataprep="elog2cbs", n_events=len(elog), gpu_s=round(tg, 3),
                          cpu_1core_s_extrapolated=round(tc, 1),
                          cpu_sample=f"reference pandas code on {len(sub)} events, scaled",
                          speedup=round(tc / tg, 1), note="GPU time includes host<->device copies")))


if __name__ == "__main__":
    main()
