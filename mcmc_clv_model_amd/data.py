"""CBS inputs: driver-side columns and the vectorised synthetic generator for the 1M/10M configs.

* ``add_driver_columns``: log_s = log(sales / (x + 1)) with -inf/NaN -> 0
  (trivariate/run_mcmc_full.py:60-67) and gender_F = 1 - gender_binary
  (trivariate/run_mcmc_full.py:100-105).
* ``synthetic_cbs``: the model of ``generate_pareto_abe`` (bivariate/mcmc.py:95-187) in closed
  form instead of a per-customer event loop: x ~ Poisson(lambda * min(tau, T)) and, given x > 0,
  t_x = min(tau, T) * U^(1/x) (the maximum of x uniform event times).  Parameters follow
  SURVEY.md §8d (c4/c5).
"""
from __future__ import annotations

import numpy as np
import pandas as pd


def add_driver_columns(df: pd.DataFrame) -> pd.DataFrame:
    df = df.copy()
    if "sales" in df and "log_s" not in df:
        with np.errstate(divide="ignore", invalid="ignore"):
            df["log_s"] = np.log(df["sales"] / (df["x"] + 1)).replace(-np.inf, 0.0).fillna(0.0)
    if "gender_binary" in df and "gender_F" not in df:
        df["gender_F"] = 1 - df["gender_binary"]
    return df


def synthetic_cbs(n: int, K: int, D: int = 2, seed: int = 20250718, T_range=(27.0, 38.86)) -> pd.DataFrame:
    """Synthetic CBS with K-1 U(-1,1) covariates named c1..c{K-1} (plus log_s when D == 3)."""
    rng = np.random.default_rng(seed)
    X = np.column_stack([np.ones(n), rng.uniform(-1.0, 1.0, size=(n, K - 1))])
    beta = np.zeros((K, D))
    beta[0, :2] = (-3.5, -3.7)
    if D == 3:
        beta[0, 2] = 3.24
    beta[1:, :] = rng.normal(0.0, 0.1, size=(K - 1, D))
    gamma = np.zeros((D, D))
    gamma[:2, :2] = [[1.4, 0.2], [0.2, 2.5]]
    if D == 3:
        gamma[2, 2] = 0.47
    theta = X @ beta + rng.multivariate_normal(np.zeros(D), gamma, size=n)
    lam, mu = np.exp(theta[:, 0]), np.exp(theta[:, 1])
    tau = rng.exponential(1.0 / mu)
    T = rng.uniform(*T_range, size=n)
    L = np.minimum(tau, T)
    x = rng.poisson(lam * L)
    u = rng.random(n)
    with np.errstate(divide="ignore"):
        t_x = np.where(x > 0, L * u ** (1.0 / np.maximum(x, 1)), 0.0)
    df = pd.DataFrame(dict(x=x.astype(np.int64), t_x=t_x, T_cal=T))
    for k in range(1, K):
        df[f"c{k}"] = X[:, k]
    if D == 3:
        df["log_s"] = theta[:, 2] + rng.normal(0.0, np.sqrt(0.47), size=n)
    return df
