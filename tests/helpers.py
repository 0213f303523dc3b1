"""Test helpers: golden-fixture loading and CBS DataFrames (test infrastructure)."""
from __future__ import annotations

import os

import numpy as np
import pandas as pd

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden(name: str):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def cdnow(name: str = "abe", n: int | None = None) -> pd.DataFrame:
    """CDNOW CBS (data/processed/cdnow_{abe,full}CBS.csv columns) + driver-side log_s / gender_F
    (trivariate/run_mcmc_full.py:60-67, trivariate/run_mcmc_abe.py:100-105)."""
    d = golden(f"cdnow_{name}_cbs.npz")
    df = pd.DataFrame({k: d[k] for k in d.files})
    if n is not None:
        df = df.iloc[:n].copy().reset_index(drop=True)
    with np.errstate(divide="ignore"):
        df["log_s"] = np.log(df["sales"] / (df["x"] + 1)).replace(-np.inf, 0.0).fillna(0.0)
    df["gender_F"] = 1 - df["gender_binary"]
    return df


def with_covariates(df: pd.DataFrame, n_cov: int, seed: int = 4242) -> pd.DataFrame:
    """c1..c{n_cov}: U(-1,1) covariate columns (the c4/c5 covariate model) added to a CBS."""
    df = df.copy()
    cov = np.random.default_rng(seed).uniform(-1.0, 1.0, size=(len(df), n_cov))
    for k in range(n_cov):
        df[f"c{k + 1}"] = cov[:, k]
    return df


def replay_case(name: str):
    """(DataFrame, covariates, fixture) of a G2 replay fixture."""
    f = golden(f"replay_{name}.npz")
    cols = dict(x=f["x"], t_x=f["t_x"], T_cal=f["T_cal"], log_s=f["log_s"])
    covs = [str(c) for c in f["covariates"]]
    for c in covs:
        cols[c] = f["cov_" + c]
    return pd.DataFrame(cols), covs, f


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)
