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


# ---------------------------------------------------------------------------------------------
# On-device data preparation (csrc/elog.hip)
# ---------------------------------------------------------------------------------------------
def elog2cbs(elog: pd.DataFrame, units="week", T_cal=None, T_tot=None, *, device: int = -1) -> pd.DataFrame:
    """Event log -> CBS on the GPU, drop-in for ``src/models/utils/elog2cbs2param.py:33-94``: same
    arguments, validation errors and columns (cust, x, t_x, litt, sales, sales_x, first, T_cal and,
    with a hold-out period, T_star, x_star, sales_star); same-day transactions are merged with their
    sales summed.  The sort, merge and per-customer statistics run in ``clv_elog2cbs``."""
    import ctypes
    from . import _lib
    from ._lib import check
    if not isinstance(elog, pd.DataFrame):
        raise ValueError("elog must be a pandas DataFrame")
    if "cust" not in elog.columns or "date" not in elog.columns:
        raise ValueError("elog must contain 'cust' and 'date' columns")
    if elog.empty:
        return pd.DataFrame(columns=["cust", "x", "t.x", "litt", "first", "T.cal"])
    dates = pd.to_datetime(elog["date"])
    if "sales" in elog.columns and not pd.api.types.is_numeric_dtype(elog["sales"]):
        raise ValueError("'sales' column must be numeric")
    T_cal_ts = dates.max() if T_cal is None else pd.to_datetime(T_cal)
    T_tot_ts = dates.max() if T_tot is None else pd.to_datetime(T_tot)
    unit_ns = int(np.timedelta64(1, units).astype("timedelta64[ns]").astype(np.int64))
    L = _lib.lib()
    if _lib.device_count() < 1:
        raise _lib.ClvError("no HIP device visible; elog2cbs has no CPU fallback")
    codes, uniques = pd.factorize(elog["cust"], sort=True)  # sorted codes keep groupby's key order
    n = len(elog)
    cust = np.ascontiguousarray(codes.astype(np.int64))
    date_ns = np.ascontiguousarray(dates.to_numpy(dtype="datetime64[ns]").view(np.int64))
    sales = (np.ascontiguousarray(elog["sales"].to_numpy(np.float64)) if "sales" in elog.columns else None)
    o = dict(cust=np.empty(n, np.int64), x=np.empty(n, np.int64), t_x=np.empty(n), litt=np.empty(n),
             sales=np.empty(n), sales_x=np.empty(n), first=np.empty(n, np.int64), T_cal=np.empty(n),
             T_star=np.empty(n), x_star=np.empty(n, np.int64), sales_star=np.empty(n))
    nc = ctypes.c_int64()
    i64 = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))  # noqa: E731
    dp = _lib.dptr
    check(L.clv_elog2cbs(int(device), n, i64(cust), i64(date_ns), dp(sales), unit_ns,
                         int(T_cal_ts.value), int(T_tot_ts.value), ctypes.byref(nc), i64(o["cust"]), i64(o["x"]),
                         dp(o["t_x"]), dp(o["litt"]), dp(o["sales"]), dp(o["sales_x"]), i64(o["first"]),
                         dp(o["T_cal"]), dp(o["T_star"]), i64(o["x_star"]), dp(o["sales_star"])))
    k = nc.value
    out = pd.DataFrame(dict(cust=uniques[o["cust"][:k]], x=o["x"][:k], t_x=o["t_x"][:k], litt=o["litt"][:k],
                            sales=o["sales"][:k], sales_x=o["sales_x"][:k],
                            first=pd.to_datetime(o["first"][:k]), T_cal=o["T_cal"][:k]))
    if "sales" not in elog.columns:
        out["sales"] = out["sales"].astype(np.int64)  # the reference sums the integer 1s it inserts
        out["sales_x"] = out["sales_x"].astype(np.int64)
    if T_cal_ts < T_tot_ts:
        out["T_star"] = o["T_star"][:k]
        out["x_star"] = o["x_star"][:k].astype(np.float64)  # left merge + fillna: float like the reference
        out["sales_star"] = o["sales_star"][:k]
    return out


def generate_pareto_abe(n: int, T_cal, T_star, beta, gamma, covars=None, seed=None, *, return_elog: bool = True,
                        device: int = -1):
    """Abe (2009) synthetic data on the GPU, drop-in for ``generate_pareto_abe``
    (bivariate/mcmc.py:95-187): returns (cbs, elog) with the reference's columns — cust, x, t_x,
    T_cal, lambda_true, mu_true, tau_true, alive_true, x_star (or x_star<h> per horizon), cov0..
    Same model and parameters; random draws from a Philox stream keyed by ``seed`` (the reference
    uses numpy's Generator), so outputs agree in distribution.  ``return_elog=False`` skips the
    event log (the CBS is formed on device either way)."""
    import ctypes
    from . import _lib
    from ._lib import check
    from .sampler import resolve_seed
    beta = np.asarray(beta, dtype=float)
    K, D = beta.shape
    assert D == 2, "beta must have two columns (log‑lambda, log‑mu)"
    gamma = np.ascontiguousarray(np.asarray(gamma, dtype=float))
    cov = None
    if covars is not None:
        cov = np.asarray(covars, dtype=float)
        if cov.ndim == 1:
            cov = cov[:, None]
        if not np.allclose(cov[:, 0], 1):
            cov = np.column_stack([np.ones(cov.shape[0]), cov])
        if cov.shape != (n, K):
            raise ValueError("covars has wrong shape relative to beta")
        cov = np.ascontiguousarray(cov)
    T_cal = np.asarray(T_cal, dtype=float).ravel()
    if T_cal.size == 1:
        T_cal = np.full(n, T_cal.item())
    T_cal = np.ascontiguousarray(T_cal)
    T_star = np.ascontiguousarray(np.asarray(T_star, dtype=float).ravel())
    L = _lib.lib()
    if _lib.device_count() < 1:
        raise _lib.ClvError("no HIP device visible; generate_pareto_abe has no CPU fallback")
    s = resolve_seed(seed)
    x = np.empty(n, np.int64)
    t_x, lam, mu, tau = (np.empty(n) for _ in range(4))
    alive = np.empty(n, np.uint8)
    x_star = np.empty((T_star.size, n), np.int64)
    cov_out = np.empty((n, K))
    n_ev = np.empty(n, np.int64)
    i64 = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))  # noqa: E731
    dp = _lib.dptr
    u8 = alive.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
    args = [int(device), n, K, dp(np.ascontiguousarray(beta)), dp(gamma), dp(cov), dp(T_cal), T_star.size, dp(T_star),
            s, i64(x), dp(t_x), dp(lam), dp(mu), dp(tau), u8, i64(x_star), dp(cov_out), i64(n_ev)]
    check(L.clv_generate_pareto_abe(*args, None, 0, None, None))
    elog = None
    if return_elog:
        off = np.ascontiguousarray(np.concatenate([[0], np.cumsum(n_ev)[:-1]]).astype(np.int64))
        rows = int(n_ev.sum())
        ec = np.empty(rows, np.int64)
        et = np.empty(rows)
        check(L.clv_generate_pareto_abe(*args, i64(off), rows, i64(ec), dp(et)))
        elog = pd.DataFrame(dict(cust=ec.astype(float), t=et))
    cbs = pd.DataFrame(dict(cust=np.arange(1, n + 1, dtype=float), x=x, t_x=t_x, T_cal=float(T_cal.max())))
    cbs["lambda_true"], cbs["mu_true"], cbs["tau_true"] = lam, mu, tau
    cbs["alive_true"] = alive.astype(bool)
    for k, ts in enumerate(T_star):
        col = f"x_star{int(ts)}" if T_star.size > 1 else "x_star"
        cbs[col] = x_star[k]
    for j in range(K):
        cbs[f"cov{j}"] = cov_out[:, j]
    return cbs, elog
