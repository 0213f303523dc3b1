"""Row f4 (data preparation on device, csrc/elog.hip) through the C ABI, against the reference's
own outputs (tests/golden/elog_abe.npz, generator_bi.npz — written by make_goldens.py from
utils/elog2cbs2param.py and bivariate/mcmc.py:95-187)."""
import numpy as np
import pandas as pd
import pytest
from scipy import stats

from tests.helpers import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def elog():
    from mcmc_clv_model_amd import _lib
    _lib.lib()
    assert _lib.device_count() >= 1, "no HIP device: GPU tests must run on an MI355X"
    f = np.load(f"{GOLDEN}/elog_abe.npz", allow_pickle=False)
    df = pd.DataFrame(dict(cust=f["cust"], date=pd.to_datetime(f["date_ns"]), sales=f["sales"]))
    return f, df


def _bits(a):
    return np.asarray(a, dtype=np.float64).view(np.uint64)


@pytest.mark.parametrize("tag,kw", [("hold", dict(units="W", T_cal="1997-09-30", T_tot="1998-06-30")),
                                    ("nohold", dict(units="D"))])
def test_elog2cbs_matches_reference(elog, tag, kw):
    """Integer columns, dates and the ratio columns t_x / T_cal / T_star bit for bit (the same
    int64-ns -> float64 division); sums (sales, litt) <= 1e-12 relative (pandas' compensated group
    sums and numpy's pairwise sums vs a sequential sum; ocml vs glibc log)."""
    from mcmc_clv_model_amd.data import elog2cbs
    f, df = elog
    got = elog2cbs(df, **kw)
    assert np.array_equal(got["cust"].to_numpy(), f[f"{tag}_cust"])
    assert np.array_equal(got["x"].to_numpy(), f[f"{tag}_x"])
    assert np.array_equal(got["first"].to_numpy(dtype="datetime64[ns]").view(np.int64), f[f"{tag}_first"])
    for c in ("t_x", "T_cal") + (("T_star",) if tag == "hold" else ()):
        assert np.array_equal(_bits(got[c]), _bits(f[f"{tag}_{c}"])), c
    for c in ("sales", "sales_x", "litt") + (("sales_star",) if tag == "hold" else ()):
        np.testing.assert_allclose(got[c].to_numpy(), f[f"{tag}_{c}"], rtol=1e-12, atol=1e-12, err_msg=c)
    if tag == "hold":
        assert np.array_equal(got["x_star"].to_numpy(), f["hold_x_star"])
    else:
        assert "x_star" not in got.columns


def test_elog2cbs_without_sales_and_validation(elog):
    from mcmc_clv_model_amd.data import elog2cbs
    f, df = elog
    got = elog2cbs(df[["cust", "date"]], units="W", T_cal="1997-09-30", T_tot="1998-06-30")
    for c in ("x", "sales", "sales_x", "x_star", "sales_star"):
        assert np.array_equal(got[c].to_numpy(), f[f"nosales_{c}"]), c
    with pytest.raises(ValueError):
        elog2cbs(df.drop(columns=["cust"]))
    with pytest.raises(ValueError):
        elog2cbs(df.assign(sales="a"))
    assert elog2cbs(df.iloc[:0]).empty


def test_generator_matches_reference_in_distribution():
    """Same model and parameters as the reference sample (20,000 customers): two-sample KS on the
    true parameters and t_x, chi-square on x and the hold-out counts, alive share within 4 sd;
    the returned event log is consistent with the CBS exactly."""
    from mcmc_clv_model_amd.data import generate_pareto_abe
    f = np.load(f"{GOLDEN}/generator_bi.npz", allow_pickle=False)
    n = 100_000
    cbs, el = generate_pareto_abe(n, float(f["T_cal_in"]), f["T_star"], f["beta"], f["gamma"], seed=77)
    assert list(cbs.columns) == ["cust", "x", "t_x", "T_cal", "lambda_true", "mu_true", "tau_true", "alive_true",
                                 "x_star20", "x_star32", "cov0", "cov1"]
    for c in ("lambda_true", "mu_true", "tau_true", "cov1"):
        assert stats.ks_2samp(cbs[c], f[c]).pvalue > 1e-4, c
    m = cbs["x"] > 0
    assert stats.ks_2samp(cbs["t_x"][m], f["t_x"][f["x"] > 0]).pvalue > 1e-4
    for c in ("x", "x_star20", "x_star32"):
        a, b = cbs[c].to_numpy(), f[c].astype(np.int64)
        edges = np.unique(np.quantile(np.concatenate([a, b]), np.linspace(0, 1, 12)).astype(int))
        ta, tb = np.histogram(a, np.append(edges, 10 ** 9))[0], np.histogram(b, np.append(edges, 10 ** 9))[0]
        keep = (ta + tb) > 0
        assert stats.chi2_contingency(np.vstack([ta[keep], tb[keep]]))[1] > 1e-4, c
    p = f["alive_true"].mean()
    assert abs(cbs["alive_true"].mean() - p) < 4 * np.sqrt(p * (1 - p) * (1 / n + 1 / len(f["x"])))
    # internal consistency with the event log (bi:75-89, bi:170-179)
    T = float(f["T_cal_in"])
    ev = el.groupby("cust")["t"]
    cal = el[el["t"] <= T].groupby("cust")["t"]
    assert np.array_equal(np.clip(cal.count().reindex(cbs["cust"]).to_numpy() - 1, 0, None), cbs["x"].to_numpy())
    assert np.array_equal(_bits(cal.max().reindex(cbs["cust"]).to_numpy()), _bits(cbs["t_x"]))
    hold = el[(el["t"] > T) & (el["t"] <= T + 20.0)].groupby("cust")["t"].size()
    assert np.array_equal(hold.reindex(cbs["cust"], fill_value=0).to_numpy(), cbs["x_star20"].to_numpy())
    assert (ev.min().to_numpy() == 0.0).all()  # every customer's first purchase at t = 0 (T_cal scalar)
    again, _ = generate_pareto_abe(n, float(f["T_cal_in"]), f["T_star"], f["beta"], f["gamma"], seed=77,
                                   return_elog=False)
    assert again.equals(cbs)
