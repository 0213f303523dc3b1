"""Row f (posterior analysis) on CPU: the oracle restatement of the reference's analysis helpers
reproduces the reference's own outputs stored in tests/golden/analysis_abe400.npz (bit for bit),
and the analysis API validates its inputs before touching the device."""
import numpy as np
import pandas as pd
import pytest

from oracle import analysis_cpu as oan
from tests.helpers import GOLDEN


@pytest.fixture(scope="module")
def fx():
    f = np.load(f"{GOLDEN}/analysis_abe400.npz", allow_pickle=False)
    cbs = pd.DataFrame(dict(x=f["x"], t_x=f["t_x"], T_cal=f["T_cal"]))
    bi = dict(level_1=list(f["bi_level1"]))
    tri = dict(level_1=list(f["tri_level1"]))
    return f, cbs, bi, tri


def _bits(a):
    return np.asarray(a, dtype=np.float64).view(np.uint64)


def test_oracle_matches_reference_outputs(fx):
    f, cbs, bi, tri = fx
    assert np.array_equal(oan.draw_future_transactions_bi(cbs, bi, 39.0, seed=42), f["xstar_bi"])
    x, sp = oan.draw_future_transactions_tri(cbs, tri, 39.0, seed=43)
    assert np.array_equal(x, f["xstar_tri"]) and np.array_equal(_bits(sp), _bits(f["spend_tri"]))
    assert np.array_equal(_bits(oan.post_mean_lambdas(bi)), _bits(f["post_mean_lambdas"]))
    assert np.array_equal(_bits(oan.post_mean_mus(bi)), _bits(f["post_mean_mus"]))
    assert _bits(oan.chain_total_loglik(bi["level_1"], cbs)) == _bits(f["chain_total_loglik"])
    st = oan.table4_stats(bi)
    for k, v in st.items():
        assert np.array_equal(_bits(v), _bits(f[f"t4_{k}"])), k


def test_reference_quirks_pinned(fx):
    """Churned customers forecast zero transactions (tau <= T_cal, so tau* = 0: bi:540); the
    trivariate spend uses the natural-scale eta column as the lognormal log-mean (tri:733)."""
    f, cbs, bi, tri = fx
    lv = np.concatenate(bi["level_1"])
    assert (f["xstar_bi"][lv[:, :, 3] < 0.5] == 0).all()
    lt = np.concatenate(tri["level_1"])
    has = f["xstar_tri"] > 0
    assert (f["spend_tri"][~has] == 0).all()
    # a spend total is at least its smallest possible lognormal draw: exp(eta - 6 sigma) per trx
    assert (f["spend_tri"][has] > f["xstar_tri"][has] * np.exp(lt[:, :, 4][has] - 6 * 0.5)).all()


def test_tracking_oracle_is_unbiased(fx):
    f, cbs, bi, tri = fx
    exp = oan.weekly_tracking_expectation(bi, f["birth_week"], f["times"])
    n_draws = sum(len(c) for c in bi["level_1"])
    sd = np.sqrt(np.maximum(exp, 1e-12) / n_draws)
    z = (f["tracking_ref"] - exp) / sd
    assert np.abs(z[exp > 0]).max() < 5.0


def test_analysis_api_validates_inputs(fx):
    from mcmc_clv_model_amd import analysis
    f, cbs, bi, tri = fx
    with pytest.raises(ValueError):
        analysis._stacked_level1(None)
    with pytest.raises(ValueError):
        analysis._stacked_level1([np.zeros((3, 4, 7))])
