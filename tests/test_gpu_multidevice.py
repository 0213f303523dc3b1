"""SURVEY §8b / verdict r1 #2, #9: multi-GPU from the drop-in entry points —
``mcmc_draw_parameters(..., devices=[...])`` (bi:437-504) spreads one run over several devices of
this process and returns the reference's layout, bit for bit the single-device run.

On the one-GPU test box the "devices" are one card named twice ([0, 0]): the chain groups / the
customer shards are separate sampler handles with their own streams and buffers exactly as on
distinct devices; only the peer-access enabling between distinct devices is not exercised.  Both
exchanges of the in-process group (clv_group, csrc/group.hip) are run: peer stores between
persistent kernels ("p2p", where both grids fit the card together) and device-to-device copies
("copy"), including a problem large enough for blocks_per_unit > 1."""
import numpy as np
import pytest

from tests.helpers import bits, cdnow

pytestmark = pytest.mark.gpu


def _same(a, b):
    assert (a["level_1"] is None) == (b["level_1"] is None)
    if a["level_1"] is not None:
        assert len(a["level_1"]) == len(b["level_1"])
        for x, y in zip(a["level_1"], b["level_1"]):
            assert x.shape == y.shape and np.array_equal(bits(x), bits(y))
    for x, y in zip(a["level_2"], b["level_2"]):
        assert np.array_equal(bits(x), bits(y))
    assert np.array_equal(bits(a["log_likelihood"]), bits(b["log_likelihood"]))
    if "summary" in a:
        for k, v in a["summary"].items():
            if k == "level1":
                assert np.array_equal(bits(v.to_numpy()), bits(b["summary"][k].to_numpy())), k
            elif k != "n_draws":
                assert np.array_equal(bits(v), bits(b["summary"][k])), k


def test_devices_chain_groups_bitwise(capsys):
    """shard='chains' (auto with 4 chains on 2 devices): two chain groups, one host thread each."""
    from mcmc_clv_model_amd import mcmc_draw_parameters
    df = cdnow("abe")
    kw = dict(mcmc=40, burnin=30, thin=2, chains=4, seed=123, trace=25)
    one = mcmc_draw_parameters(df, ["first_sales_scaled"], **kw)
    out1 = capsys.readouterr().out
    two = mcmc_draw_parameters(df, ["first_sales_scaled"], devices=[0, 0], **kw)
    out2 = capsys.readouterr().out
    _same(one, two)
    assert out1 == out2 and out1.count("\n") == 4 * 2  # the reference's trace lines, in its order


@pytest.mark.parametrize("D,sink,exchange", [(2, "full", "auto"), (3, "summary+pct", "auto"), (2, "summary", "copy"),
                                             (3, "full", "copy")])
def test_devices_customer_shards_bitwise(D, sink, exchange):
    """shard='customers': every chain's customers split over the devices, one exchange per sweep
    (p2p: both CDNOW-size grids fit the card together; copy forced), bitwise the one-device run."""
    from mcmc_clv_model_amd import mcmc_draw_parameters, mcmc_draw_parameters_rfm_m
    fn, covs = ((mcmc_draw_parameters, ["first_sales_scaled"]) if D == 2 else
                (mcmc_draw_parameters_rfm_m, ["gender_F", "age_scaled"]))
    df = cdnow("full")
    kw = dict(mcmc=21, burnin=9, thin=3, chains=2, seed=9, trace=0, draw_sink=sink)
    one = fn(df, covs, **kw)
    two = fn(df, covs, devices=[0, 0], shard="customers", exchange=exchange, **kw)
    assert two.pop("exchange") == ("p2p" if exchange == "auto" else "copy")
    _same(one, two)


def test_devices_customer_shards_large_units_copy():
    """blocks_per_unit > 1 (150,000 customers: unit partials of 2 blocks, summed by group_kernel
    before the copies) on three shards; the three grids do not fit the card together, so the group
    picks the copy exchange by itself."""
    from mcmc_clv_model_amd import mcmc_draw_parameters
    from mcmc_clv_model_amd.data import synthetic_cbs
    df = synthetic_cbs(150_000, 3, 2, seed=31)
    kw = dict(mcmc=6, burnin=4, thin=2, chains=1, seed=5, trace=0, draw_sink="summary")
    one = mcmc_draw_parameters(df, ["c1", "c2"], **kw)
    three = mcmc_draw_parameters(df, ["c1", "c2"], devices=[0, 0, 0], **kw)
    assert three.pop("exchange") == "copy"
    _same(one, three)


def test_devices_argument_errors():
    from mcmc_clv_model_amd import mcmc_draw_parameters
    df = cdnow("abe", 600)
    with pytest.raises(ValueError, match="shard must be"):
        mcmc_draw_parameters(df, [], mcmc=2, burnin=1, chains=2, trace=0, devices=[0, 0], shard="rows")
    with pytest.raises(ValueError, match="summary\\+pct"):
        mcmc_draw_parameters(df, [], mcmc=2, burnin=1, chains=2, trace=0, devices=[0, 0], shard="chains",
                             draw_sink="summary+pct")
    with pytest.raises(ValueError, match="philox"):
        mcmc_draw_parameters(df, [], mcmc=2, burnin=1, chains=2, trace=0, devices=[0, 0], rng="replay")
    with pytest.raises(ValueError, match="exchange must be"):
        mcmc_draw_parameters(df, [], mcmc=2, burnin=1, chains=1, trace=0, devices=[0, 0], exchange="rccl")
