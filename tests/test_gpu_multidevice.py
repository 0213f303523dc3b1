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
                                             (3, "full", "copy"), (2, "summary", "p2p"), (3, "full", "p2p")])
def test_devices_customer_shards_bitwise(D, sink, exchange):
    """shard='customers': every chain's customers split over the devices, one exchange per sweep,
    bitwise the one-device run.  Shards sharing a device: "auto" takes the copy exchange (the two
    persistent kernels would have to run concurrently from two streams, which HIP does not promise);
    "p2p" requested explicitly runs the peer stores between the two resident grids (both CDNOW-size
    grids fit the card together) or, if a wait times out, the copy fallback — same bits either way."""
    from mcmc_clv_model_amd import mcmc_draw_parameters, mcmc_draw_parameters_rfm_m
    fn, covs = ((mcmc_draw_parameters, ["first_sales_scaled"]) if D == 2 else
                (mcmc_draw_parameters_rfm_m, ["gender_F", "age_scaled"]))
    df = cdnow("full")
    kw = dict(mcmc=21, burnin=9, thin=3, chains=2, seed=9, trace=0, draw_sink=sink)
    one = fn(df, covs, **kw)
    two = fn(df, covs, devices=[0, 0], shard="customers", exchange=exchange, **kw)
    ex = two.pop("exchange")
    assert ex == "copy" if exchange != "p2p" else ex in ("p2p", "copy")
    _same(one, two)


def test_group_p2p_timeout_falls_back_to_copy(monkeypatch):
    """the group-level fallback.  A shard whose persistent launch never runs (test hook
    CLV_TEST_P2P_STALL_RANK=1) leaves shard 0 waiting for its mail: the wait bound (300 ms here)
    expires, shard 0 keeps its state, the group redoes the call through the copy exchange and keeps
    it — results bitwise the unsharded run, clv_group_exchange reports copy, and after the group is
    destroyed no shard is left connected."""
    from mcmc_clv_model_amd.sampler import HipGroup, HipSampler, build_problem, make_prior
    from mcmc_clv_model_amd import distributed as Dm
    df = cdnow("full")
    p = build_problem(df, ["first_sales_scaled"], 2)
    kw = dict(mcmc=6, burnin=4, thin=2, chains=2, seed=17, draw_sink="summary")
    with HipSampler(p, **kw) as s:
        s.run(10)
        ref = s.get_state()
        ref_sums, _ = s.read_summary()
    monkeypatch.setenv("CLV_WAIT_TIMEOUT_MS", "300")
    plan = Dm.plan(p.N, 2)
    prior = make_prior(p, p.N)
    shards = []
    for r in range(2):
        b, e = plan.shard(r)
        shards.append(HipSampler(Dm.slice_problem(p, b, e), n_global=p.N, shard_begin=r * plan.blocks_per_rank * 256,
                                 world_size=2, rank=r, blocks_per_rank=plan.blocks_per_rank,
                                 blocks_per_unit=plan.blocks_per_unit, prior=prior, device=0, **kw))
    g = None
    try:
        g = HipGroup(shards, "p2p")
        assert g.exchange == "p2p" and all(sh.p2p_info()["connected"] for sh in shards)
        monkeypatch.setenv("CLV_TEST_P2P_STALL_RANK", "1")
        g.run(10)
        monkeypatch.delenv("CLV_TEST_P2P_STALL_RANK")
        assert g.exchange == "copy"
        assert not any(sh.p2p_info()["connected"] for sh in shards)
        g.close()
        for r, sh in enumerate(shards):
            b, e = plan.shard(r)
            lam, mu, beta, sigma = sh.get_state()
            assert np.array_equal(bits(lam), bits(ref[0][:, b:e])) and np.array_equal(bits(mu), bits(ref[1][:, b:e]))
            assert np.array_equal(bits(beta), bits(ref[2])) and np.array_equal(bits(sigma), bits(ref[3]))
            sums, _ = sh.read_summary()
            assert np.array_equal(bits(sums), bits(ref_sums[:, :, b:e]))
            assert sh.p2p_info()["mail_memory"] in ("uncached", "fine-grained", "device")
    finally:
        if g is not None:  # the group before its shards (clv_group_destroy touches the shards)
            g.close()
        for sh in shards:
            sh.close()


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
