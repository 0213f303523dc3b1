"""Row (e), peer exchange: the persistent sweep kernel at world size > 1 (clv_p2p_connect,
include/clvmcmc.h) — each chain's level-2 workgroup stores its rank's unit partials straight into
every rank's mail buffer and sums all ranks' units in the global fixed order — reproduces the
unsharded run bit for bit (state, level-2 records, log-likelihood, summaries).

On the one-GPU test box the "ranks" share the card: in one process (mail pointers, one host
thread per rank, since every rank's launch must be resident at once) and in two processes
(hipIpcMemHandle exchange over a gloo group, through ShardedSampler(exchange="p2p") incl. its
bitwise verification against the all-gather path)."""
import os
import socket
import subprocess
import sys
import threading

import numpy as np
import pytest

from tests.helpers import bits, cdnow

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ref_run(p, sweeps, kw):
    from mcmc_clv_model_amd.sampler import HipSampler
    with HipSampler(p, **kw) as s:
        s.run(sweeps)
        st = s.get_state()
        sums = s.read_summary()[0] if kw["draw_sink"] == "summary" else None
        l1, l2, ll = s.read_draws(level1=kw["draw_sink"] == "full")
    return st, sums, l1, l2, ll


@pytest.mark.parametrize("D,covs,n,world,sink", [(2, ["first_sales_scaled"], 23570, 2, "summary"),
                                                 (3, ["gender_F", "age_scaled"], 23570, 3, "full"),
                                                 (2, [], 2357, 2, "full"),
                                                 # c4's instance (bivariate K=5, persist_kernel<2,5,true>)
                                                 # and c5's (trivariate K=9): synthetic covariates
                                                 (2, ["c1", "c2", "c3", "c4"], 40000, 2, "summary"),
                                                 (3, [f"c{k}" for k in range(1, 9)], 20000, 2, "summary")])
def test_p2p_persistent_bitwise_equals_unsharded(D, covs, n, world, sink):
    """K = 5 / 9 at world 2 on one card: the driver's 8-GPU c4 layout (125k customers per rank)
    would need 8 x 490 workgroups resident on ONE GPU at once, so the instance is checked here at
    the largest size whose two grids fit one card together."""
    import torch
    from mcmc_clv_model_amd import distributed as Dm
    from mcmc_clv_model_amd.data import synthetic_cbs
    from mcmc_clv_model_amd.sampler import HipSampler, build_problem, make_prior
    if covs and covs[0] == "c1":
        df = synthetic_cbs(n, len(covs) + 1, D, seed=n)
    else:
        df = cdnow("full", n) if n > 2357 else cdnow("abe", n)
    p = build_problem(df, covs, D)
    kw = dict(mcmc=9, burnin=4, thin=2, chains=2, seed=4242, draw_sink=sink)
    chunks = (1, 5, 7)
    sweeps = sum(chunks)
    ref, ref_sums, ref_l1, ref_l2, ref_ll = _ref_run(p, sweeps, kw)

    plan = Dm.plan(p.N, world)
    prior = make_prior(p, p.N)
    shards = []
    for r in range(world):
        b, e = plan.shard(r)
        shards.append(HipSampler(Dm.slice_problem(p, b, e), n_global=p.N, shard_begin=r * plan.blocks_per_rank * 256,
                                 world_size=world, rank=r, blocks_per_rank=plan.blocks_per_rank,
                                 blocks_per_unit=plan.blocks_per_unit, prior=prior, **kw))
    try:
        info = [sh.p2p_info() for sh in shards]
        assert all(i["capable"] and not i["connected"] for i in info), info
        with pytest.raises(Exception, match="clv_p2p_connect"):
            shards[0].run(1)  # sharded clv_run needs the connection
        if D == 2:  # bivariate: the initial draw from the initial state, through the all-gather path
            nd = shards[0].partials()[1]
            gathered = torch.zeros(nd * world, dtype=torch.float64, device="cuda")
            for r, sh in enumerate(shards):
                sh.copy_partials(gathered.data_ptr() + r * nd * 8)
                sh.synchronize()
            for sh in shards:
                sh.hyper(gathered.data_ptr())
                sh.synchronize()
        ptrs = [i["mail_ptr"] for i in info]
        for sh in shards:
            sh.p2p_connect(ptrs=ptrs)
        assert all(sh.p2p_info()["connected"] for sh in shards)

        for n_run in chunks:  # every rank's launch runs at once (one host thread each)
            errs = []

            def go(sh):
                try:
                    sh.run(n_run)
                except Exception as e:  # noqa: BLE001
                    errs.append(e)

            th = [threading.Thread(target=go, args=(sh,)) for sh in shards]
            for t in th:
                t.start()
            for t in th:
                t.join(timeout=60)
            assert not any(t.is_alive() for t in th)
            assert not errs, errs
        for r, sh in enumerate(shards):
            b, e = plan.shard(r)
            assert sh.sweeps_done == sweeps
            lam, mu, beta, sigma = sh.get_state()
            assert np.array_equal(bits(lam), bits(ref[0][:, b:e])) and np.array_equal(bits(mu), bits(ref[1][:, b:e]))
            assert np.array_equal(bits(beta), bits(ref[2])) and np.array_equal(bits(sigma), bits(ref[3]))
            l1, l2, ll = sh.read_draws(level1=sink == "full")
            assert np.array_equal(bits(l2), bits(ref_l2)) and np.array_equal(bits(ll), bits(ref_ll))
            if sink == "full":
                assert np.array_equal(bits(l1), bits(ref_l1[:, :, b:e]))
            else:
                assert np.array_equal(bits(sh.read_summary()[0]), bits(ref_sums[:, :, b:e]))
    finally:
        for sh in shards:
            sh.close()


@pytest.mark.parametrize("D,covs,n,world,sink,persistent_off", [
    (2, ["first_sales_scaled"], 23570, 2, "full", True),
    (3, ["gender_F", "age_scaled"], 23570, 3, "summary", True),
    # too large for a resident grid per shard: the fused exchange by itself, blocks_per_unit 4
    (2, ["c1", "c2", "c3", "c4"], 300000, 2, "summary", False)])
def test_fused_exchange_bitwise_equals_unsharded(monkeypatch, D, covs, n, world, sink, persistent_off):
    """World size > 1 without the persistent grid (verdict r1 #7: the c4/c5-size shards exchanged
    without an RCCL all-gather and a separate level-2 launch per sweep): clv_run launches the sweep
    kernel once per sweep (hipGraph chunks of 64) and its fused tail stores this rank's unit
    partials into every rank's mail, waits for all ranks' units in its own and draws — bitwise the
    unsharded run (state, draws / summaries, level-2 records, log-likelihood)."""
    import torch
    from mcmc_clv_model_amd import distributed as Dm
    from mcmc_clv_model_amd.data import synthetic_cbs
    from mcmc_clv_model_amd.sampler import HipSampler, build_problem, make_prior
    if persistent_off:
        monkeypatch.setenv("CLV_PERSISTENT", "0")
    df = synthetic_cbs(n, len(covs) + 1, D, seed=n) if covs[0] == "c1" else cdnow("full", n)
    p = build_problem(df, covs, D)
    kw = dict(mcmc=40, burnin=50, thin=3, chains=2 if n < 100000 else 1, seed=2024, draw_sink=sink)
    chunks = (1, 5, 70, 3)
    sweeps = sum(chunks)
    kw["mcmc"] = sweeps - kw["burnin"]
    ref, ref_sums, ref_l1, ref_l2, ref_ll = _ref_run(p, sweeps, kw)
    plan = Dm.plan(p.N, world)
    prior = make_prior(p, p.N)
    shards = []
    for r in range(world):
        b, e = plan.shard(r)
        shards.append(HipSampler(Dm.slice_problem(p, b, e), n_global=p.N, shard_begin=r * plan.blocks_per_rank * 256,
                                 world_size=world, rank=r, blocks_per_rank=plan.blocks_per_rank,
                                 blocks_per_unit=plan.blocks_per_unit, prior=prior, **kw))
    try:
        info = [sh.p2p_info() for sh in shards]
        assert all(i["capable"] and not i["persistent"] for i in info), info
        assert all(not sh.launch_info()["persistent"] for sh in shards)
        if D == 2:
            nd = shards[0].partials()[1]
            gathered = torch.zeros(nd * world, dtype=torch.float64, device="cuda")
            for r, sh in enumerate(shards):
                sh.copy_partials(gathered.data_ptr() + r * nd * 8)
                sh.synchronize()
            for sh in shards:
                sh.hyper(gathered.data_ptr())
                sh.synchronize()
        ptrs = [i["mail_ptr"] for i in info]
        for sh in shards:
            sh.p2p_connect(ptrs=ptrs)
        for n_run in chunks:
            errs = []

            def go(sh):
                try:
                    sh.run(n_run)
                except Exception as e:  # noqa: BLE001
                    errs.append(e)

            th = [threading.Thread(target=go, args=(sh,)) for sh in shards]
            for t in th:
                t.start()
            for t in th:
                t.join(timeout=120)
            assert not any(t.is_alive() for t in th)
            assert not errs, errs
        for r, sh in enumerate(shards):
            b, e = plan.shard(r)
            assert sh.sweeps_done == sweeps
            lam, mu, beta, sigma = sh.get_state()
            assert np.array_equal(bits(lam), bits(ref[0][:, b:e])) and np.array_equal(bits(mu), bits(ref[1][:, b:e]))
            assert np.array_equal(bits(beta), bits(ref[2])) and np.array_equal(bits(sigma), bits(ref[3]))
            l1, l2, ll = sh.read_draws(level1=sink == "full")
            assert np.array_equal(bits(l2), bits(ref_l2)) and np.array_equal(bits(ll), bits(ref_ll))
            if sink == "full":
                assert np.array_equal(bits(l1), bits(ref_l1[:, :, b:e]))
            else:
                assert np.array_equal(bits(sh.read_summary()[0]), bits(ref_sums[:, :, b:e]))
    finally:
        for sh in shards:
            sh.close()


WORKER = r"""
import json, os, sys
sys.path.insert(0, os.environ["CLV_ROOT"])
import numpy as np
import torch.distributed as dist
from tests.helpers import bits, cdnow
from mcmc_clv_model_amd.sampler import HipSampler, build_problem
from mcmc_clv_model_amd.distributed import ShardedSampler
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
D = int(os.environ["CLV_D"])
covs = ["first_sales_scaled"] if D == 2 else ["gender_F", "age_scaled"]
p = build_problem(cdnow("full", 12000), covs, D)
kw = dict(mcmc=6, burnin=12, thin=2, chains=2, seed=7, draw_sink="summary")
with HipSampler(p, **kw) as s:          # unsharded reference, before any rank's persistent launch
    s.run(17)
    ref = s.get_state()
    ref_sums = s.read_summary()[0]
dist.init_process_group("gloo")
if os.environ.get("CLV_TEST_STALL_PERSISTENT_RANK") == str(rank):
    # test hook: this rank's persistent launches never run (its peer's wait times out), fused ones do
    from mcmc_clv_model_amd import _lib, sampler as S
    run0 = S.HipSampler.run
    def run(self, n):
        if self.p2p_info()["persistent"]:
            raise _lib.ClvError("test hook: persistent launch withheld")
        return run0(self, n)
    S.HipSampler.run = run
ss = ShardedSampler(p, rank=rank, world=world, device=0, exchange="p2p", verify_sweeps=4, **kw)
ss.step(9)
ss.step(8)
ss.synchronize()
b, e = ss.begin, ss.end
got = ss.s.get_state()
ok = (ss.exchange == "p2p" and ss.s.sweeps_done == 17
      and all(np.array_equal(bits(x), bits(y[:, b:e] if i < 2 else y)) for i, (x, y) in enumerate(zip(got, ref)))
      and np.array_equal(bits(ss.s.read_summary()[0]), bits(ref_sums[:, :, b:e])))
print(json.dumps(dict(rank=rank, ok=bool(ok), note=ss.p2p_note)), flush=True)
ss.close()
dist.destroy_process_group()
"""


@pytest.mark.parametrize("D,persistent,stall", [(2, "1", None), (3, "1", None), (2, "0", None), (2, "1", 1)])
def test_p2p_two_processes_ipc(D, persistent, stall):
    """Two processes (one rank each) on the one GPU: hipIpcMemHandle exchange, verification
    against the all-gather path, then 17 sweeps in two steps — bitwise equal to the unsharded run
    (persistent = "0": through the fused exchange).  stall = 1: rank 1 withholds its persistent
    launches, so the persistent exchange fails its verification on both ranks and ShardedSampler
    falls back to the fused exchange (round 6), verified the same way, before RCCL."""
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), CLV_ROOT=ROOT, CLV_D=str(D), CLV_PERSISTENT=persistent)
        if stall is not None:
            env["CLV_TEST_STALL_PERSISTENT_RANK"] = str(stall)
        procs.append(subprocess.Popen([sys.executable, "-c", WORKER], env=env, cwd=ROOT, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    for pr in procs:
        try:
            out, err = pr.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((pr.returncode, out, err))
    for rc, out, err in outs:
        assert rc == 0, err[-3000:]
        import json
        res = json.loads(out.strip().splitlines()[-1])
        assert res["ok"], res
        if stall is not None:
            assert "persistent: verification against RCCL failed" in res["note"], res
            assert res["note"].endswith("fused exchange verified bitwise against RCCL over 4 sweeps"), res
        else:
            kind = "persistent" if persistent == "1" else "fused"
            assert res["note"] == f"{kind} exchange verified bitwise against RCCL over 4 sweeps", res


@pytest.mark.parametrize("persistent", ["1", "0"])
def test_p2p_abort_leaves_state_unchanged_and_rollback(monkeypatch, persistent):
    """a call whose wait times out (here: the peer rank never launches) fails and
    leaves its rank's state, sweep count and summary sums exactly as before the call; after
    reconnecting, and after a completed step is undone with clv_rollback on every rank and redone,
    the run is still bitwise the unsharded one.  persistent = "0": the fused exchange (one sweep
    launch per sweep; the call's launches after the timed-out one return at once)."""
    import torch
    from mcmc_clv_model_amd import _lib
    from mcmc_clv_model_amd import distributed as Dm
    from mcmc_clv_model_amd.sampler import HipSampler, build_problem, make_prior
    monkeypatch.setenv("CLV_WAIT_TIMEOUT_MS", "300")
    monkeypatch.setenv("CLV_PERSISTENT", persistent)
    p = build_problem(cdnow("full", 23570), ["first_sales_scaled"], 2)
    kw = dict(mcmc=9, burnin=1, thin=1, chains=2, seed=77, draw_sink="summary")
    world = 2
    ref, ref_sums, _, ref_l2, ref_ll = _ref_run(p, 10, kw)
    plan = Dm.plan(p.N, world)
    prior = make_prior(p, p.N)
    shards = []
    for r in range(world):
        b, e = plan.shard(r)
        shards.append(HipSampler(Dm.slice_problem(p, b, e), n_global=p.N, shard_begin=r * plan.blocks_per_rank * 256,
                                 world_size=world, rank=r, blocks_per_rank=plan.blocks_per_rank,
                                 blocks_per_unit=plan.blocks_per_unit, prior=prior, **kw))

    def run_all(n, ranks=None):
        errs = []

        def go(sh):
            try:
                sh.run(n)
            except Exception as e:  # noqa: BLE001
                errs.append(e)
        th = [threading.Thread(target=go, args=(shards[r],)) for r in (ranks or range(world))]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=60)
        assert not any(t.is_alive() for t in th)
        return errs

    def connect():
        ptrs = [sh.p2p_info()["mail_ptr"] for sh in shards]
        for sh in shards:
            sh.p2p_connect(ptrs=ptrs)
        for sh in shards:
            sh.synchronize()

    try:
        assert all(sh.p2p_info()["persistent"] == (persistent == "1") for sh in shards)
        nd = shards[0].partials()[1]
        gathered = torch.zeros(nd * world, dtype=torch.float64, device="cuda")
        for r, sh in enumerate(shards):
            sh.copy_partials(gathered.data_ptr() + r * nd * 8)
            sh.synchronize()
        for sh in shards:
            sh.hyper(gathered.data_ptr())
            sh.synchronize()
        connect()
        assert not run_all(3)
        before = shards[0].get_state()
        sums_before = shards[0].read_summary()[0].copy()
        errs = run_all(4, ranks=[0])  # rank 1 never launches: rank 0's first wait times out
        assert len(errs) == 1 and isinstance(errs[0], _lib.ClvError) and "state unchanged" in str(errs[0])
        # the wait record names the missing peer unit and the ranks' progress: rank 0 polls for
        # sweep 4, rank 1's level-2 side last polled for sweep 3 (it never started sweep 4)
        msg = str(errs[0])
        assert "[wait record: sweep 4, chain " in msg and "peer unit partial" in msg, msg
        assert "(rank 1, local unit" in msg and "0:4 1:3" in msg, msg
        # written by the wave whose own bound expired, not by one that only saw the abort flag
        import re
        waited = float(re.search(r" polls, ([0-9.]+) ms;", msg).group(1))
        assert waited >= 300.0, msg
        assert shards[0].sweeps_done == 3
        after = shards[0].get_state()
        assert all(np.array_equal(bits(x), bits(y)) for x, y in zip(before, after))
        assert np.array_equal(bits(shards[0].read_summary()[0]), bits(sums_before))
        assert not shards[0].p2p_info()["connected"]
        connect()
        assert not run_all(4)
        assert not run_all(2)
        for sh in shards:  # a completed step undone on every rank, then redone
            sh.rollback()
            assert sh.sweeps_done == 7
        with pytest.raises(_lib.ClvError, match="nothing to roll back"):
            shards[0].rollback()
        assert not run_all(3)
        for r, sh in enumerate(shards):
            b, e = plan.shard(r)
            assert sh.sweeps_done == 10
            lam, mu, beta, sigma = sh.get_state()
            assert np.array_equal(bits(lam), bits(ref[0][:, b:e])) and np.array_equal(bits(mu), bits(ref[1][:, b:e]))
            assert np.array_equal(bits(beta), bits(ref[2])) and np.array_equal(bits(sigma), bits(ref[3]))
            assert np.array_equal(bits(sh.read_summary()[0]), bits(ref_sums[:, :, b:e]))
            _, l2, ll = sh.read_draws(level1=False)
            assert np.array_equal(bits(l2), bits(ref_l2)) and np.array_equal(bits(ll), bits(ref_ll))
    finally:
        for sh in shards:
            sh.close()
