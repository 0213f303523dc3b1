#!/usr/bin/env python
"""The fused peer exchange's sweep time on one card (A/B helper, round 6): `world` shards of one
synthetic problem in this process, each on its own stream and host thread (the ranks' launches run
concurrently, as test_gpu_p2p.py's), CLV_PERSISTENT=0 so every shard takes the fused exchange (one
sweep launch per sweep whose tail exchanges the unit partials through the peers' mail).  Prints
us per sweep over `sweeps` timed sweeps after 50 warm-up sweeps.  Not a scaling measurement: all
ranks share one GPU.

    CLV_LIB_PATH=... python tools/fx_ab.py [D K n_per_rank world sweeps]
"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["CLV_PERSISTENT"] = "0"


def main(D=3, K=9, n_rank=300_000, world=2, sweeps=300):
    import torch
    from mcmc_clv_model_amd import distributed as Dm
    from mcmc_clv_model_amd.data import synthetic_cbs
    from mcmc_clv_model_amd.sampler import HipSampler, build_problem, make_prior
    p = build_problem(synthetic_cbs(n_rank * world, K, D, seed=11), [f"c{k}" for k in range(1, K)], D)
    plan = Dm.plan(p.N, world)
    prior = make_prior(p, p.N)
    kw = dict(mcmc=5000, burnin=5000, thin=1, chains=1, seed=3, draw_sink="summary")
    shards = []
    for r in range(world):
        b, e = plan.shard(r)
        shards.append(HipSampler(Dm.slice_problem(p, b, e), n_global=p.N, shard_begin=r * plan.blocks_per_rank * 256,
                                 world_size=world, rank=r, blocks_per_rank=plan.blocks_per_rank,
                                 blocks_per_unit=plan.blocks_per_unit, prior=prior, **kw))
    try:
        assert not any(sh.p2p_info()["persistent"] for sh in shards)
        if D == 2:  # the bivariate initial draw through the all-gather path
            nd = shards[0].partials()[1]
            g = torch.zeros(nd * world, dtype=torch.float64, device="cuda")
            for r, sh in enumerate(shards):
                sh.copy_partials(g.data_ptr() + r * nd * 8)
                sh.synchronize()
            for sh in shards:
                sh.hyper(g.data_ptr())
                sh.synchronize()
        ptrs = [sh.p2p_info()["mail_ptr"] for sh in shards]
        for sh in shards:
            sh.p2p_connect(ptrs=ptrs)

        def run_all(n):
            errs = []

            def go(sh):
                try:
                    sh.run(n)
                except Exception as e:  # noqa: BLE001
                    errs.append(e)
            th = [threading.Thread(target=go, args=(sh,)) for sh in shards]
            for t in th:
                t.start()
            for t in th:
                t.join(timeout=120)
            assert not errs, errs
        run_all(50)
        t0 = time.perf_counter()
        run_all(sweeps)
        dt = time.perf_counter() - t0
        print(json.dumps(dict(D=D, K=K, n_per_rank=n_rank, world=world, sweeps=sweeps,
                              us_per_sweep=round(dt / sweeps * 1e6, 3), lib=os.environ.get("CLV_LIB_PATH", "in-tree"))),
              flush=True)
    finally:
        for sh in shards:
            sh.close()


if __name__ == "__main__":
    a = [int(x) for x in sys.argv[1:]]
    main(*a)
