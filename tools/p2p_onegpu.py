#!/usr/bin/env python
"""Peer-exchange overhead on ONE GPU: W processes (gloo group for the handle exchange) each run a
1/W shard of a bench workload (CLV_P2P_WORKLOAD, default c2) through ShardedSampler(exchange="p2p")
on the same card, so the exchange is IPC-mapped device memory instead of xGMI; compared with the
world-size-1 run of the same problem (same total work on the card).  c2: the persistent kernel's
exchange; c4 (1M customers, shards too large for a resident grid): the sweep kernel's fused
exchange.  Prints one JSON line per rank 0."""
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
WORKLOAD = os.environ.get("CLV_P2P_WORKLOAD", "c2")
WARM = 200 if WORKLOAD in ("c1", "c2", "c3") else 20


def load_workload():
    """bench.load_workload(WORKLOAD); CLV_P2P_N overrides a synthetic workload's customer count
    (e.g. c4 at 125,000: one 8-rank shard of c4 split over the W processes on this card)."""
    import bench
    n = os.environ.get("CLV_P2P_N")
    if n:
        D, data, *rest = bench.WORKLOADS[WORKLOAD]
        _, _, K, seed = data.split(":")
        bench.WORKLOADS[WORKLOAD] = (D, f"synthetic:{int(n)}:{K}:{seed}", *rest)
    return bench.load_workload(WORKLOAD)


def worker(sweeps):
    import torch.distributed as dist
    import bench
    from mcmc_clv_model_amd.sampler import build_problem
    from mcmc_clv_model_amd.distributed import ShardedSampler
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    df, D, covs, ch, burnin, mcmc, thin, sink = load_workload()
    p = build_problem(df, covs, D)
    dist.init_process_group("gloo")
    ss = ShardedSampler(p, rank=rank, world=world, chains=ch, mcmc=mcmc, burnin=burnin, thin=thin, seed=42,
                        draw_sink=sink, device=0, exchange="p2p", verify_sweeps=8)
    ss.step(WARM)
    ss.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    ss.step(sweeps)
    ss.synchronize()
    dist.barrier()
    dt = time.perf_counter() - t0
    if rank == 0:
        print(json.dumps(dict(workload=WORKLOAD, n=len(df), world=world, us_per_sweep=dt / sweeps * 1e6,
                              exchange=ss.exchange, persistent=ss.launch_info()["persistent"], note=ss.p2p_note,
                              env={k: v for k, v in os.environ.items() if k.startswith("CLV_")})), flush=True)
    if os.environ.get("CLV_LIB_PATH", "").endswith("_stamps.so"):  # level-2 workgroup timeline, one sweep
        import ctypes
        import numpy as np
        s = ss.s
        nb = -(-s.n // 256)
        wg = np.zeros(s.chains * (nb + 1) * 12, np.uint64)
        assert s._L.clv_debug_wg_stamps(s.h, wg.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))) == 0
        wg = wg.astype(np.int64).reshape(s.chains, nb + 1, 12)
        for c in range(s.chains):
            t = wg[c, nb]
            R = t[5]  # previous sweep's publish
            last = wg[c, :nb, 5].max()
            print(f"rank {rank} chain {c} (us after the previous publish): last local partial {(last - R) / 100:.2f}"
                  f"  local partials seen {(t[2] - R) / 100:.2f}  units formed {(t[10] - t[2]) / 100:.2f}"
                  f"  polls done {(t[11] - t[10]) / 100:.2f}  summed {(t[6] - t[11]) / 100:.2f}"
                  f"  draw {(t[3] - t[6]) / 100:.2f}  published {(t[4] - R) / 100:.2f}", flush=True)
    ss.close()
    dist.destroy_process_group()


def main(world=2, sweeps=3000):
    from mcmc_clv_model_amd.sampler import HipSampler, build_problem
    import bench
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = [subprocess.Popen([sys.executable, __file__, "--worker", str(sweeps)], cwd=ROOT,
                              env=dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                                       MASTER_PORT=str(port))) for r in range(world)]
    rc = [p.wait(timeout=300) for p in procs]
    assert rc == [0] * world, rc
    df, D, covs, ch, burnin, mcmc, thin, sink = load_workload()
    with HipSampler(build_problem(df, covs, D), mcmc=mcmc, burnin=burnin, thin=thin, chains=ch, seed=42,
                    draw_sink=sink) as s:
        s.run(WARM)
        s.synchronize()
        t0 = time.perf_counter()
        s.run(sweeps)
        s.synchronize()
        print(json.dumps(dict(workload=WORKLOAD, world=1, us_per_sweep=(time.perf_counter() - t0) / sweeps * 1e6)))


if __name__ == "__main__":
    if sys.argv[1:2] == ["--worker"]:
        worker(int(sys.argv[2]))
    else:
        main(*(int(a) for a in sys.argv[1:3]))
