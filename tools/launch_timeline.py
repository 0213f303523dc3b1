#!/usr/bin/env python
"""Where a short persistent launch's time goes (verdict r3 #1): the stamps build
(libclvmcmc_stamps.so), c2, a 5-sweep warm-up launch, then launches of NSWEEPS (1 and 2 by default)
sweeps.  Per customer workgroup, s_memrealtime (10 ns) relative to the earliest workgroup entry:
entry, prologue done (loads, tables, z/tau and MH variates of the first sweep), (beta, Sigma)
observed, MH done, partial stored, next-sweep work done; the level-2 workgroups' partials-seen and
publish; next to the launch's event-timed duration.  min / median / max over workgroups."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("CLV_LIB_PATH", os.path.join(ROOT, "mcmc_clv_model_amd", "libclvmcmc_stamps.so"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    import bench
    from mcmc_clv_model_amd.sampler import HipSampler, build_problem
    df, D, covs, ch, burnin, mcmc, thin, sink = bench.load_workload("c2")
    s = HipSampler(build_problem(df, covs, D), mcmc=mcmc, burnin=burnin, thin=thin, chains=ch, seed=42,
                   draw_sink=sink)
    nb = -(-s.n // 256)
    for n in [int(x) for x in os.environ.get("NSWEEPS", "1,2").split(",")]:
        for rep in range(3):
            s.run(5)
            s.synchronize()
            time.sleep(0.05)
            s.set_timing(True)
            s.run(n)
            s.synchronize()
            kt = s.kernel_time()
            s.set_timing(False)
            wg = np.zeros(s.chains * (nb + 1) * 12, np.uint64)
            assert s._L.clv_debug_wg_stamps(s.h, wg.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))) == 0
            wg = wg.astype(np.int64).reshape(s.chains, nb + 1, 12)
            cust, l2 = wg[:, :nb].reshape(-1, 12), wg[:, nb]
            t0 = cust[:, 7].min()
            us = lambda v: [round(float(np.min(v)) / 100, 2), round(float(np.median(v)) / 100, 2),
                            round(float(np.max(v)) / 100, 2)]
            row = dict(sweeps=n, rep=rep, launch_us=round(kt["sweep_ms"] * 1e3, 2),
                       entry=us(cust[:, 7] - t0), prologue_done=us(cust[:, 10] - t0))
            if n <= 2:  # it_stamp = 0: the first sweep's stamps
                act = cust[:, 3] > 0
                row.update(observe=us(cust[:, 1] - t0), mh_done=us(cust[act, 3] - t0), partial=us(cust[:, 5] - t0),
                           next_done=us(cust[:, 6] - t0), l2_seen=us(l2[:, 2] - t0), l2_drawn=us(l2[:, 3] - t0),
                           l2_published=us(l2[:, 4] - t0))
            print(json.dumps(row), flush=True)
    s.close()


if __name__ == "__main__":
    main()
