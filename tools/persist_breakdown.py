#!/usr/bin/env python
"""Timeline of one sweep inside the persistent kernel (diagnostic library libclvmcmc_stamps.so).

Per chain, relative to the moment the level-2 workgroup published the sweep's (beta, Sigma)
(s_memrealtime, 10 ns ticks), medians / maxima over the chain's customer workgroups of:
  observe   publish -> the workgroup holds (beta, Sigma)   coeffs -> log-posterior constants
  MH        the MH steps                                    finish -> state + statistics
  store     block reduce + partial store issued             next   -> draws stored + z / tau of s+1
and the level-2 workgroup's: all partials seen, draw done, next (beta, Sigma) published.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("CLV_LIB_PATH", os.path.join(ROOT, "mcmc_clv_model_amd", "libclvmcmc_stamps.so"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main(workload="c2", sweeps=1500):
    import bench
    from mcmc_clv_model_amd.sampler import HipSampler, build_problem
    df, D, covs, ch, burnin, mcmc, thin, sink = bench.load_workload(workload)
    p = build_problem(df, covs, D)
    s = HipSampler(p, mcmc=mcmc, burnin=burnin, thin=thin, chains=ch, seed=42, draw_sink=sink)
    info = s.launch_info()
    print(info)
    import time
    s.run(200)
    s.synchronize()
    t0 = time.perf_counter()
    s.run(sweeps)
    s.synchronize()
    print(f"wall: {(time.perf_counter() - t0) / sweeps * 1e6:.2f} us per sweep ({os.environ['CLV_LIB_PATH']})")
    if not os.environ["CLV_LIB_PATH"].endswith("_stamps.so"):
        return
    nb = -(-s.n // 256)
    wg = np.zeros(s.chains * (nb + 1) * 12, np.uint64)
    assert s._L.clv_debug_wg_stamps(s.h, wg.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))) == 0
    wg = wg.astype(np.int64).reshape(s.chains, nb + 1, 12)
    print(f"{workload}: persistent={info['persistent']}, chains={s.chains}, N={s.n}, {nb} customer workgroups per chain")
    us = 0.01
    for c in range(s.chains):
        cust, tail = wg[c, :nb], wg[c, nb]
        R = tail[5]
        if R == 0 or (cust[:, 1] == 0).any():
            print(f"  chain {c}: no persistent stamps")
            continue
        act = cust[:, 3] > 0
        cols = dict(observe=cust[:, 1] - R, coeffs=(cust[:, 2] - cust[:, 1])[act], MH=(cust[:, 3] - cust[:, 2])[act],
                    finish=(cust[:, 4] - cust[:, 3])[act], store=cust[:, 5] - cust[:, 4], next=cust[:, 6] - cust[:, 5])
        txt = "  ".join(f"{n} {np.median(v) * us:5.2f}/{v.max() * us:5.2f}" for n, v in cols.items())
        print(f"  chain {c} (median/max us): {txt}")
        # by placement: workgroups on shared CUs (linear dispatch position < P or >= n_cu) vs alone
        T, ncu = info["workgroups"], info["n_cu"]
        pos = cust[:, 11]
        shared = (pos < T - ncu) | (pos >= ncu)
        for tag, m in (("shared", shared), ("alone ", ~shared)):
            if not m.any():
                continue
            ph = dict(top=cust[m, 0] - R, observe=cust[m, 1] - R, MH=cust[m, 3] - cust[m, 2], finish=cust[m, 4] - cust[m, 3],
                      store=cust[m, 5] - cust[m, 4], next=cust[m, 6] - cust[m, 5], partial=cust[m, 5] - R,
                      nextdone=cust[m, 6] - R)
            print(f"    {tag} x{int(m.sum()):3d} (median/max us): " +
                  "  ".join(f"{n} {np.median(v) * us:5.2f}/{v.max() * us:5.2f}" for n, v in ph.items()))
        print(f"    last partial issued {(cust[:, 5].max() - R) * us:6.2f}  tail: variates {(tail[1] - tail[0]) * us:5.2f}"
              f"  partials seen {(tail[2] - R) * us:6.2f}  draw {(tail[3] - tail[2]) * us:5.2f} (reduce {(tail[6] - tail[2]) * us:4.2f}"
              f" algebra {(tail[7] - tail[6]) * us:4.2f} finalize {(tail[3] - tail[7]) * us:4.2f})"
              f"  published {(tail[4] - R) * us:6.2f} us (= sweep period)")
    st = np.zeros(1024 * 8, np.uint64)
    assert s._L.clv_debug_stamps(s.h, st.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))) == 0
    st = st.reshape(1024, 8).astype(np.int64)
    for c in range(min(s.chains, 8)):
        t = np.sort(st[:, c][st[:, c] > 0])
        d = np.diff(t) * us / 4  # every 4th sweep from the launch's first
        print("    per-sweep period by launch position (x400 sweeps):", np.round([d[k:k + 100].mean() for k in range(0, len(d), 100)], 2).tolist())
        if len(d):
            big = np.sort(d)[-5:]
            print(f"  chain {c}: publish-to-publish over {len(d)} sweeps: mean {d.mean():6.2f} median {np.median(d):6.2f}"
                  f"  p10 {np.percentile(d, 10):6.2f}  p90 {np.percentile(d, 90):6.2f}  top5 {np.round(big, 2).tolist()} us;"
                  f" span {(t[-1] - t[0]) * us:8.1f} us")
    s.close()


if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["c2"]), *(int(a) for a in sys.argv[2:3]))
