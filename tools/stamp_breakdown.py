#!/usr/bin/env python
"""Where does a sweep launch spend its time?  Runs a workload on the diagnostic library
(libclvmcmc_stamps.so: `make -C mcmc_clv_model_amd/csrc STAMPS=1`) and reports, per launch, the
medians of the in-kernel s_memrealtime stamps (100 MHz):
  customer phase  = last workgroup's end of customer work - first workgroup start
  first/last      = first workgroup end, last workgroup start (relative to first start)
  ticket->tail    = last ticket -> tail start;  tail = fused level-2 draw duration
Diagnostic only: the stamps' atomics perturb the kernel slightly; read shares, not absolutes.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("CLV_LIB_PATH", os.path.join(ROOT, "mcmc_clv_model_amd", "libclvmcmc_stamps.so"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main(workload="c2", sweeps=1500, chains=None):
    import bench
    from mcmc_clv_model_amd.sampler import HipSampler, build_problem
    df, D, covs, ch, burnin, mcmc, thin, sink = bench.load_workload(workload)
    p = build_problem(df, covs, D)
    s = HipSampler(p, mcmc=mcmc, burnin=burnin, thin=thin, chains=chains or ch, seed=42, draw_sink=sink)
    s.run(sweeps)
    st = np.zeros(1024 * 8, np.uint64)
    rc = s._L.clv_debug_stamps(s.h, st.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    assert rc == 0, s._L.clv_last_error()
    st = st.reshape(1024, 8).astype(np.int64)
    ok = (st[:, 3] > 0) & (st[:, 0] > 0)
    st = st[ok]
    us = lambda a: np.median(a) * 0.01  # noqa: E731  (10 ns ticks -> us)
    rel = st - st[:, :1]
    print(f"{workload}: {ok.sum()} launches, chains={chains or ch}, N={len(df)}")
    print(f"  launch total (first start -> tail end): {us(rel[:, 3]):8.2f} us")
    print(f"  customer phase (-> last block end):     {us(rel[:, 1]):8.2f} us")
    print(f"  first block end:                        {us(rel[:, 4]):8.2f} us")
    print(f"  last block start:                       {us(rel[:, 5]):8.2f} us")
    print(f"  last block end -> tail start:           {us(st[:, 2] - st[:, 1]):8.2f} us")
    print(f"  tail (level-2 draw):                    {us(st[:, 3] - st[:, 2]):8.2f} us")
    print(f"    tail: unit reduction                  {us(st[:, 6] - st[:, 2]):8.2f} us")
    print(f"    tail: level-2 algebra (one lane)      {us(st[:, 7] - st[:, 6]):8.2f} us")
    print(f"    tail: record + counters               {us(st[:, 3] - st[:, 7]):8.2f} us")
    if os.environ.get("CLV_STAMP_L2SPLIT"):  # a build with -DCLV_STAMP_L2SPLIT: slot 5 = draw end
        print(f"      algebra: level2_draw                {us(st[:, 5] - st[:, 6]):8.2f} us")
        print(f"      algebra: finalize_hyper             {us(st[:, 7] - st[:, 5]):8.2f} us")
    # placement of the latest launch's workgroups: per CU (XCC, SE, CU) count and durations
    nb = -(-s.n // 256)
    wg = np.zeros(s.chains * (nb + 1) * 12, np.uint64)
    assert s._L.clv_debug_wg_stamps(s.h, wg.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))) == 0
    wg = wg.reshape(-1, 12).astype(np.int64)[:s.chains * nb]
    hw, xcc = wg[:, 2], wg[:, 3] & 0xF
    cu, se = (hw >> 8) & 0xF, (hw >> 13) & 0x7
    key = xcc * 1000 + se * 100 + cu
    uniq, cnt = np.unique(key, return_counts=True)
    dur = (wg[:, 1] - wg[:, 0]) * 0.01
    per_wg_cnt = cnt[np.searchsorted(uniq, key)]
    print(f"  workgroups {len(wg)} on {len(uniq)} CUs; WGs per CU histogram:",
          {int(k): int(v) for k, v in zip(*np.unique(cnt, return_counts=True))})
    for k in sorted(set(per_wg_cnt.tolist())):
        d = dur[per_wg_cnt == k]
        print(f"    CUs with {k} WG(s): WG customer-phase duration median {np.median(d):7.2f} us, max {d.max():7.2f} us")
    ok2 = (wg[:, 7] > wg[:, 4]) & (wg[:, 1] > wg[:, 0])
    clk = (wg[ok2, 7] - wg[ok2, 4]) / ((wg[ok2, 1] - wg[ok2, 0]) * 1e-8) / 1e9
    mh = wg[ok2, 6] - wg[ok2, 5]
    pre = wg[ok2, 5] - wg[ok2, 4]
    post = wg[ok2, 7] - wg[ok2, 6]
    pc = per_wg_cnt[ok2]
    print(f"  shader clock (s_memtime / s_memrealtime): median {np.median(clk):.2f} GHz")
    for k in sorted(set(pc.tolist())):
        sel = pc == k
        bar = (wg[ok2, 8] - wg[ok2, 4])[sel]
        zt = (wg[ok2, 9] - wg[ok2, 8])[sel]
        print(f"    CUs with {k} WG(s): wave-0 cycles  start->barrier {np.median(bar):7.0f}  z/tau {np.median(zt):7.0f}"
              f"  ->MH {np.median(pre[sel] - bar - zt):6.0f}  MH {np.median(mh[sel]):8.0f}"
              f"  finish+reduce {np.median(post[sel]):8.0f}")
    print("  WGs per XCC:", {int(k): int(v) for k, v in zip(*np.unique(xcc, return_counts=True))})
    s.close()


if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["c2"]), *(int(x) for x in sys.argv[2:]))
