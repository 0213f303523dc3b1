#!/usr/bin/env python
"""Where the persistent kernel's workgroups land (diagnostic library libclvmcmc_stamps.so): per
workgroup the HW_ID / XCC_ID recorded in the persistent kernel, the CUs holding two workgroups and
which chains share them, and whether the second round of the dispatch lands on the CUs of the
first (workgroup i + n_cu on the CU of workgroup i, linear dispatch order)."""
import collections
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("CLV_LIB_PATH", os.path.join(ROOT, "mcmc_clv_model_amd", "libclvmcmc_stamps.so"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def cu_key(hw, xcc):
    # gfx9 HW_ID: wave[3:0] simd[5:4] pipe[7:6] cu[11:8] sh[12] se[15:13]
    return (int(xcc) & 0xF, (int(hw) >> 13) & 0x7, (int(hw) >> 12) & 1, (int(hw) >> 8) & 0xF)


def main(workload="c2", sweeps=300):
    import bench
    from mcmc_clv_model_amd.sampler import HipSampler, build_problem
    df, D, covs, ch, burnin, mcmc, thin, sink = bench.load_workload(workload)
    p = build_problem(df, covs, D)
    s = HipSampler(p, mcmc=mcmc, burnin=burnin, thin=thin, chains=ch, seed=42, draw_sink=sink)
    s.run(sweeps)
    s.synchronize()
    nb = -(-s.n // 256)
    wg = np.zeros(s.chains * (nb + 1) * 12, np.uint64)
    assert s._L.clv_debug_wg_stamps(s.h, wg.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))) == 0
    wg = wg.reshape(s.chains, nb + 1, 12)
    where, chain_of = {}, {}
    for c in range(s.chains):
        for b in range(nb + 1):
            if b == nb:
                continue  # the level-2 workgroup records no placement
            lin = int(wg[c, b, 11])  # dispatch position (linear blockIdx)
            where[lin] = cu_key(wg[c, b, 8], wg[c, b, 9])
            chain_of[lin] = c
    per_cu = collections.defaultdict(list)
    for lin, k in where.items():
        per_cu[k].append(lin)
    n_cu = len(per_cu)
    occ = collections.Counter(len(v) for v in per_cu.values())
    print(f"{workload}: {len(where)} workgroups on {n_cu} CUs; workgroups per CU: {dict(occ)}")
    pairs = collections.Counter()
    for v in per_cu.values():
        if len(v) == 2:
            a, b = sorted(v)
            pairs[(chain_of[a], chain_of[b])] += 1
    print("chain pairs on shared CUs (older, younger):", dict(pairs))
    same = sum(1 for lin in where if lin + 256 in where and where[lin] == where[lin + 256])
    print(f"workgroup i and i+256 on the same CU: {same} of {max(0, len(where) - 256)}")
    print("XCC of the first 24 dispatched workgroups:", [where.get(lin, (None,))[0] for lin in range(24)])
    s.close()


if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["c2"]), *(int(a) for a in sys.argv[2:3]))
