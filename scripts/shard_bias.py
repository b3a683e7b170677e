#!/usr/bin/env python3
"""Column-shard bias of the CPU oracle (SURVEY 8e protocol): posterior means of sigmaE, sigmaG,
h2 = sigmaG / (sigmaG + sigmaE) and the number of non-zero effects for S = 1, 2, 4, 8 column
shards (one residual exchange per sweep, or E exchanges per sweep), against the 1-shard chain, on
a C5-like aspect (N >> P / shard).  Prints one JSON line per configuration.

  python scripts/shard_bias.py [--N 4000] [--P 2000] [--keep 3000] [--burn 300] [--B 64]
"""
import argparse
import json
import os
import sys
from multiprocessing import Pool

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
HYP = dict(sigma0=0.01, v0E=1e-4, s02E=1e-3, v0G=1e-4, s02G=1e-3)
CVA = [1e-4, 1e-3, 1e-2]


def chain(job):
    from oracle import oracle as O
    a, S, E, seed = job
    X, Y, _ = O.synth_cohort(20261015, a.N, a.P, h2=0.5)
    o = O.Oracle(O.V2, X, Y, cva=CVA, seed=seed, order_mode=O.ORDER_BLOCKED, block_size=a.B,
                 n_shards=S, n_exchanges=E, **HYP)
    o.sweep(a.burn)
    rows = []
    for _ in range(a.keep):
        o.sweep(1)
        se, sg = o.scalar(O.S_SIGMAE), o.scalar(O.S_SIGMAG)
        rows.append([se, sg, sg / (sg + se), np.count_nonzero(o.vector(O.V_BETA))])
    return (S, E, seed), np.array(rows)


def mean_se(a, nb=30):
    a = a[: len(a) // nb * nb].reshape(nb, -1, a.shape[1]).mean(axis=1)
    return a.mean(axis=0), a.std(axis=0, ddof=1) / np.sqrt(nb)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=4000)
    ap.add_argument("--P", type=int, default=2000)
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--burn", type=int, default=300)
    ap.add_argument("--keep", type=int, default=3000)
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--configs", default="1:1:11,1:1:12,2:1:21,4:1:41,8:1:81,8:2:82,8:4:84,8:8:88")
    a = ap.parse_args()
    from oracle import oracle as O
    O.build()
    jobs = [(a,) + tuple(int(v) for v in c.split(":")) for c in a.configs.split(",")]
    with Pool(min(a.procs, len(jobs))) as pool:
        res = dict(pool.map(chain, jobs))
    base = [k for k in res if k[0] == 1][0]
    mb, sb = mean_se(res[base])
    names = ["sigmaE", "sigmaG", "h2", "nonzero"]
    for k, r in res.items():
        m, s = mean_se(r)
        z = (m - mb) / np.sqrt(s ** 2 + sb ** 2)
        print(json.dumps({"N": a.N, "P": a.P, "B": a.B, "shards": k[0], "exchanges_per_sweep": k[1], "seed": k[2],
                          "mean": dict(zip(names, np.round(m, 6).tolist())),
                          "mc_se": dict(zip(names, np.round(s, 6).tolist())),
                          "rel_shift_vs_1shard": dict(zip(names, np.round((m - mb) / mb, 5).tolist())),
                          "z_vs_1shard": dict(zip(names, np.round(z, 2).tolist()))}), flush=True)


if __name__ == "__main__":
    main()
