import sys, os, gc
sys.path.insert(0, os.getcwd())
import numpy as np
from oracle import oracle as O
import bayesrrcpp_amd as B
from bayesrrcpp_amd import _lib as L
HYP = dict(sigma0=0.01, v0E=1e-4, s02E=1e-3, v0G=1e-4, s02G=1e-3)
def mk(N, P, Bs, cva=[1e-3, 1e-2], order=0):
    X, Y, _ = O.synth_cohort(20261015, N, P, h2=0.5, n_causal=20)
    s = B.Session(L.MODEL_V2, N, P, K=len(cva)+1, block_size=Bs, order_mode=order)
    s.upload_x(X).set_y(Y).set_bayesr(**HYP, cva=cva).init(7)
    o = O.Oracle(O.V2, X, Y, cva=cva, seed=7, order_mode=order, block_size=Bs, **HYP)
    return s, o
def check(tag, s, o, sweeps=1):
    for it in range(sweeps):
        s.sweep(1); o.sweep(1)
    bg, bo = s.vector(L.BETA), o.vector(O.V_BETA)
    ordr = o.vector(O.V_ORDER).astype(int)
    pos = {m: i for i, m in enumerate(ordr)}
    bad = np.nonzero(np.abs(bg - bo) > 1e-9)[0]
    first = min([pos[b] for b in bad]) if len(bad) else None
    print(f"{tag}: nbad={len(bad)} first_bad_pos={first} eps_err={np.max(np.abs(s.vector(L.EPS)-o.vector(O.V_EPS))):.2e}")
# 1) A alive while B runs
sA, oA = mk(257, 333, 64); sA.sweep(1)
sB, oB = mk(257, 333, 128); check("B with A alive", sB, oB)
del sA, oA, sB, oB; gc.collect()
# 2) A destroyed then B
sA, oA = mk(257, 333, 64); sA.sweep(1); del sA, oA; gc.collect()
sB, oB = mk(257, 333, 128); check("B after A destroyed", sB, oB)
del sB, oB; gc.collect()
# 3) one-block problems after A
sA, oA = mk(257, 333, 64); sA.sweep(1); del sA, oA; gc.collect()
for P in (64, 128, 256):
    s, o = mk(257, P, 128, order=2); check(f"IDENTITY P={P} B=128", s, o)
    del s, o; gc.collect()
s, o = mk(257, 333, 128, order=2); check("IDENTITY P=333 B=128", s, o)
