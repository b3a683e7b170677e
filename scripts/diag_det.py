import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np
from oracle import oracle as O
import bayesrrcpp_amd as B
from bayesrrcpp_amd import _lib as L
HYP = dict(sigma0=0.01, v0E=1e-4, s02E=1e-3, v0G=1e-4, s02G=1e-3)
cfg = [int(a) for a in sys.argv[1:4]]
N, P, Bs = cfg
cva = [1e-3, 1e-2]
X, Y, _ = O.synth_cohort(20261015, N, P, h2=0.5, n_causal=20)
def gpu_run(sweeps=3):
    s = B.Session(L.MODEL_V2, N, P, K=3, block_size=Bs)
    s.upload_x(X).set_y(Y).set_bayesr(**HYP, cva=cva).init(7)
    out = []
    for it in range(sweeps):
        s.sweep(1); out.append((s.vector(L.BETA), s.vector(L.EPS), s.scalar(L.SIGMAE)))
    return out
o = O.Oracle(O.V2, X, Y, cva=cva, seed=7, order_mode=0, block_size=Bs, **HYP)
oo = []
for it in range(3):
    o.sweep(1); oo.append((o.vector(O.V_BETA), o.vector(O.V_EPS), o.scalar(O.S_SIGMAE)))
for rep in range(3):
    g = gpu_run()
    msg = []
    for it in range(3):
        msg.append(f"it{it}: d_oracle={np.max(np.abs(g[it][0]-oo[it][0])):.2e}")
    print(f"N={N} P={P} B={Bs} rep={rep}", " ".join(msg))
