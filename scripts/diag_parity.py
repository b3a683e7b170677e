import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np
from oracle import oracle as O
import bayesrrcpp_amd as B
from bayesrrcpp_amd import _lib as L
HYP = dict(sigma0=0.01, v0E=1e-4, s02E=1e-3, v0G=1e-4, s02G=1e-3)
def run(N, P, Bs, cva, sweeps=20):
    X, Y, _ = O.synth_cohort(20261015, N, P, h2=0.5, n_causal=20)
    s = B.Session(L.MODEL_V2, N, P, K=len(cva)+1, block_size=Bs)
    s.upload_x(X).set_y(Y).set_bayesr(**HYP, cva=cva).init(7)
    o = O.Oracle(O.V2, X, Y, cva=cva, seed=7, order_mode=0, block_size=Bs, **HYP)
    for it in range(sweeps):
        s.sweep(1); o.sweep(1)
        bg, bo = s.vector(L.BETA), o.vector(O.V_BETA)
        cg, co = s.vector(L.COMP), o.vector(O.V_COMP)
        eg, eo = s.vector(L.EPS), o.vector(O.V_EPS)
        err = np.max(np.abs(bg-bo)); ee = np.max(np.abs(eg-eo))
        if err > 1e-9 or ee > 1e-9 or not np.array_equal(cg, co):
            bad = np.nonzero(np.abs(bg-bo) > 1e-9)[0]
            print(f"N={N} P={P} B={Bs} K={len(cva)+1}: diverge it={it} beta_err={err:.3g} eps_err={ee:.3g} ncomp_diff={(cg!=co).sum()} bad={bad[:8]} order_pos={[list(o.vector(O.V_ORDER)).index(b) for b in bad[:4]]}")
            print("  sigmaE", s.scalar(L.SIGMAE), o.scalar(O.S_SIGMAE), "mu", s.scalar(L.MU), o.scalar(O.S_MU))
            return
    print(f"N={N} P={P} B={Bs} K={len(cva)+1}: OK {sweeps} sweeps")
for args in [(257,333,64,[1e-3,1e-2]), (257,333,128,[1e-3,1e-2]), (300,333,64,[1e-3,1e-2]), (600,333,64,[1e-3,1e-2]), (257,333,64,[1e-4,1e-3,1e-2]), (3000,512,64,[1e-3,1e-2]), (3000,512,128,[1e-4,1e-3,1e-2])]:
    run(*args)
