"""Debug: xsq after init for a small cohort (GPU)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import bayesrrcpp_amd as B
from bayesrrcpp_amd import _lib as L
from oracle import oracle as O
X, Y, _ = O.synth_cohort(20261015, 300, 500, h2=0.5, n_causal=30)
for pb in ["0", "1"]:
    os.environ["BRR_PER_BLOCK"] = pb
    s = B.Session(L.MODEL_V2, 300, 500, K=4, block_size=128, order_mode=2)
    s.upload_x(X)
    print("after upload |X| col sums", s.vector(200)[:3], "host", np.abs(X[:, :3]).sum(0))
    s.set_y(Y).set_bayesr(cva=[1e-4, 1e-3, 1e-2], sigma0=0.01, v0E=1e-4, s02E=1e-3, v0G=1e-4, s02G=1e-3).init(7)
    print("per_block", pb, "fused wg", s.scalar(104), "xsq[:4]", s.vector(L.XSQ)[:4], "eps[:3]", s.vector(L.EPS)[:3])
    s.sweep(1)
    print("  after sweep beta nz", int(np.count_nonzero(s.vector(L.BETA))), "sigmaE", s.scalar(L.SIGMAE))
