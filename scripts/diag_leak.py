import sys, os, json, subprocess
sys.path.insert(0, os.getcwd())
import numpy as np
from oracle import oracle as O
import bayesrrcpp_amd as B
from bayesrrcpp_amd import _lib as L
HYP = dict(sigma0=0.01, v0E=1e-4, s02E=1e-3, v0G=1e-4, s02G=1e-3)
def gpu(N, P, Bs, cva):
    X, Y, _ = O.synth_cohort(20261015, N, P, h2=0.5, n_causal=20)
    s = B.Session(L.MODEL_V2, N, P, K=len(cva)+1, block_size=Bs)
    s.upload_x(X).set_y(Y).set_bayesr(**HYP, cva=cva).init(7)
    s.sweep(1)
    return s.scalar(L.SIGMAE), s.vector(L.BETA)
def orc(N, P, Bs, cva):
    X, Y, _ = O.synth_cohort(20261015, N, P, h2=0.5, n_causal=20)
    o = O.Oracle(O.V2, X, Y, cva=cva, seed=7, order_mode=0, block_size=Bs, **HYP)
    o.sweep(1)
    return o.scalar(O.S_SIGMAE), o.vector(O.V_BETA)
if len(sys.argv) > 1:
    which, N, P, Bs = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    f = gpu if which == "gpu" else orc
    se, b = f(N, P, Bs, [1e-3, 1e-2])
    print(json.dumps({"se": se, "bsum": float(np.abs(b).sum())}))
    sys.exit(0)
A = (257, 333, 64); Bc = (257, 333, 128)
for f in (gpu, orc):
    f(*A, [1e-3, 1e-2])
    se, b = f(*Bc, [1e-3, 1e-2])
    fresh = json.loads(subprocess.run([sys.executable, __file__, f.__name__, *map(str, Bc)], capture_output=True, text=True).stdout.strip().splitlines()[-1])
    print(f.__name__, "after A:", se, float(np.abs(b).sum()), " fresh:", fresh)
