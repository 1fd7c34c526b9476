import sys, os, numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO, os.path.join(REPO, "oracle")]
import oracle
from orpcd_amd import _native
from workloads import c3_pair
s, t = c3_pair()
s, _, _ = oracle.radius_scale(s); t, _, _ = oracle.radius_scale(t)
ctx = _native.Context(0)
on, of = oracle.fpfh(s, 0.1, 20, 0.1, 20)
gn, gf = ctx.fpfh(s, 0.1, 20, 0.1, 20)
print("normals max diff", np.abs(gn - on).max(), "bitwise equal rows", np.mean(np.all(gn == on, axis=1)))
bad = ~np.all(np.abs(gf - of) <= 1e-9, axis=1)
print("fpfh rows differing", bad.sum(), "max", np.abs(gf - of).max())
# feature NN with oracle features on both sides vs GPU
gi = ctx.feature_nn(of, of)
print("self-NN == identity", np.mean(gi == np.arange(len(of))))
o = oracle.fgr(s, t, of, of, seed=0)
g = ctx.fgr(s, t, of, of, seed=0)
print("fgr same feats: n_mutual", o["n_mutual"], g["n_mutual"], "dT", np.abs(o["T"] - g["T"]).max())
g2 = ctx.fgr(s, t, gf, gf, seed=0)
print("fgr gpu feats: n_mutual", g2["n_mutual"], "dT", np.abs(o["T"] - g2["T"]).max())
