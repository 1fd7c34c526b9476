import sys, os
sys.path[:0]=['multi-scale-pointcloud-registration_amd','.']
import numpy as np
from orpcd_amd import _native
from workloads import c5_pair
s,t=c5_pair()
ctx=_native.Context(0)
ctx.set_option("sched", int(sys.argv[1]))
ctx.set_target(t); ctx.set_source(s)
r=ctx.gicp_batch(np.eye(3)[None], np.zeros((1,3)), max_iteration=int(sys.argv[2]))
print("ok", r["iters"], r["rmse"], flush=True)
