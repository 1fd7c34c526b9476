"""FGR phases at C3 (ORPCD_FGR_TRACE=1), own features and Q4:  python tools/fgr_phases.py"""
import sys, os, time
sys.path[:0]=['/root/repo/multi-scale-pointcloud-registration_amd','/root/repo']
import numpy as np
from workloads import c3_pair
from orpcd_amd import FastGlobalOptimizer
def rs(c):
    c0=c.mean(axis=0,keepdims=True); return (c-c0)/np.max(np.linalg.norm(c-c0,axis=1))
s,t=c3_pair(100000); s,t=rs(s),rs(t)
for q4 in (False, True):
    opt=FastGlobalOptimizer(seed=0, target_features_from_source=q4)
    opt.optimize(s,t)
    os.environ['ORPCD_FGR_TRACE']='1'
    print('--- q4' if q4 else '--- own', flush=True)
    t0=time.perf_counter(); opt.optimize(s,t); print('total', (time.perf_counter()-t0)*1e3, 'ms', flush=True)
    del os.environ['ORPCD_FGR_TRACE']
