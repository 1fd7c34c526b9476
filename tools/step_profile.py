"""Host-side profile (cProfile) of 10 C2 multistart steps:  python tools/step_profile.py"""
import sys, os, time, cProfile, pstats
sys.path[:0]=['/root/repo/multi-scale-pointcloud-registration_amd','/root/repo']
import numpy as np
from orpcd_amd import Aligner, GeneralizedICP, Preprocessor
from workloads import c2_pair
s,t=c2_pair(50000); s=Preprocessor([]).preprocess(s); t=Preprocessor([]).preprocess(t)
opt=GeneralizedICP(); al=Aligner(Preprocessor([]),Preprocessor([]),opt,attempts=30)
for k in range(3):
    np.random.seed(1000+k); al.multistart_registration(s,t)
ctx=opt.context
t0=time.perf_counter()
pr=cProfile.Profile(); pr.enable()
for k in range(10):
    np.random.seed(2000+k); al.multistart_registration(s,t)
pr.disable()
el=time.perf_counter()-t0
print('ms/step', el/10*1e3)
st=pstats.Stats(pr); st.sort_stats('tottime').print_stats(12)
