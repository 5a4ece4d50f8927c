import time, sys
import numpy as np
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from vvc_amd import parser as PZ
d=open(__import__('os').path.join(__import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))), 'tests/golden/streams/ra2160l_q27.bin'),'rb').read()
best=[1e9,1e9]
for rep in range(6):
    s=PZ.Stream(d); tp=td=0
    for i in range(len(s)):
        t=time.perf_counter(); s.parse(i); t1=time.perf_counter(); s.derive(i); t2=time.perf_counter()
        tp+=t1-t; td+=t2-t1
        n = s.dmvr_split(i, 0, 1 << 30)[1]
        s.refine(i, np.zeros((n, 2), np.int32))
    best=[min(best[0],tp),min(best[1],td)]
    s.close()
print("parse %.1f ms derive %.1f ms" % (best[0]*1e3, best[1]*1e3))
