"""The bucketed signed fold's level counts predicted on the CPU (round 5): C4's first n edges mapped bipartite, the
sample's giant component as C, level 1 by source, level 2 by the other end (or by the source again). Prints the
emitted / slow counts the GPU's GELLY_BUCKET_STATS line should match. python tools/sim_bip_levels.py [n]"""
import sys, numpy as np, time
import os
ROOT=os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0]=[ROOT, os.path.join(ROOT,'gelly-streaming_amd')]
from gelly_stream import generators as G
import scipy.sparse as sp, scipy.sparse.csgraph as cg
n=int(sys.argv[1]) if len(sys.argv)>1 else 1<<27
t=time.time()
cfg=G.CONFIGS["c4_kron26"]; E,V=cfg.info()
p=G.to_bipartite(G.generate_host(cfg,0,n)).reshape(-1,2)
print('gen',time.time()-t, p.shape, flush=True)
u=p[:,0].astype(np.int64); v=p[:,1].astype(np.int64)
s=1<<21
A=sp.coo_matrix((np.ones(s,np.int8),(u[:s],v[:s])),shape=(V,V))
nc,lab=cg.connected_components(A,directed=False)
seen=np.zeros(V,bool); seen[u[:s]]=True; seen[v[:s]]=True
cnt=np.bincount(lab[seen]); big=np.argmax(cnt)
C=(lab==big)&seen
print('C size',C.sum(),'even',C[::2].sum(),'odd',C[1::2].sum())
inC=C[u]
print('level1 emitted',inC.sum(),'slow',(~inC).sum())
N1=np.zeros(V,bool); N1[v[inC]]=True
M=C|N1
su,sv=u[~inC],v[~inC]
e2=M[sv]
print('level2 (by target) emitted',e2.sum(),'slow',(~e2).sum())
e2s=M[su]
print('level2 (by source) emitted',e2s.sum())
# a third level, by the source again (the level-2 slow list swapped back)
N2=np.zeros(V,bool); N2[su[e2]]=True
M2=M|N2
s2u,s2v=su[~e2],sv[~e2]
e3=M2[s2u]
print('level3 (by source) emitted',e3.sum(),'slow',(~e3).sum())
in_giant=np.zeros(V,bool)
