"""Replays find_best_subset_score (BIC_OLS.cpp:125-172) in Python on
the oracle's stored lists for a hepatitis prefix and reports how many walk
steps the dominated sets need before their first visited key >= -ts, by
parent-set size (wide layers).  Usage:
    python tests/golden/walk_sim.py <columns> <lambda>"""
import sys, numpy as np
import os
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in ('tests', 'urlearning-cpp_amd', 'oracle'):
    sys.path.insert(0, os.path.join(R, p))
import oracle
from test_gpu_wide import load_csv_ascii
cols=int(sys.argv[1]); lam=float(sys.argv[2])
X = load_csv_ascii(os.path.join(R, 'tests', 'golden', 'hepatitis.clean.csv'))[:, :cols]
ds = oracle.Dataset(X); n=cols
def walk(P, pv0, cache, thr, z):
    L=len(pv0)
    pv=[[0]*L for _ in range(L+1)]; pv[0]=list(pv0)
    Ts=[0]*(L+1); idxs=[0]*(L+1); inner=[0]*(L+1); is_=[0]*(L+1); js=[0]*(L+1); us=[0]*(L+1)
    Ts[0]=P; chk={0}; d=0; steps=0; maxd=0
    while True:
        steps+=1
        mm=L-d
        if not inner[d]:
            if idxs[d]==mm:
                if d==0: return False, steps, maxd
                d-=1; chk.add(Ts[d+1]); continue
            u=pv[d][idxs[d]]; T2=Ts[d]^(1<<u)
            if T2 in chk: idxs[d]+=1; continue
            ok = T2 != P and T2 != (P|1) and not ((T2 & 1) and not z)
            if ok and T2 in cache:
                if cache[T2]>=thr: return True, steps, d
                idxs[d]+=1; continue
            inner[d]=1; is_[d]=0; js[d]=0; us[d]=u
            for k in range(mm-1): pv[d+1][k]=0
            continue
        if is_[d]==mm: inner[d]=0; idxs[d]+=1; continue
        pi=pv[d][is_[d]]; is_[d]+=1
        if pi==us[d]: continue
        pv[d+1][js[d]]=pi; js[d]+=1
        Ts[d+1]=Ts[d]^(1<<us[d]); idxs[d+1]=0; inner[d+1]=0
        d+=1; maxd=max(maxd,d)
st_dom=[]; st_sto=[]
for v in range(n):
    s, sc = ds.score_variable(lam, v, (1<<n)-1, n-1)
    cache = {int(a): float(b) for a,b in zip(s,sc)}
    others=[b for b in range(n) if b!=v]; z = v!=0
    for m in range(1, 1<<(n-1)):
        P=0
        for i,b in enumerate(others):
            if m>>i&1: P|=1<<b
        ts = ds.cbic_raw(lam, v, P)
        if ts >= 0: continue
        bits=[b for b in range(n) if P>>b&1]
        # local: pv in global bits; var 0 = bit 0 global ok
        dom, steps, dep = walk(P, bits, cache, -ts, z)
        assert dom == (P not in cache), (v, P)
        (st_dom if dom else st_sto).append((steps, len(bits), dep))
a=np.array(st_dom); b=np.array(st_sto) if st_sto else np.zeros((1,3))
print('dominated', len(a), 'steps mean', a[:,0].mean(), 'p50', np.median(a[:,0]), 'p99', np.percentile(a[:,0],99), 'max', a[:,0].max(), 'depth hist', np.bincount(a[:,2]))
print('stored', len(st_sto), 'steps mean', b[:,0].mean(), 'max', b[:,0].max())
for L in range(1, n):
    sel=a[a[:,1]==L]
    if len(sel): print(L, len(sel), 'mean steps', sel[:,0].mean(), 'max', sel[:,0].max())
