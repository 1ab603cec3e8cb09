#!/usr/bin/env python3
"""Study behind the row DARE kernel's exchange-free inverse (DESIGN.md §3 "Row DARE"):
the SDA doubling matrices W = I + G H of many DARE problems inverted by
Gauss-Jordan WITHOUT row exchanges (numpy, FP64) against np.linalg.inv:
largest relative error of the inverse, smallest pivot / row-max ratio and the
doublings to convergence, per problem family — hover 6 / 9 states with random
SPD Q and R and random mass, hover with diagonal tuner-range weights, and the
random general systems of the GPU tests.  CPU only; output in
profiles/r04/dare_nopivot_study.txt.

  python scripts/dare_nopivot_study.py
"""
import os
import sys

import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lqr-quadcopter-test_amd"))
from quadtrack.controllers.riccati_lqr import build_augmented_lqi_system, build_linearized_system  # noqa: E402


def system(n, dt, mass=1.0):
    """The hover model (riccati_lqr.py:187-316): 6-state, or the 9-state LQI augmentation."""
    A, B = build_linearized_system(dt, mass)
    return build_augmented_lqi_system(A, B, dt) if n == 9 else (A, B)


def gj_nopiv(W):
    a=W.copy(); n=len(a)
    minratio=np.inf
    for k in range(n):
        p=a[k,k]
        minratio=min(minratio, abs(p)/np.max(np.abs(a[k])))
        for i in range(n):
            if i==k: continue
            f=a[i,k]/p
            a[i,:]-=f*a[k,:]
            a[i,k]=-f
        a[k,:]/=p; a[k,k]=1/p
    return a, minratio

def sda(A,B,Q,R, it=64):
    G=B@np.linalg.solve(R,B.T); H=Q.copy(); A=A.copy()
    worst=0; minr=np.inf
    for k in range(it):
        W=np.eye(len(A))+G@H
        Wi,mr=gj_nopiv(W); minr=min(minr,mr)
        ref=np.linalg.inv(W)
        err=np.max(np.abs(Wi-ref))/np.max(np.abs(ref))
        worst=max(worst,err)
        Y1=Wi@A; Y2=Wi@G
        Hn=H+A.T@H@Y1; G=G+A@Y2@A.T; A=A@Y1
        d=np.linalg.norm(Hn-H); H=Hn
        if d<=1e-14*np.linalg.norm(H): break
    return worst, minr, k+1

rng=np.random.default_rng(0)
rows=[]
# hover systems
for n in (6,9):
    for trial in range(200):
        A,B=system(n,0.01,rng.uniform(0.5,2.0))
        M=rng.normal(size=(n,n)); Q=M@M.T*rng.uniform(1e-4,10)+np.eye(n)*rng.uniform(0,1e-3)
        L=rng.normal(size=(4,4))*0.3; R=L@L.T+np.eye(4)
        rows.append(('hover%d'%n,)+sda(A,B,Q,R))
    for trial in range(200):
        A,B=system(n,0.01)
        qd=np.concatenate([rng.uniform([5e-5,5e-5,10],[5e-4,5e-4,25]),rng.uniform([1e-3,1e-3,2],[1e-2,1e-2,8])]+([rng.uniform([1e-4]*3,[1e-2]*3)] if n==9 else []))
        rows.append(('diag%d'%n,)+sda(A,B,np.diag(qd),np.diag(rng.uniform(0.5,2,4))))
# random general (test-like)
for n,p in ((1,1),(3,8),(16,1),(16,8),(10,6),(2,1),(5,2),(9,4),(12,5)):
    for trial in range(67):
        A=rng.normal(size=(n,n))*(0.4/np.sqrt(n))+np.eye(n)*0.6
        B=rng.normal(size=(n,p)); M=rng.normal(size=(n,n)); Q=M@M.T+np.eye(n)*0.1
        L=rng.normal(size=(p,p))*0.3; R=L@L.T+np.eye(p)
        rows.append(('rand%d_%d'%(n,p),)+sda(A,B,Q,R))
import collections
agg=collections.defaultdict(lambda:[0,np.inf,0])
for name,w,mr,it in rows:
    a=agg[name]; a[0]=max(a[0],w); a[1]=min(a[1],mr); a[2]=max(a[2],it)
for k,v in agg.items(): print(k, 'max inv rel err %.2e'%v[0], 'min pivot ratio %.2e'%v[1], 'max it',v[2])
