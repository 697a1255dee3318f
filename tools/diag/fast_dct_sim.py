#!/usr/bin/env python3
"""Diagnostic (CPU, oracle only): how often K1's fast forward transform (FMA
chains, xform_common.hpp fdct_core) must fall back to the reference-order
transform on the bench frame: per 16-block unit, whether any output's t = Y *
fl(1/Q) lies within beta = B * r * (1 + 2^-20) + |t| * 2^-21 of a
half-integer, with B = kFastBound * (S_i + 0.5 * A) (S_i: the row's sum of
|T|, A: the block's sum of |x|).  Y and T here are the reference-order float32
values (the fast values differ from them by at most B, which moves the count
by a negligible amount).  Also reports today's near-tie units (the divide
fallback alone).  Usage: python3 tools/diag/fast_dct_sim.py
"""
import os, sys, numpy as np, re
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'yuv-manipulations-2_amd')]
from oracle import oracle
import myyuv_file
src=open(os.path.join(ROOT, 'yuv-manipulations-2_amd', 'csrc', 'codec_common.hpp')).read()
m=re.search(r'#define MYYUV_DCT_MATRIX(.*?)\}', src, re.S)
D=np.array([float(x.strip().rstrip('f')) for x in re.findall(r'[-0-9.e]+f', m.group(1))],np.float32).reshape(8,8)
g = myyuv_file.YUVFile.load(os.path.join(ROOT, 'tests', 'golden', 'chef-with-trumpet-big-DCT-50.myyuv'))
w,h=g.width,g.height
raw=np.frombuffer(oracle.decompress(g.data,w,h,tuple(g.params)),np.uint8)
planes=[(raw[:w*h].reshape(h,w),0),(raw[w*h:w*h*5//4].reshape(h//2,w//2),1),(raw[w*h*5//4:].reshape(h//2,w//2),1)]
u=2.0**-24; g8=8*u/(1-8*u); dmax=0.5
c1=4.79e-7  # kFastBound
for q in (50,90,100):
  tot_units=0; bad_units=0; bad_out=0; nout=0; old_units=0
  for pl,ch in planes:
    Q=np.array(oracle.qtable(q,ch),np.float32).reshape(8,8)
    H,W=pl.shape
    X=(pl.reshape(H//8,8,W//8,8).transpose(0,2,1,3).reshape(-1,8,8).astype(np.int32)-128).astype(np.float32)
    # reference-order float32 T and Y
    T=np.zeros(X.shape,np.float32)
    for k in range(8): T=(T+(D[:,k][None,:,None]*X[:,k,:][:,None,:]).astype(np.float32)).astype(np.float32)
    Y=np.zeros(X.shape,np.float32)
    for k in range(8): Y=(Y+(T[:,:,k][:,:,None]*D[:,k][None,None,:]).astype(np.float32)).astype(np.float32)
    A=np.abs(X).sum((1,2))           # per block
    S=np.abs(T).sum(2)               # per block, row i
    B=c1*(S+dmax*A[:,None])          # per row
    r=(np.float32(1)/Q).astype(np.float32)
    t=(Y*r[None]).astype(np.float32)
    e=np.abs(t-np.rint(t))
    old=(np.abs(t)*2**-21+e)>=0.5
    new=(np.abs(t)*2**-21+e+B[:,:,None]*r[None]*(1+2**-20))>=0.5
    nb=len(X); nu=(nb+15)//16
    pad=nu*16-nb
    nbad=np.concatenate([new.reshape(nb,-1).any(1), np.zeros(pad,bool)]).reshape(nu,16).any(1)
    obad=np.concatenate([old.reshape(nb,-1).any(1), np.zeros(pad,bool)]).reshape(nu,16).any(1)
    tot_units+=nu; bad_units+=nbad.sum(); old_units+=obad.sum(); bad_out+=new.sum(); nout+=new.size
  print(f"q{q}: units needing the exact path {bad_units}/{tot_units} = {bad_units/tot_units:.4f} (near-tie units today {old_units/tot_units:.4f}); unsafe outputs {bad_out/nout:.2e}")
