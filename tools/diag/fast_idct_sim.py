#!/usr/bin/env python3
"""Diagnostic (CPU, oracle only): how often a fast inverse transform (FMA
chains, bound-checked like K1's fast path) could not prove its pixels on the
bench frame.  For each block, Zq = Z * Q (exact), the reference-order float32
U and R of K6 (DCT.cpp:330-334); the bound per output row i is
B_i = kFastBound * (S_i + 0.5 * A) (S_i: the row's sum of |U|, A: the block's
sum of |Zq|); an output fails when clamp(R, -128, 127) lies within B_i of a
half-integer.  Reports the failing share of the non-constant blocks (those
with an AC coefficient: the fused decoder writes DC-only blocks as constants)
and of 16-block units of them (a per-wave test).  Usage:
python3 tools/diag/fast_idct_sim.py
"""
import os, re, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'yuv-manipulations-2_amd')]
from oracle import oracle  # noqa: E402
import myyuv_file  # noqa: E402
src = open(os.path.join(ROOT, 'yuv-manipulations-2_amd', 'csrc', 'codec_common.hpp')).read()
m = re.search(r'#define MYYUV_DCT_MATRIX(.*?)\}', src, re.S)
D = np.array([float(x.strip().rstrip('f')) for x in re.findall(r'[-0-9.e]+f', m.group(1))], np.float32).reshape(8, 8)
g = myyuv_file.YUVFile.load(os.path.join(ROOT, 'tests', 'golden', 'chef-with-trumpet-big-DCT-50.myyuv'))
w, h = g.width, g.height
raw = np.frombuffer(oracle.decompress(g.data, w, h, tuple(g.params)), np.uint8)
planes = [(raw[:w * h].reshape(h, w), 0), (raw[w * h:w * h * 5 // 4].reshape(h // 2, w // 2), 1),
          (raw[w * h * 5 // 4:].reshape(h // 2, w // 2), 1)]
c1 = 4.79e-7  # kFastBound
for q in (50, 90):
    nb_ac = bad_blocks = 0
    bad_units = units = 0
    for pl, ch in planes:
        Q = np.array(oracle.qtable(q, ch), np.float32).reshape(8, 8)
        H, W = pl.shape
        X = (pl.reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 8, 8).astype(np.float64) - 128)
        Y = np.einsum('ik,bkl,vl->biv', D.astype(np.float64), X, D.astype(np.float64))
        Z = np.round(Y / Q).astype(np.float32)  # (statistics: the float64 coefficients)
        Zq = (Z * Q).astype(np.float32)
        ac = (Z.reshape(-1, 64)[:, 1:] != 0).any(1)
        Zq = Zq[ac]
        # reference order: U[i][j] = sum_k D[k][i] * Zq[k][j]; R[i][v] = sum_k U[i][k] * D[k][v]
        U = np.zeros(Zq.shape, np.float32)
        for k in range(8):
            U = (U + (D[k, :][None, :, None] * Zq[:, k, :][:, None, :]).astype(np.float32)).astype(np.float32)
        R = np.zeros(Zq.shape, np.float32)
        for k in range(8):
            R = (R + (U[:, :, k][:, :, None] * D[k, :][None, None, :]).astype(np.float32)).astype(np.float32)
        A = np.abs(Zq).sum((1, 2))
        S = np.abs(U).sum(2)
        B = c1 * (S + 0.5 * A[:, None])
        c = np.clip(R, -128, 127)
        e = np.abs(c - np.round(c))
        fail = ((0.5 - e) <= B[:, :, None]).any((1, 2))
        nb_ac += len(fail)
        bad_blocks += int(fail.sum())
        nu = len(fail) // 16
        units += nu
        bad_units += int(fail[:nu * 16].reshape(nu, 16).any(1).sum())
    print(f"q{q}: blocks with AC {nb_ac}, failing {bad_blocks} ({100 * bad_blocks / nb_ac:.2f} %); "
          f"16-block units {units}, with a failing block {bad_units} ({100 * bad_units / max(units, 1):.1f} %)")
