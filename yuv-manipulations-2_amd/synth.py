"""Synthetic IYUV frames of SURVEY.md §8(d), reproducible from their definition.

* tiled: plane_out[y][x] = plane_src[(y + oy) mod Hs][(x + ox) mod Ws] per plane,
  from the decoded chef-big frame (4032x3008); frame f of the batch config
  uses origin (f*8 mod Ws, f*8 mod Hs) (chroma origin halved).
* noise: byte i = byte (i mod 8), little-endian, of splitmix64 output number
  floor(i/8)+1, seed 1234 (first bytes db 1c 18 2f 1b f6 0c bb).
"""
import numpy as np


def splitmix64_bytes(n, seed=1234):
    words = (n + 7) // 8
    gamma = np.uint64(0x9E3779B97F4A7C15)
    idx = np.arange(1, words + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + idx * gamma
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.view(np.uint8)[:n].copy()


def noise_frame(w, h, seed=1234):
    return splitmix64_bytes(w * h * 3 // 2, seed)


def tiled_frame(src_iyuv, ws, hs, w, h, ox=0, oy=0):
    """src_iyuv: bytes/ndarray of a ws x hs IYUV frame."""
    src = np.frombuffer(bytes(src_iyuv), np.uint8) if not isinstance(src_iyuv, np.ndarray) else src_iyuv
    y = src[: ws * hs].reshape(hs, ws)
    u = src[ws * hs: ws * hs * 5 // 4].reshape(hs // 2, ws // 2)
    v = src[ws * hs * 5 // 4: ws * hs * 3 // 2].reshape(hs // 2, ws // 2)

    def tile(p, pw, ph, ox, oy):
        rows = (np.arange(ph) + oy) % p.shape[0]
        cols = (np.arange(pw) + ox) % p.shape[1]
        return p[rows][:, cols]

    out = [tile(y, w, h, ox, oy), tile(u, w // 2, h // 2, ox // 2, oy // 2),
           tile(v, w // 2, h // 2, ox // 2, oy // 2)]
    return np.concatenate([p.ravel() for p in out])


def batch_origin(f, ws, hs):
    return (f * 8) % ws, (f * 8) % hs


def tiled_frame_torch(src, ws, hs, w, h, ox=0, oy=0):
    """tiled_frame on src's device: src is a uint8 tensor holding the ws x hs
    IYUV frame; returns the w x h IYUV frame as a flat uint8 tensor (the
    bench and the GPU tests build the 512-frame batch in HBM this way)."""
    import torch
    dev = src.device
    y = src[: ws * hs].view(hs, ws)
    u = src[ws * hs: ws * hs * 5 // 4].view(hs // 2, ws // 2)
    v = src[ws * hs * 5 // 4: ws * hs * 3 // 2].view(hs // 2, ws // 2)

    def tile(p, pw, ph, ox, oy):
        rows = (torch.arange(ph, device=dev) + oy) % p.shape[0]
        cols = (torch.arange(pw, device=dev) + ox) % p.shape[1]
        return p.index_select(0, rows).index_select(1, cols).reshape(-1)

    return torch.cat([tile(y, w, h, ox, oy), tile(u, w // 2, h // 2, ox // 2, oy // 2),
                      tile(v, w // 2, h // 2, ox // 2, oy // 2)])
