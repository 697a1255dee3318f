"""Diagnostic (CPU, oracle only): wave iterations of the decoder's symbol loop
under alternative schedules, on the bench frame (chef-big, q50 by default).

  cur   : today's k_decode_idct — lane per block, 64-block waves, the unrolled
          loop runs 8 * ceil(max msz / 8) positions per wave;
  skip  : lane per block, a step decodes one nonzero symbol or one whole run of
          zero symbols: max over lanes of (nonzeros + zero runs);
  queue : waves of G blocks, a lane takes the next unassigned block when its
          block is done (greedy, in block order): makespan of per-block
          cost msz (queue) or nonzeros + zero runs (queue+skip), plus one
          switch step per block.

  python tools/k5_queue_sim.py [quality] [group]
"""
import os
import sys
import heapq

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yuv-manipulations-2_amd")]
from oracle import oracle  # noqa: E402
import myyuv_file  # noqa: E402

ZZ = np.array([0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27,
               20, 13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
               58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63])


def block_costs(C):
    Z = C.reshape(-1, 64)[:, ZZ]
    nz = Z != 0
    last = np.where(nz.any(1), 63 - np.argmax(nz[:, ::-1], axis=1), 0)
    msz = last + 1
    pos = np.arange(64)[None, :]
    inmsg = pos < msz[:, None]
    nnz = (nz & inmsg).sum(1)
    zero = (~nz) & inmsg
    starts = zero & ~np.concatenate([np.zeros((len(Z), 1), bool), zero[:, :-1]], 1)
    runs = starts.sum(1)
    return msz, nnz + runs


def makespan(costs, lanes=64, switch=1):
    h = [0] * lanes
    for c in costs:
        t = heapq.heappop(h)
        heapq.heappush(h, t + c + switch)
    return max(h)


def main():
    q = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    G = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    g = myyuv_file.YUVFile.load(os.path.join(ROOT, "tests/golden/chef-with-trumpet-big-DCT-50.myyuv"))
    w, h = g.width, g.height
    raw = np.frombuffer(oracle.decompress(g.data, w, h, tuple(g.params)), np.uint8)
    planes = [(raw[:w * h].reshape(h, w), 0), (raw[w * h:w * h * 5 // 4].reshape(h // 2, w // 2), 1),
              (raw[w * h * 5 // 4:].reshape(h // 2, w // 2), 1)]
    tot = {"cur": 0, "skip": 0, "queue": 0, "queue+skip": 0, "sum_msz": 0, "sum_skip": 0, "waves64": 0}
    for pl, chroma in planes:
        Q = oracle.qtable(q, chroma)
        H, W = pl.shape
        blks = pl.reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64)
        C = np.stack([oracle.fdct_block(np.ascontiguousarray(b), Q) for b in blks])
        msz, sk = block_costs(C)
        tot["sum_msz"] += int(msz.sum())
        tot["sum_skip"] += int(sk.sum())
        for a in range(0, len(msz), 64):
            m = msz[a:a + 64]
            tot["cur"] += 8 * int(np.ceil(m.max() / 8))
            tot["skip"] += int(sk[a:a + 64].max())
            tot["waves64"] += 1
        for a in range(0, len(msz), G):
            tot["queue"] += makespan(msz[a:a + G])
            tot["queue+skip"] += makespan(sk[a:a + G])
    print(f"q{q}, queue groups of {G} blocks: {tot}")
    print(f"lane efficiency today {tot['sum_msz'] / (64 * tot['cur']):.3f}")


if __name__ == "__main__":
    main()
