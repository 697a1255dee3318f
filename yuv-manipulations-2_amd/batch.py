"""Multi-GPU batch driver: independent IYUV frames sharded one frame per GPU
(BASELINE.json configs[3]), compressed where they live, and the
compressed streams gathered to rank 0 — the one exchange step of the path.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI on
the GPU box; "gloo" for the CPU tests).  The gather is two collectives:
  1. all_gather of the per-frame u32 payload sizes (fixed shape),
  2. one exact-size point-to-point transfer per rank to rank 0: each rank
     packs its streams back to back (no padding to a worst case), rank 0
     posts one receive per rank (batch_isend_irecv) and splits the buffers
     by the gathered sizes.  A few large messages keep every xGMI link busy;
     one message per frame would be thousands of small RCCL operations.
The codec itself is a callable, so the same driver runs the HIP codec
(myyuv_hip, device tensors) or, in tests, the CPU restatement (host tensors).
"""
import torch


def shard(n_frames, world, rank):
    """Frame f goes to rank f mod world (round-robin)."""
    return list(range(rank, n_frames, world))


def gather_streams(dist, payloads, sizes, n_frames, world, rank, device):
    """Collect every rank's compressed streams on rank 0.

    payloads: list of uint8 tensors (each at least sizes[i] long), in the
    order of shard(n_frames, world, rank); sizes: int32 tensor of the same
    length (on `device`).  Returns, on rank 0, the list of n_frames payload
    tensors in frame order; None elsewhere.
    """
    per = (n_frames + world - 1) // world
    mine = torch.zeros(per, dtype=torch.int32, device=device)
    if len(payloads):
        mine[: len(payloads)] = sizes[: len(payloads)]
    parts = [torch.empty(per, dtype=torch.int32, device=device) for _ in range(world)]
    dist.all_gather(parts, mine)
    hs = [p.cpu().tolist() for p in parts]
    counts = [len(shard(n_frames, world, r)) for r in range(world)]
    totals = [sum(hs[r][: counts[r]]) for r in range(world)]
    if rank != 0:
        if totals[rank] > 0:
            packed = torch.cat([payloads[i][: hs[rank][i]] for i in range(counts[rank])])
            for req in dist.batch_isend_irecv([dist.P2POp(dist.isend, packed, 0)]):
                req.wait()
        return None
    out = [None] * n_frames
    for i, f in enumerate(shard(n_frames, world, 0)):
        out[f] = payloads[i][: hs[0][i]]
    bufs, ops = {}, []
    for r in range(1, world):
        if totals[r] > 0:
            bufs[r] = torch.empty(totals[r], dtype=torch.uint8, device=device)
            ops.append(dist.P2POp(dist.irecv, bufs[r], r))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    for r in range(1, world):
        off = 0
        for i, f in enumerate(shard(n_frames, world, r)):
            n = hs[r][i]
            out[f] = bufs[r][off:off + n] if n else torch.empty(0, dtype=torch.uint8, device=device)
            off += n
    return out


def run_batch(dist, frames, compress, n_frames, world, rank, device):
    """Compress this rank's shard with `compress(frame_index) -> (payload
    tensor, size tensor)` and gather all streams to rank 0."""
    payloads, sizes = [], []
    for f in shard(n_frames, world, rank):
        p, s = compress(f)
        payloads.append(p)
        sizes.append(s.reshape(1))
    size_t = torch.cat(sizes) if sizes else torch.zeros(0, dtype=torch.int32, device=device)
    return gather_streams(dist, payloads, size_t.to(torch.int32), n_frames, world, rank, device)
