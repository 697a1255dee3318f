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


def agree_status(dist, code, device):
    """Every rank's status code (0 = ok) on every rank, in rank order: an
    all_gather of one int64 per rank.  The bench calls it after its untimed
    pass and after the timed region, so a rank whose codec failed makes every
    rank exit with the same verdict instead of leaving the others blocked in
    the next collective (SURVEY.md §5 "Batch: a per-rank status allgather")."""
    t = torch.tensor([int(code)], dtype=torch.int64, device=device)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return [int(p.item()) for p in parts]


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


class ChunkedGather:
    """The gather of `gather_streams`, overlapped with the compression.

    Every rank produces the same number of frames, in chunks (the bench: a
    few launch groups).  For chunk c, `add` all-gathers the chunk's u32 sizes
    on a side stream once the chunk's kernels are done (`ready` events), and
    posts the point-to-point transfers of chunk c - 1, whose sizes are on the
    host by then: one packed exact-size message per rank to rank 0, as in
    gather_streams.  So the transfers of a chunk run while the next chunks
    compute, and the host waits only for a size exchange that finished long
    before.  Every rank issues the same collectives in the same order:
    all_gather(0), all_gather(1), P2P(0), all_gather(2), P2P(1), ...

    Local frame i of rank r is global frame r + world * i (shard()).  With
    CPU tensors (gloo tests) there are no streams and every step is eager.

    Sizes are clamped to [0, cap] (the payload slot) on every rank before any
    transfer is sized, so a failed frame (a size past its slot or negative)
    cannot make a sender and rank 0 disagree on a message length, which would
    hang the point-to-point phase; every rank sees the same all-gathered
    sizes, so `bad_ranks` (the ranks that reported such a size) is the same
    set everywhere and the caller's status exchange fails them all cleanly.
    """

    def __init__(self, dist, world, rank, device, cap=None):
        self.dist, self.world, self.rank, self.device = dist, world, rank, device
        self.cap = cap
        self.bad_ranks = set()
        self.bytes = 0  # bytes this rank sent (rank 0: received) so far
        self.cuda = device.type == "cuda"
        self.side = torch.cuda.Stream(device) if self.cuda else None
        self.pending = []  # (local indices, payloads, host sizes [world][k], ready event)
        self.works = []
        self.keep = []
        self.recv = []  # rank 0: (local indices, sizes [world][k], {rank: buffer})
        self.received = 0

    def _stream(self):
        import contextlib
        return torch.cuda.stream(self.side) if self.cuda else contextlib.nullcontext()

    def add(self, local, payloads, sizes, ready=()):
        """local: this chunk's local frame indices (the same list on every
        rank); payloads: tensors holding the streams; sizes: int32 tensor of
        their sizes; ready: CUDA events after which both are valid."""
        k = len(local)
        if self.cuda:
            for e in ready:
                self.side.wait_event(e)
        with self._stream():
            parts = [torch.empty(k, dtype=torch.int32, device=self.device) for _ in range(self.world)]
            self.dist.all_gather(parts, sizes[:k].contiguous())
            stacked = torch.stack(parts)
            if self.cuda:
                hs = torch.empty(stacked.shape, dtype=torch.int32, pin_memory=True)
                hs.copy_(stacked, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.side)
            else:
                hs, ev = stacked.clone(), None
        self.pending.append((list(local), payloads, hs, ev))
        if len(self.pending) > 1:
            self._post(self.pending.pop(0))

    def _post(self, item):
        local, payloads, hs, ev = item
        if ev is not None:
            ev.synchronize()
        hs = hs.tolist()
        for r, row in enumerate(hs):
            for j, n in enumerate(row):
                if n < 0 or (self.cap is not None and n > self.cap):
                    self.bad_ranks.add(r)
                    row[j] = min(max(n, 0), self.cap if self.cap is not None else 0)
        dist, rank = self.dist, self.rank
        with self._stream():
            if rank != 0:
                total = sum(hs[rank])
                if total > 0:
                    packed = torch.cat([p[:n] for p, n in zip(payloads, hs[rank])])
                    self.keep.append(packed)  # alive until finish() has waited
                    self.bytes += total
                    self.works += dist.batch_isend_irecv([dist.P2POp(dist.isend, packed, 0)])
                return
            own = {i: p[:n] for i, p, n in zip(local, payloads, hs[0])}
            bufs, ops = {}, []
            for r in range(1, self.world):
                total = sum(hs[r])
                if total > 0:
                    self.bytes += total
                    bufs[r] = torch.empty(total, dtype=torch.uint8, device=self.device)
                    ops.append(dist.P2POp(dist.irecv, bufs[r], r))
            if ops:
                self.works += dist.batch_isend_irecv(ops)
            self.recv.append((local, hs, bufs, own))

    def finish(self, n_local):
        """Posts what is left and waits for every transfer.  Rank 0 returns
        the world * n_local streams in global frame order; None elsewhere."""
        while self.pending:
            self._post(self.pending.pop(0))
        for w in self.works:
            w.wait()
        if self.rank != 0:
            return None
        out = [None] * (self.world * n_local)
        for local, hs, bufs, own in self.recv:
            for i, t in own.items():
                out[self.world * i] = t
            for r in range(1, self.world):
                off = 0
                for i, n in zip(local, hs[r]):
                    b = bufs.get(r)
                    out[r + self.world * i] = b[off:off + n] if n else torch.empty(0, dtype=torch.uint8,
                                                                                   device=self.device)
                    off += n
        self.received = sum(t is not None for t in out)
        return out
