"""Host model of k_stream_out_coop's dword ownership (k_stream.hip): a plane
split into tiles of chunks (>= 7 bytes each, at any byte alignment); every
tile claims the dwords whose first byte is its own, finds the chunk holding
that byte from the chunk marks' max-scan, and completes a dword that runs
past a chunk with the next chunk's first bytes (the next tile's first, at a
tile's end); a plane's first and last partial dwords are byte stores.  The
model must write every content byte exactly once, with its chunk's value, and
nothing outside the plane's content.  CPU only: the GPU parity tests check the
kernel's streams against the oracle."""
import random


def model_plane(rnd):
    tiles = [[rnd.randint(7, 40) if rnd.random() < 0.8 else rnd.randint(7, 160)
              for _ in range(rnd.randint(1, 256 if rnd.random() < 0.3 else 40))]
             for _ in range(rnd.randint(1, 5))]
    base = rnd.randint(0, 11)  # the plane's first content byte (any alignment)
    truth, pos = {}, base
    for ti, t in enumerate(tiles):
        for k, sz in enumerate(t):
            for i in range(sz):
                truth[pos + i] = (ti, k, i)
            pos += sz
    end = pos
    written = {}

    def put(b, val):
        written.setdefault(b, []).append(val)

    P0 = base
    for ti, t in enumerate(tiles):
        nloc, tot = len(t), sum(t)
        off = [0]
        for sz in t:
            off.append(off[-1] + sz)
        plane_first, plane_end = ti == 0, ti == len(tiles) - 1
        D0 = (P0 + 3) >> 2
        J = ((P0 + tot - 1) >> 2) - D0 + 1
        lead = 4 * D0 - P0
        if plane_first and lead:
            for k in range(lead):
                put(P0 + k, (ti, 0, k))
        # marks + max-scan: the last chunk whose first dword is at or before j
        marks = [0] * J
        for c in range(nloc):
            jc = 0 if c == 0 else ((P0 + off[c]) >> 2) - D0
            assert 0 <= jc < J and marks[jc] == 0  # one chunk starts per dword at most
            marks[jc] = c + 1
        run = 0
        for j in range(J):
            run = max(run, marks[j])
            D = D0 + j
            b = 4 * D - P0
            c = run - 1
            if off[c] > b:
                c -= 1
            avail = off[c + 1] - b
            if avail < 4 and c + 1 == nloc and plane_end:
                for i in range(avail):
                    put(4 * D + i, (ti, c, b - off[c] + i))
                continue
            for i in range(4):
                if i < avail:
                    put(4 * D + i, (ti, c, b - off[c] + i))
                elif c + 1 < nloc:
                    put(4 * D + i, (ti, c + 1, i - avail))
                else:
                    put(4 * D + i, (ti + 1, 0, i - avail))
        P0 += tot
    return truth, written, base, end


def test_every_byte_written_once_with_its_value():
    rnd = random.Random(2024)
    for _ in range(500):
        truth, written, base, end = model_plane(rnd)
        for b in range(base, end):
            assert written.get(b) == [truth[b]], b
        assert all(base <= b < end for b in written)
