"""Deterministic generators of coefficient blocks and pixel frames that hit the
edge classes of the entropy coder (SURVEY.md §4 "What the build should do"):
all-zero, single symbol, no zeros at all (the freq[0] insert-then-erase path),
13/14, 29/30, 59/60 and 64 distinct symbols (libstdc++ rehash boundaries),
code length 7, and more than 32 symbols of one length (two groups).
Code length 8 is legal in the format but unreachable from the encoder: with at
most 64 samples and libstdc++'s heap tie-breaking the Fibonacci chain breaks on
the first tie (a 200k-block random search around Fibonacci weights found no
length-8 code), so length-8 tables are covered by hand-built chunks in the
decoder tests instead."""
import numpy as np


def _block_with_distinct(rng, n_distinct, zeros="some", lo=-1024, hi=1023):
    """64 zig-zag symbols with exactly n_distinct distinct values."""
    pool = rng.choice(np.arange(lo, hi + 1), size=200, replace=False)
    if zeros == "none":
        pool = pool[pool != 0]
    else:
        pool = pool[pool != 0]
    vals = list(pool[:n_distinct])
    if zeros == "some" and n_distinct >= 2:
        vals[-1] = 0  # zero is one of the distinct symbols
    vals = np.array(vals, dtype=np.int16)
    msg = np.concatenate([vals, rng.choice(vals, 64 - n_distinct)]) if n_distinct < 64 else vals
    rng.shuffle(msg)
    if zeros == "trailing" and n_distinct < 64:
        # message of the distinct symbols followed by trailing zeros
        body = np.concatenate([vals, rng.choice(vals, max(0, 48 - n_distinct))])[: min(64, max(n_distinct, 48))]
        rng.shuffle(body)
        msg = np.zeros(64, np.int16)
        msg[: len(body)] = body
        if msg[len(body) - 1] == 0:
            msg[len(body) - 1] = vals[0] if vals[0] != 0 else 1
    return msg.astype(np.int16)


def fibonacci_block(depth):
    """Frequencies 1,1,1,2,3,5,8,... (Fibonacci) force a code length of `depth`
    (depth 8 needs 55 of the 64 samples)."""
    fib = [1, 1]
    while len(fib) < depth:
        fib.append(fib[-1] + fib[-2])
    freqs = [1] + fib[:depth]
    total = sum(freqs)
    assert total <= 64, total
    freqs[-1] += 64 - total
    msg = []
    for i, f in enumerate(freqs):
        msg += [i + 1] * f
    return np.array(msg, np.int16)


def edge_blocks(seed=7):
    """List of (name, int16[64] zig-zag ordered coefficients)."""
    rng = np.random.default_rng(seed)
    out = [("all_zero", np.zeros(64, np.int16))]
    b = np.zeros(64, np.int16)
    b[0] = 37
    out.append(("dc_only", b))
    out.append(("single_symbol_full", np.full(64, -5, np.int16)))
    b = np.zeros(64, np.int16)
    b[63] = 1
    out.append(("last_only", b))
    out.append(("min_max", np.array([-1024, 1023] * 32, np.int16)))
    for n in (2, 3, 7, 12, 13, 14, 15, 28, 29, 30, 31, 58, 59, 60, 61, 63, 64):
        for zeros in ("none", "some", "trailing"):
            if n == 64 and zeros != "none":
                continue
            for rep in range(3):
                out.append((f"distinct{n}_{zeros}_{rep}", _block_with_distinct(rng, n, zeros)))
    for d in (5, 6, 7, 8):
        blk = fibonacci_block(d)
        out.append((f"fib_depth{d}", blk))
        out.append((f"fib_depth{d}_neg", (-blk).astype(np.int16)))
    # > 32 symbols of one length: 40 distinct, mostly equal frequency
    vals = rng.choice(np.arange(-300, 300), 40, replace=False).astype(np.int16)
    msg = np.concatenate([vals, vals[:24]])
    out.append(("two_groups", msg.astype(np.int16)))
    vals = rng.choice(np.arange(1, 500), 64, replace=False).astype(np.int16)
    out.append(("64_equal", vals))
    # random small-alphabet blocks with trailing zeros, like natural images
    for i in range(200):
        msz = int(rng.integers(1, 65))
        alpha = rng.integers(-8, 9, size=int(rng.integers(1, 12)))
        body = rng.choice(alpha, msz).astype(np.int16)
        if body[-1] == 0:
            body[-1] = 3
        blk = np.zeros(64, np.int16)
        blk[:msz] = body
        out.append((f"natural_{i}", blk))
    for i in range(100):
        out.append((f"uniform_{i}", rng.integers(-1024, 1024, 64).astype(np.int16)))
    return out


def edge_frame(w=256, h=128, seed=11):
    """Pixel frame mixing flat, gradient, checker and noise blocks."""
    rng = np.random.default_rng(seed)
    n = w * h * 3 // 2
    fr = np.empty(n, np.uint8)
    planes = [(0, w, h), (w * h, w // 2, h // 2), (w * h * 5 // 4, w // 2, h // 2)]
    for off, pw, ph in planes:
        p = np.empty((ph, pw), np.uint8)
        for by in range(ph // 8):
            for bx in range(pw // 8):
                kind = (by * 7 + bx * 3) % 6
                if kind == 0:
                    blk = np.full((8, 8), rng.integers(0, 256))
                elif kind == 1:
                    blk = np.add.outer(np.arange(8), np.arange(8)) * rng.integers(1, 16) + rng.integers(0, 64)
                elif kind == 2:
                    blk = ((np.add.outer(np.arange(8), np.arange(8)) % 2) * 255)
                elif kind == 3:
                    blk = rng.integers(0, 256, (8, 8))
                elif kind == 4:
                    blk = rng.integers(120, 136, (8, 8))
                else:
                    blk = np.where(rng.random((8, 8)) < 0.5, 0, 255)
                p[by * 8:(by + 1) * 8, bx * 8:(bx + 1) * 8] = np.clip(blk, 0, 255)
        fr[off: off + pw * ph] = p.ravel()
    return fr
