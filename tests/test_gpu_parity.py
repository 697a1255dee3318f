"""GPU parity: the HIP path (libmyyuv_hip.so through its C ABI) against the
CPU restatement (oracle/), the reference's golden files, and — when the
reference library built by oracle/Makefile is present — the reference itself.
Integer/byte work: every comparison is bit-exact."""
import hashlib
import os

import numpy as np
import pytest

import blockgen

pytestmark = pytest.mark.gpu

SMALL_W, SMALL_H = 992, 736


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.mark.parametrize("q,gold", [(50, "chef-with-trumpet-DCT-50.myyuv"),
                                    (90, "chef-with-trumpet-DCT-90.myyuv")])
def test_golden_compress_small(codec, golden, q, gold):
    raw = golden("chef-with-trumpet.myyuv")
    g = golden(gold)
    pay = codec.compress(raw.data, raw.width, raw.height, (q, q, q))
    assert pay == g.data
    # whole file, as myyuv_cli -compress writes it
    assert sha(raw.compressed(bytes([q] * 3), pay).dumps()) == sha(g.dumps())


@pytest.mark.parametrize("gold", ["chef-with-trumpet-DCT-50.myyuv", "chef-with-trumpet-DCT-90.myyuv"])
def test_golden_decompress_small(codec, golden, oracle, gold):
    g = golden(gold)
    out = codec.decompress(g.data, g.width, g.height, tuple(g.params))
    assert out == oracle.decompress(g.data, g.width, g.height, tuple(g.params))


def test_golden_decompress_small_known_hash(codec, golden):
    g = golden("chef-with-trumpet-DCT-50.myyuv")
    out = codec.decompress(g.data, g.width, g.height, tuple(g.params))
    assert sha(g.decompressed(out).dumps()) == \
        "a95127da471524c1f7860c47d9b11e2c835ffa220c6d7aadf71e0fb6e45a9306"


def test_golden_big_roundtrip(codec, golden, chef_big):
    f, raw_oracle = chef_big
    raw = codec.decompress(f.data, f.width, f.height, tuple(f.params))
    assert raw == raw_oracle
    dec_file = f.decompressed(raw)
    assert sha(dec_file.dumps()) == "5e7769191188285cc127c6b4da900b3420f064191f707383c82128c14e497e5c"
    pay = codec.compress(raw, f.width, f.height, (50, 50, 50))
    assert len(pay) == 3363749
    assert sha(pay) == "fe9b7317653c2b44a9f24436f0e349b083b4e368cf9653e8777e9f7a79cebfcc"
    assert sha(dec_file.compressed(b"222", pay).dumps()) == \
        "18405d3e6f79a0054fbdb166ae76f58d8dbffc605263f4c3c0b65e51babefbf7"


def test_golden_big_decode_repeat(codec, chef_big):
    """Repeated decodes of the 4K stream stay bit-exact (guards against
    schedule-dependent results: a K5 variant once decoded ~1% of the blocks
    wrongly, differently on every run)."""
    f, raw_oracle = chef_big
    for _ in range(4):
        assert codec.decompress(f.data, f.width, f.height, tuple(f.params)) == raw_oracle


@pytest.mark.parametrize("q", [1, 5, 25, 50, 51, 75, 90, 99, 100])
def test_edge_frame_vs_oracle(codec, oracle, q):
    w, h = 256, 128
    fr = blockgen.edge_frame(w, h)
    pay = codec.compress(fr.tobytes(), w, h, (q, q, q))
    assert pay == oracle.compress(fr.tobytes(), w, h, (q, q, q))
    assert codec.decompress(pay, w, h, (q, q, q)) == oracle.decompress(pay, w, h, (q, q, q))


@pytest.mark.parametrize("q", [(50, 50, 50), (90, 90, 90), (100, 100, 100), (10, 60, 95)])
def test_noise_vs_oracle(codec, oracle, q):
    import synth
    w, h = 512, 256
    fr = synth.noise_frame(w, h)
    pay = codec.compress(fr.tobytes(), w, h, q)
    assert pay == oracle.compress(fr.tobytes(), w, h, q)
    assert codec.decompress(pay, w, h, q) == oracle.decompress(pay, w, h, q)


@pytest.mark.gpu
@pytest.mark.parametrize("q,fix_grid", [((90, 90, 90), None), ((100, 100, 100), None),
                                        ((50, 50, 50), "8"), ((75, 75, 75), "8")])
def test_fdct_unproven_units_listed_in_batches(oracle, q, fix_grid):
    """K1 appends every unit its fast path cannot prove to one of 32 device
    lists (unit ua to list ua % 32, one atomic counter per list) and
    k_fdct_fix transforms the listed units in the reference's order
    (k_transform.hip).  A K1 grid of 1 % of the resident workgroups
    (MYYUV_K1_GRID_PCT) gives each wave hundreds of units of a noise batch,
    a third or more of them unproven; with MYYUV_FIX_GRID=8 (q <= 75) the fix
    kernel has 32 waves, one per list, so each walks its list's many entries
    grid-stride.  Every frame must equal the oracle's."""
    import myyuv_hip
    import synth

    env = {"MYYUV_K1_GRID_PCT": "1", "MYYUV_FIX_GRID": fix_grid}
    old = {k: os.environ.get(k) for k in env}
    for k, v in env.items():
        if v is not None:
            os.environ[k] = v
    try:
        c = myyuv_hip.Codec(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    try:
        w, h = 2048, 1024  # 12,288 units over ~80 waves
        frames = [synth.noise_frame(w, h, seed=s).tobytes() for s in range(3)]
        frames.append(blockgen.edge_frame(w, h, seed=5).tobytes())
        got = c.compress_batch(frames, w, h, q)
        for f, p in zip(frames, got):
            assert p == oracle.compress(f, w, h, q)
    finally:
        c.close()


@pytest.mark.parametrize("q", [(50, 50, 50), (100, 100, 100)])
def test_noise_long_overflow_list(codec, oracle, q):
    """A noise frame whose blocks nearly all exceed 8 distinct symbols: the
    single frame's overflow worklist is longer than kR16GateSingle (16,384),
    so the CAP-16 tier (k_huff_encode_r16) takes it first, and the blocks with
    more than 16 distinct symbols it leaves go to the wave pass (at most
    kWaveEncodeLimit, 24,576, of them) or the lane-per-block CAP-64 pass."""
    import synth
    w, h = 2048, 1024  # 49,152 blocks
    fr = synth.noise_frame(w, h)
    pay = codec.compress(fr.tobytes(), w, h, q)
    assert pay == oracle.compress(fr.tobytes(), w, h, q)
    assert codec.decompress(pay, w, h, q) == oracle.decompress(pay, w, h, q)


def sparse_basis_frame(w, h, seed):
    """Every 8x8 block is 128 + a * basis(u, v) for a random (u, v) (zero for a
    quarter of the blocks): after quantisation mostly one or two nonzero
    coefficients per block, in random rows and columns, so K6's per-unit
    zero-row / zero-column skipping meets every pattern of live steps."""
    rng = np.random.default_rng(seed)
    n = np.arange(8)
    C = np.cos((2 * n[None, :] + 1) * n[:, None] * np.pi / 16)  # C[u][x]
    out = np.empty(w * h * 3 // 2, np.uint8)
    planes = [(0, w, h), (w * h, w // 2, h // 2), (w * h * 5 // 4, w // 2, h // 2)]
    for off, pw, ph in planes:
        nb = (pw // 8) * (ph // 8)
        u, v = rng.integers(0, 8, nb), rng.integers(0, 8, nb)
        amp = rng.choice([0.0, 20.0, 60.0, 110.0], nb) * rng.choice([-1.0, 1.0], nb)
        blk = 128 + amp[:, None, None] * C[u][:, :, None] * C[v][:, None, :]
        img = np.clip(np.rint(blk), 0, 255).astype(np.uint8)
        img = img.reshape(ph // 8, pw // 8, 8, 8).transpose(0, 2, 1, 3).reshape(ph, pw)
        out[off:off + pw * ph] = img.reshape(-1)
    return out.tobytes()


@pytest.mark.parametrize("q", [(50, 50, 50), (90, 90, 90), (5, 20, 100)])
def test_sparse_blocks_vs_oracle(codec, oracle, q):
    w, h = 1024, 512
    fr = sparse_basis_frame(w, h, sum(q))
    pay = oracle.compress(fr, w, h, q)
    assert codec.compress(fr, w, h, q) == pay
    assert codec.decompress(pay, w, h, q) == oracle.decompress(pay, w, h, q)


def flat_block_frame(w, h, seed, busy):
    """IYUV frame of flat 8x8 blocks (every value 0..255 occurs: DC-only blocks
    over the whole DC range), with a `busy` share of blocks, at random
    positions, carrying noise (blocks with AC coefficients between them)."""
    rng = np.random.default_rng(seed)
    out = []
    for pw, ph in ((w, h), (w // 2, h // 2), (w // 2, h // 2)):
        nb = (pw // 8) * (ph // 8)
        vals = np.resize(rng.permutation(256), nb).astype(np.float64)
        blk = np.repeat(vals[:, None], 64, 1)
        noisy = rng.random(nb) < busy
        blk[noisy] += rng.normal(0, 24, (int(noisy.sum()), 64))
        img = np.clip(np.rint(blk), 0, 255).astype(np.uint8)
        out.append(img.reshape(ph // 8, pw // 8, 8, 8).transpose(0, 2, 1, 3).reshape(-1))
    return np.concatenate(out).tobytes()


@pytest.mark.parametrize("q,busy", [((1, 1, 1), 0.0), ((50, 50, 50), 0.3), ((97, 97, 97), 0.1),
                                    ((100, 100, 100), 0.5), ((3, 60, 100), 0.02)])
def test_dc_blocks_vs_oracle(codec, oracle, q, busy):
    """The fused decoder's DC-only blocks (constant rows) and its compacted
    units of the other blocks, across the DC range and mixes of both."""
    w, h = 512, 256
    fr = flat_block_frame(w, h, int(busy * 100) + sum(q), busy)
    pay = oracle.compress(fr, w, h, q)
    assert codec.compress(fr, w, h, q) == pay
    assert codec.decompress(pay, w, h, q) == oracle.decompress(pay, w, h, q)


@pytest.mark.parametrize("wh", [(16, 16), (48, 16), (16, 48), (1008, 16), (144, 272)])
def test_odd_geometries(codec, oracle, wh):
    w, h = wh
    rng = np.random.default_rng(w * 1000 + h)
    fr = rng.integers(0, 256, w * h * 3 // 2).astype(np.uint8).tobytes()
    for q in (20, 80):
        pay = codec.compress(fr, w, h, (q, q, q))
        assert pay == oracle.compress(fr, w, h, (q, q, q))
        assert codec.decompress(pay, w, h, (q, q, q)) == oracle.decompress(pay, w, h, (q, q, q))


def test_fdct_blocks_vs_oracle(codec, oracle):
    rng = np.random.default_rng(3)
    px = rng.integers(0, 256, (4096, 64)).astype(np.uint8)
    px[:64] = 128
    px[64:128] = 0
    px[128:192] = 255
    for q, chroma in ((1, 0), (50, 0), (90, 1), (100, 0)):
        Q = oracle.qtable(q, chroma)
        got = codec.fdct_blocks(px, Q)
        zig = np.array([0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40,
                        48, 41, 34, 27, 20, 13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29,
                        22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54,
                        47, 55, 62, 63])
        for i in range(0, 4096, 97):
            ref = oracle.fdct_block(px[i], Q)
            assert np.array_equal(got[i], ref[zig]), (q, i)


def test_huff_encode_edge_blocks(codec, oracle):
    blocks = blockgen.edge_blocks()
    coefs = np.stack([b for _, b in blocks])
    chunks = codec.huff_encode_blocks(coefs)
    from oracle.oracle import huff_encode_block
    zz = np.array([0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48,
                   41, 34, 27, 20, 13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15,
                   23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63])
    for (name, b), got in zip(blocks, chunks):
        natural = np.zeros(64, np.int16)
        natural[zz] = b  # zig-zag order -> natural order for the oracle API
        assert got == huff_encode_block(natural), name


@pytest.mark.parametrize("gold", ["chef-with-trumpet-DCT-50.myyuv", "chef-with-trumpet-DCT-90.myyuv"])
def test_decode_errors_match_oracle(codec, oracle, golden, gold):
    """Every malformed stream (defined in the reference or not) fails on the
    GPU exactly as in the oracle, with the same first bad block."""
    import malformed
    import myyuv_hip
    g = golden(gold)
    w, h, q = g.width, g.height, tuple(g.params)
    for name, pay, kind in malformed.cases(g.data):
        try:
            oracle.decompress(pay, w, h, q)
            exp = 0
        except RuntimeError as e:
            exp = e.args[0]
        try:
            codec.decompress(pay, w, h, q)
            got = 0
        except myyuv_hip.CodecError as e:
            got = e.code
        assert got == exp, (name, got, exp)
        assert exp != 0, name


def test_argument_errors(codec):
    import myyuv_hip
    fr = bytes(64 * 64 * 3 // 2)
    with pytest.raises(myyuv_hip.CodecError) as e:
        codec.compress(fr, 64, 64, (0, 50, 50))
    assert e.value.code == myyuv_hip.E_QUALITY
    assert str(e.value) == "Level of quality must be between 1 and 100"
    with pytest.raises(myyuv_hip.CodecError) as e:
        codec.compress(bytes(72 * 64 * 3 // 2), 72, 64, (50, 50, 50))
    assert e.value.code == myyuv_hip.E_WIDTH
    with pytest.raises(myyuv_hip.CodecError) as e:
        codec.compress(bytes(64 * 40 * 3 // 2), 64, 40, (50, 50, 50))
    assert e.value.code == myyuv_hip.E_HEIGHT


def test_device_api_roundtrip(codec, golden):
    import torch
    import myyuv_hip
    raw = golden("chef-with-trumpet.myyuv")
    g = golden("chef-with-trumpet-DCT-50.myyuv")
    w, h = raw.width, raw.height
    cap = myyuv_hip.payload_bound(w, h)
    d_in = torch.frombuffer(bytearray(raw.data), dtype=torch.uint8).cuda()
    d_pay = torch.empty(cap, dtype=torch.uint8, device="cuda")
    d_size = torch.zeros(1, dtype=torch.int32, device="cuda")
    d_out = torch.empty(w * h * 3 // 2, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        codec.compress_device(d_in.data_ptr(), w, h, (50, 50, 50), d_pay.data_ptr(), cap,
                              d_size.data_ptr(), stream)
        codec.decompress_device(d_pay.data_ptr(), d_size.data_ptr(), cap, w, h, (50, 50, 50),
                                d_out.data_ptr(), stream)
    rc, bad = codec.sync_status(stream)
    assert rc == 0
    n = int(d_size.item())
    assert bytes(d_pay[:n].cpu().numpy()) == g.data
    assert bytes(d_out.cpu().numpy()) == codec.decompress(g.data, w, h, (50, 50, 50))


@pytest.mark.parametrize("wh", [(64, 64), (128, 48)])
def test_irregular_tables_match_oracle(codec, oracle, wh):
    """Valid streams whose Huffman tables the reference encoder never writes
    (lengths out of order, a length split over groups, > 32 codes of one
    length): K5 decodes them on its general path, bit-exact with the oracle."""
    import malformed
    import synth
    w, h = wh
    q = 100  # noise at q=100: chunks long enough for the crafted tables
    fr = synth.noise_frame(w, h).tobytes()
    pay = oracle.compress(fr, w, h, (q, q, q))
    for name, p in malformed.irregular_cases(pay):
        exp = oracle.decompress(p, w, h, (q, q, q))
        assert exp != oracle.decompress(pay, w, h, (q, q, q)), name
        assert codec.decompress(p, w, h, (q, q, q)) == exp, name


def _batch_frames(golden, w, h, n):
    """n distinct frames of one geometry: the chef-small frame, tiled shifts
    of it (SURVEY.md §8d generator) and a noise frame."""
    import synth
    raw = golden("chef-with-trumpet.myyuv").data
    frames = []
    for f in range(n):
        if f % 3 == 2:
            frames.append(synth.noise_frame(w, h, seed=77 + f).tobytes())
        else:
            ox, oy = synth.batch_origin(f, SMALL_W, SMALL_H)
            frames.append(bytes(synth.tiled_frame(raw, SMALL_W, SMALL_H, w, h, ox, oy)))
    return frames


@pytest.mark.parametrize("wh,n,q", [((992, 736), 3, (50, 50, 50)), ((144, 272), 5, (90, 40, 75)),
                                    ((1008, 16), 2, (1, 100, 50)), ((1024, 1024), 9, (90, 90, 90))])
def test_batch_device_matches_single_frames(codec, oracle, golden, wh, n, q):
    """One launch per kernel over n frames (blocks numbered across the batch,
    per-frame scans and output slots): every payload and every decoded frame
    equals the oracle's single-frame result.  The 9-frame 1024x1024 q90 batch
    (three noise frames) lists ~108k overflow blocks, past one resident round
    of the CAP-64 lane pass: the CAP-16 register tier takes them and ~86k
    blocks with more than 16 symbols go on to the lane pass, grid-stride."""
    import torch
    import myyuv_hip
    w, h = wh
    frames = _batch_frames(golden, w, h, n)
    fb = w * h * 3 // 2
    cap = (myyuv_hip.payload_bound(w, h) + 3) & ~3
    d_in = torch.frombuffer(bytearray(b"".join(frames)), dtype=torch.uint8).cuda()
    d_pay = torch.zeros(n * cap, dtype=torch.uint8, device="cuda")
    d_sizes = torch.zeros(n, dtype=torch.int32, device="cuda")
    d_out = torch.empty(n * fb, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    codec.reserve_batch(w, h, n)
    for _ in range(2):  # twice: nothing may depend on a fresh workspace
        codec.compress_batch_device(d_in.data_ptr(), n, w, h, q, d_pay.data_ptr(), cap,
                                    d_sizes.data_ptr(), stream)
        codec.decompress_batch_device(d_pay.data_ptr(), d_sizes.data_ptr(), cap, n, w, h, q,
                                      d_out.data_ptr(), stream)
        rc, bad = codec.sync_status(stream)
        assert rc == 0, (rc, bad)
        pay = d_pay.cpu().numpy()
        out = d_out.cpu().numpy()
        sizes = d_sizes.cpu().numpy()
        for f in range(n):
            exp = oracle.compress(frames[f], w, h, q)
            got = bytes(pay[f * cap: f * cap + int(sizes[f])])
            assert got == exp, f
            assert bytes(out[f * fb:(f + 1) * fb]) == oracle.decompress(exp, w, h, q), f


@pytest.mark.parametrize("n", [1, 2, 3])
def test_k2_windows_stay_inside_the_tiles(codec, oracle, chef_big, n):
    """Round 5's advice: with 4-tile K2 windows and a tile count of 1, 2 or 3
    mod 8 (chef-big: 1,113 tiles per frame), K2's grid once had a window past
    the last tile, which wrote tile-info words beyond the buffer.  A canary
    band after the batch's last tile must survive the compression, and the
    streams must stay the pinned / oracle bytes."""
    import torch
    import myyuv_hip
    f, raw = chef_big
    w, h, q = f.width, f.height, (50, 50, 50)
    nt = n * myyuv_hip.batch_tiles(w, h)
    assert nt % 8 == n  # the regime the advice names
    fb = w * h * 3 // 2
    cap = (myyuv_hip.payload_bound(w, h) + 3) & ~3
    d_in = torch.frombuffer(bytearray(raw * n), dtype=torch.uint8).cuda()
    d_pay = torch.zeros(n * cap, dtype=torch.uint8, device="cuda")
    d_sizes = torch.zeros(n, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    codec.reserve_batch(w, h, n)
    codec.tinfo_guard(nt, True)
    codec.compress_batch_device(d_in.data_ptr(), n, w, h, q, d_pay.data_ptr(), cap, d_sizes.data_ptr(), stream)
    rc, bad = codec.sync_status(stream)
    assert rc == 0, (rc, bad)
    assert codec.tinfo_guard(nt, False) == 0
    pay = d_pay.cpu().numpy()
    sizes = d_sizes.cpu().numpy()
    for i in range(n):
        got = bytes(pay[i * cap: i * cap + int(sizes[i])])
        assert sha(got) == "fe9b7317653c2b44a9f24436f0e349b083b4e368cf9653e8777e9f7a79cebfcc", i
    if n == 1:  # the host-buffer entry point too
        codec.tinfo_guard(nt, True)
        assert sha(codec.compress(raw, w, h, q)) == "fe9b7317653c2b44a9f24436f0e349b083b4e368cf9653e8777e9f7a79cebfcc"
        assert codec.tinfo_guard(nt, False) == 0


def test_batch_decode_error_reports_frame(codec, oracle, golden):
    """A malformed chunk in frame 1 of a batch: the reference's error, at the
    batch-global index of the failing block (frame 1 * blocks per frame + block)."""
    import torch
    import malformed
    import myyuv_hip
    g = golden("chef-with-trumpet-DCT-50.myyuv")
    w, h, q = g.width, g.height, tuple(g.params)
    nblk = (w // 8) * (h // 8) + 2 * (w // 16) * (h // 16)
    name, badpay = next((n, p) for n, p, kind in malformed.cases(g.data) if n == "bad_code")
    try:
        oracle.decompress(badpay, w, h, q)
        raise AssertionError("oracle accepted " + name)
    except RuntimeError as e:
        exp_code = e.args[0]
    single_bad = None
    try:
        codec.decompress(badpay, w, h, q)
    except myyuv_hip.CodecError as e:
        assert e.code == exp_code
        single_bad = e.bad_block
    assert single_bad is not None and single_bad >= 0
    cap = (max(len(g.data), len(badpay)) + 3) & ~3
    buf = bytearray(2 * cap)
    buf[:len(g.data)] = g.data
    buf[cap:cap + len(badpay)] = badpay
    d_pay = torch.frombuffer(buf, dtype=torch.uint8).cuda()
    d_sizes = torch.tensor([len(g.data), len(badpay)], dtype=torch.int32, device="cuda")
    d_out = torch.empty(2 * w * h * 3 // 2, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    codec.decompress_batch_device(d_pay.data_ptr(), d_sizes.data_ptr(), cap, 2, w, h, q,
                                  d_out.data_ptr(), stream)
    rc, bad = codec.sync_status(stream)
    assert rc == exp_code
    assert bad == nblk + single_bad


def test_batch_split_into_launches(oracle, golden):
    """A batch whose coefficient image would reach 4 GiB runs as several
    launches (kMaxLaunchBlocks; here forced down to two 256x128 frames per
    launch with MYYUV_LAUNCH_BLOCKS): 7 frames (launches of 2, 2, 2, 1) give
    every frame's single-frame bytes, and a decode error in frame 5 names its
    batch-global block, as one launch does."""
    import torch
    import malformed
    import myyuv_hip
    from conftest import _codec_with
    w, h, q, n = 256, 128, (70, 60, 50), 7
    nblk = (w // 8) * (h // 8) + 2 * (w // 16) * (h // 16)
    frames = _batch_frames(golden, w, h, n)
    c = _codec_with({"MYYUV_LAUNCH_BLOCKS": str(2 * nblk + 5)})
    try:
        fb = w * h * 3 // 2
        cap = (myyuv_hip.payload_bound(w, h) + 3) & ~3
        d_in = torch.frombuffer(bytearray(b"".join(frames)), dtype=torch.uint8).cuda()
        d_pay = torch.zeros(n * cap, dtype=torch.uint8, device="cuda")
        d_sizes = torch.zeros(n, dtype=torch.int32, device="cuda")
        d_out = torch.empty(n * fb, dtype=torch.uint8, device="cuda")
        stream = torch.cuda.current_stream().cuda_stream
        c.compress_batch_device(d_in.data_ptr(), n, w, h, q, d_pay.data_ptr(), cap, d_sizes.data_ptr(), stream)
        c.decompress_batch_device(d_pay.data_ptr(), d_sizes.data_ptr(), cap, n, w, h, q, d_out.data_ptr(), stream)
        rc, bad = c.sync_status(stream)
        assert rc == 0, (rc, bad)
        pay, out, sizes = d_pay.cpu().numpy(), d_out.cpu().numpy(), d_sizes.cpu().numpy()
        pays = []
        for f in range(n):
            exp = oracle.compress(frames[f], w, h, q)
            pays.append(exp)
            assert bytes(pay[f * cap: f * cap + int(sizes[f])]) == exp, f
            assert bytes(out[f * fb:(f + 1) * fb]) == oracle.decompress(exp, w, h, q), f
        # a malformed stream as frame 5 (the third launch)
        _, badpay = next((nm, p) for nm, p, kind in malformed.cases(pays[5]) if nm == "bad_code")
        with pytest.raises(myyuv_hip.CodecError) as single:
            c.decompress(badpay, w, h, q)
        assert single.value.bad_block >= 0
        cap2 = (max(len(p) for p in pays + [badpay]) + 3) & ~3
        buf = bytearray(n * cap2)
        lens = []
        for f in range(n):
            p = badpay if f == 5 else pays[f]
            buf[f * cap2: f * cap2 + len(p)] = p
            lens.append(len(p))
        d_pay2 = torch.frombuffer(buf, dtype=torch.uint8).cuda()
        d_sz2 = torch.tensor(lens, dtype=torch.int32, device="cuda")
        c.decompress_batch_device(d_pay2.data_ptr(), d_sz2.data_ptr(), cap2, n, w, h, q, d_out.data_ptr(), stream)
        rc, bad = c.sync_status(stream)
        assert rc == single.value.code
        assert bad == 5 * nblk + single.value.bad_block
    finally:
        c.close()


@pytest.mark.parametrize("cap", [8, 64, 4096, 100000])
def test_device_compress_capacity_is_respected(codec, golden, oracle, cap):
    """compress_device into a slot smaller than the payload: MYYUV_E_CAPACITY,
    the true size is still reported, and no byte past `cap` is written
    (canary after the slot); the tile writers skip what does not fit."""
    import torch
    import myyuv_hip
    raw = golden("chef-with-trumpet.myyuv")
    w, h, q = raw.width, raw.height, (50, 50, 50)
    want = oracle.compress(raw.data, w, h, q)
    assert cap < len(want)
    dev = torch.device("cuda", 0)
    d_in = torch.frombuffer(bytearray(raw.data), dtype=torch.uint8).to(dev)
    d_pay = torch.full((cap + 4096,), 0xA5, dtype=torch.uint8, device=dev)
    d_size = torch.zeros(1, dtype=torch.int32, device=dev)
    st = torch.cuda.Stream(dev)
    st.wait_stream(torch.cuda.current_stream(dev))
    codec.compress_device(d_in.data_ptr(), w, h, q, d_pay.data_ptr(), cap, d_size.data_ptr(), st.cuda_stream)
    rc, _ = codec.sync_status(st.cuda_stream)
    assert rc == myyuv_hip.E_CAPACITY
    assert int(d_size.item()) == len(want)
    tail = d_pay[cap:].cpu()
    assert bool((tail == 0xA5).all())


def sweep_frame(w, h, rng, sigma=None):
    """A smooth random gradient plus Gaussian noise of a random strength (0 to
    48), optionally quantised to a few levels: from DC-only blocks through
    every K2 class to noise whose blocks nearly all overflow (a 1024x1024
    frame of it passes the CAP-16 tier's single-frame gate)."""
    out = []
    sigma = float(rng.choice([0.0, 2.0, 6.0, 16.0, 48.0])) if sigma is None else sigma
    levels = int(rng.choice([0, 0, 4, 16]))
    for pw, ph in ((w, h), (w // 2, h // 2), (w // 2, h // 2)):
        y, x = np.mgrid[0:ph, 0:pw]
        a, b, c = rng.uniform(-1.5, 1.5, 3)
        img = 128 + a * (x - pw / 2) * 64 / max(pw, 1) + b * (y - ph / 2) * 64 / max(ph, 1) \
            + c * 40 * np.sin(x / 7.0 + y / 11.0) + rng.normal(0, sigma, (ph, pw))
        if levels:
            img = np.round(img / (256 / levels)) * (256 / levels)
        out.append(np.clip(np.rint(img), 0, 255).astype(np.uint8).reshape(-1))
    return np.concatenate(out).tobytes()


@pytest.mark.parametrize("seed", range(12))
def test_random_sweep_vs_oracle(codec, oracle, seed):
    """Seeded random geometries (multiples of 16 up to 1024), per-plane
    qualities (1..100) and content (sweep_frame): stream and decode equal the
    oracle's."""
    rng = np.random.default_rng(1000 + seed)
    w, h = (int(v) * 16 for v in rng.integers(1, 65, 2))
    q = tuple(int(v) for v in rng.integers(1, 101, 3))
    sigma = None
    if seed % 4 == 0:  # strong noise over 1024x1024: a single-frame overflow list past the tier's gate
        w, h, sigma = 1024, 1024, 48.0
        q = tuple(max(v, 40) for v in q)
    fr = sweep_frame(w, h, rng, sigma)
    pay = oracle.compress(fr, w, h, q)
    assert codec.compress(fr, w, h, q) == pay, (w, h, q)
    assert codec.decompress(pay, w, h, q) == oracle.decompress(pay, w, h, q), (w, h, q)
