"""The pipelined host-buffer batches:
myyuv_gpu_dct_{compress,decompress}_{frames,batch} cut a batch into chunks
that upload, run and download at once on three streams.  Every frame's bytes
must equal the single-frame call's (and the oracle's / the pinned files'),
whatever the chunking; errors must name the batch-global failing block."""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

BIG_Q50_SHA = "fe9b7317653c2b44a9f24436f0e349b083b4e368cf9653e8777e9f7a79cebfcc"


def _frames(golden, n, w=256, h=128):
    """n distinct frames: the small golden frame tiled at per-frame origins,
    every fourth one noise."""
    import synth
    raw = golden("chef-with-trumpet.myyuv").data
    out = []
    for f in range(n):
        if f % 4 == 3:
            out.append(bytes(synth.noise_frame(w, h, seed=100 + f)))
        else:
            ox, oy = synth.batch_origin(f, 992, 736)
            out.append(bytes(synth.tiled_frame(raw, 992, 736, w, h, ox, oy)))
    return out


@pytest.mark.parametrize("n", [1, 2, 9, 20, 70])
def test_host_batch_roundtrip_matches_oracle(codec, oracle, golden, n):
    """n = 1 .. 70: one chunk, two chunks of one frame, and chunks of 1, 2
    and 8 frames over both slots many times (pipe_chunk: n / 8, 1 .. 8)."""
    w, h, q = 256, 128, (60, 50, 90)
    frames = _frames(golden, n)
    want = [oracle.compress(f, w, h, q) for f in frames]
    assert codec.compress_batch(frames, w, h, q) == want
    assert codec.compress_frames(frames, w, h, q) == want
    dec = [oracle.decompress(p, w, h, q) for p in want]
    assert codec.decompress_batch(want, w, h, q) == dec
    assert codec.decompress_frames(want, w, h, q) == dec


def test_host_batch_big_frames(codec, chef_big):
    """Three 4032x3008 frames: the golden DCT-50 stream decodes to the pinned
    frame, which compresses to the pinned q50 stream, which decodes as the
    single-frame call does (hashes: a byte diff of 18 MB is slow)."""
    f, raw = chef_big
    w, h, q = f.width, f.height, (50, 50, 50)
    sha = lambda b: hashlib.sha256(b).hexdigest()  # noqa: E731
    assert [sha(o) for o in codec.decompress_batch([f.data] * 3, w, h, q)] == [sha(raw)] * 3
    pays = codec.compress_frames([raw] * 3, w, h, q)
    assert [sha(p) for p in pays] == [BIG_Q50_SHA] * 3
    want = sha(codec.decompress(pays[0], w, h, q))
    assert [sha(o) for o in codec.decompress_frames(pays, w, h, q)] == [want] * 3


def test_host_batch_decode_error_names_the_block(codec, oracle, golden):
    """A malformed stream as frame 13 of 20 (chunks of 2 frames: the error is
    found in the seventh chunk, slot 0): the oracle's error code, at
    13 * blocks per frame + the single-frame call's block index."""
    import malformed
    import myyuv_hip
    g = golden("chef-with-trumpet-DCT-50.myyuv")
    w, h, q = g.width, g.height, tuple(g.params)
    nblk = (w // 8) * (h // 8) + 2 * (w // 16) * (h // 16)
    _, badpay = next((nm, p) for nm, p, kind in malformed.cases(g.data) if nm == "bad_code")
    with pytest.raises(myyuv_hip.CodecError) as single:
        codec.decompress(badpay, w, h, q)
    with pytest.raises(RuntimeError) as ref:
        oracle.decompress(badpay, w, h, q)
    assert single.value.code == ref.value.args[0] and single.value.bad_block >= 0
    pays = [g.data] * 20
    pays[13] = badpay
    for call in (codec.decompress_batch, codec.decompress_frames):
        with pytest.raises(myyuv_hip.CodecError) as e:
            call(pays, w, h, q)
        assert e.value.code == single.value.code
        assert e.value.bad_block == 13 * nblk + single.value.bad_block
    # the context still works after the failed batch
    assert codec.decompress_batch([g.data] * 3, w, h, q) == [oracle.decompress(g.data, w, h, q)] * 3


def test_host_batch_header_error_comes_first(codec, golden):
    """A stream whose DCTYUV header is short fails the whole call with the
    reference's DCTYUV::load message before any frame is decoded."""
    import myyuv_hip
    g = golden("chef-with-trumpet-DCT-50.myyuv")
    with pytest.raises(myyuv_hip.CodecError) as e:
        codec.decompress_batch([g.data, g.data[:10]], g.width, g.height, tuple(g.params))
    assert e.value.code == myyuv_hip.E_DCTYUV_SIZE


def test_host_batch_capacity(codec, golden):
    """compress_batch into slots smaller than a payload: MYYUV_E_CAPACITY."""
    import ctypes
    import myyuv_hip
    raw = golden("chef-with-trumpet.myyuv").data
    n = 3
    src = np.frombuffer(raw * n, np.uint8)
    cap = 1000
    out = np.zeros(n * cap, np.uint8)
    sizes = (ctypes.c_uint32 * n)()
    q = np.array([50, 50, 50], np.uint8)
    rc = myyuv_hip.load().myyuv_gpu_dct_compress_batch(codec._h, myyuv_hip._u8(src), n, 992, 736,
                                                       myyuv_hip._u8(q), myyuv_hip._u8(out), cap, sizes)
    assert rc == myyuv_hip.E_CAPACITY
    assert sizes[0] == len(golden("chef-with-trumpet-DCT-50.myyuv").data)
    assert not out.any()  # nothing was written into a slot too small for it
