"""The fused single-pass encoder k_encode_tile (MYYUV_ENCODER=fused; SURVEY.md
§8f row 4: K1's transform into an LDS coefficient image, then K2 over it, per
256-block tile).  Not the product (slower than K1 -> K2 through
HBM), so it runs here rather than in every `codec` test: the reference's
golden files, the pinned 4032x3008 stream, the quality edge cases, noise, the
overflow tiers and batches, all bit-exact against the oracle."""
import hashlib

import pytest

import blockgen

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("q,gold", [(50, "chef-with-trumpet-DCT-50.myyuv"),
                                    (90, "chef-with-trumpet-DCT-90.myyuv")])
def test_fused_golden_small(fused_encoder, golden, q, gold):
    raw = golden("chef-with-trumpet.myyuv")
    assert fused_encoder.compress(raw.data, raw.width, raw.height, (q, q, q)) == golden(gold).data


def test_fused_big_pinned(fused_encoder, chef_big):
    f, raw = chef_big
    pay = fused_encoder.compress(raw, f.width, f.height, (50, 50, 50))
    assert hashlib.sha256(pay).hexdigest() == "fe9b7317653c2b44a9f24436f0e349b083b4e368cf9653e8777e9f7a79cebfcc"


@pytest.mark.parametrize("q", [1, 25, 50, 51, 90, 100])
def test_fused_edge_frame(fused_encoder, oracle, q):
    w, h = 256, 128
    fr = blockgen.edge_frame(w, h).tobytes()
    assert fused_encoder.compress(fr, w, h, (q, q, q)) == oracle.compress(fr, w, h, (q, q, q))


@pytest.mark.parametrize("q", [(50, 50, 50), (90, 90, 90), (10, 60, 95)])
def test_fused_noise(fused_encoder, oracle, q):
    import synth
    w, h = 512, 256
    fr = bytes(synth.noise_frame(w, h))
    assert fused_encoder.compress(fr, w, h, q) == oracle.compress(fr, w, h, q)


def test_fused_host_batch(fused_encoder, oracle, golden):
    """A batch of 9 frames through the pipelined host batch (chunks of 1):
    every stream equals the oracle's."""
    import synth
    raw = golden("chef-with-trumpet.myyuv").data
    w, h, q = 256, 128, (75, 75, 75)
    frames = [bytes(synth.tiled_frame(raw, 992, 736, w, h, *synth.batch_origin(f, 992, 736))) for f in range(9)]
    assert fused_encoder.compress_batch(frames, w, h, q) == [oracle.compress(f, w, h, q) for f in frames]
