"""BMP -> IYUV: YUV(const BMP&, IYUV), i.e.
bmp_to_yuv_map[IYUV] (myyuv_yuv.cpp:88-128) over BMP::colorData
(myyuv_bmp.cpp:77-101).

Pins: the reference's own image pair — chef-with-trumpet.bmp (gzipped copy in
tests/golden) converts to the pixel data of chef-with-trumpet.myyuv — and, in
this container, the reference library itself (oracle/_ref, ref_harness.cpp's
ref_bmp_to_iyuv over myyuv::BMP(path)) on synthetic images covering the three
orientations of colorData, 24 and 32 bpp, and noise (saturated colours make
the reference's uint8 chroma sum wrap; so must ours).  The GPU tests
compare K7 (csrc/k_color.hip) with the oracle byte for byte.
"""
import gzip
import os
import tempfile

import numpy as np
import pytest

from conftest import GOLDEN

ORIENTS = [(1, -1), (-1, 1), (1, 1)]  # colorData's three sign cases


def chef_bmp():
    import myyuv_file

    with gzip.open(os.path.join(GOLDEN, "chef-with-trumpet.bmp.gz"), "rb") as f:
        return myyuv_file.BMPFile.load(f.read())


def synth(w, h, bits, seed):
    import myyuv_file

    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, abs(w) * abs(h) * bits // 8, dtype=np.uint8).tobytes()
    return myyuv_file.BMPFile(w, h, bits, data)


def synth_cases():
    out = []
    for i, (sw, sh) in enumerate(ORIENTS):
        for bits in (24, 32):
            for (w, h) in ((64, 48), (4, 2), (992, 6)):
                out.append((sw * w, sh * h, bits, 100 * i + bits + w))
    return out


@pytest.fixture(scope="module")
def ref():
    from oracle import ref as R

    if not R.available("serial"):
        pytest.skip("oracle/_ref not built (needs /root/reference; `make -C oracle ref`)")
    return R


# ---------------------------------------------------------------- CPU: oracle
def test_golden_pair_header():
    b = chef_bmp()
    assert (b.width, b.height, b.bit_count) == (992, 736, 32)
    assert b.is_valid_header() and len(b.data) == 992 * 736 * 4


def test_oracle_matches_golden_iyuv(oracle, golden):
    b = chef_bmp()
    want = golden("chef-with-trumpet.myyuv")
    assert (want.width, want.height) == (992, 736)
    assert oracle.bmp_to_iyuv(b.data, b.width, b.height, b.bit_count) == want.data


@pytest.mark.parametrize("w,h,bits,seed", synth_cases())
def test_oracle_vs_reference_synthetic(oracle, ref, w, h, bits, seed):
    b = synth(w, h, bits, seed)
    with tempfile.NamedTemporaryFile(suffix=".bmp", delete=False) as f:
        f.write(b.dumps())
    try:
        rw, rh, want = ref.bmp_to_iyuv(f.name)
    finally:
        os.unlink(f.name)
    assert (rw, rh) == (abs(w), abs(h))
    assert oracle.bmp_to_iyuv(b.data, w, h, bits) == want


def test_oracle_vs_reference_golden_file(oracle, ref):
    b = chef_bmp()
    with tempfile.NamedTemporaryFile(suffix=".bmp", delete=False) as f:
        f.write(gzip.open(os.path.join(GOLDEN, "chef-with-trumpet.bmp.gz")).read())
    try:
        _, _, want = ref.bmp_to_iyuv(f.name)
    finally:
        os.unlink(f.name)
    assert oracle.bmp_to_iyuv(b.data, b.width, b.height, b.bit_count) == want


def test_chroma_sum_wraps(oracle):
    """Known answers worked by hand: a pure-blue quad has Cb 255 per pixel,
    divide_roundnearest(255, 4) = 64, and the uint8 sum of four 64s is 0 —
    the reference's IYUV Cb for saturated blue is 0, not 255.  Pure red:
    Cr 255 -> 0 likewise; Y = (uint8)(0.114f*255) = 29 and (0.299f*255) = 76."""
    blue = oracle.bmp_to_iyuv(bytes([255, 0, 0, 0] * 8), 4, -2, 32)
    red = oracle.bmp_to_iyuv(bytes([0, 0, 255, 0] * 8), 4, -2, 32)
    assert list(blue) == [29] * 8 + [0, 0] + [108, 108]
    assert list(red) == [76] * 8 + [84, 84] + [0, 0]


@pytest.mark.parametrize("w,h,bits,code", [
    (6, -2, 32, 15),   # width % 4 (isValidHeader) -> "BMP is invalid"
    (4, -2, 0, 15),
    (-4, -2, 32, 16),  # both negative -> "Unaccounted width and height sign"
    (0, 2, 32, 16),
    (4, 0, 32, 16),
    (4, -3, 32, 17),   # odd height (reference: assert)
    (4, -2, 16, 17),   # 16 bpp (reference: assert bit_count == 32)
])
def test_oracle_errors(oracle, w, h, bits, code):
    data = bytes(abs(w) * abs(h) * max(bits, 8) // 8)
    with pytest.raises(RuntimeError) as e:
        oracle.bmp_to_iyuv(data, w, h, bits)
    assert e.value.args[0] == code


def test_error_strings():
    import myyuv_hip

    assert myyuv_hip.strerror(15) == "BMP is invalid"
    assert myyuv_hip.strerror(16) == "Unaccounted width and height sign"


# ---------------------------------------------------------------- GPU: K7
@pytest.mark.gpu
def test_gpu_golden(codec, golden):
    b = chef_bmp()
    assert codec.bmp_to_iyuv(b.data, b.width, b.height, b.bit_count) == golden("chef-with-trumpet.myyuv").data


@pytest.mark.gpu
def test_gpu_chroma_sum_wraps(codec):
    assert list(codec.bmp_to_iyuv(bytes([255, 0, 0, 0] * 8), 4, -2, 32)) == [29] * 8 + [0, 0, 108, 108]


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,bits,seed", synth_cases())
def test_gpu_vs_oracle_synthetic(codec, oracle, w, h, bits, seed):
    b = synth(w, h, bits, seed)
    assert codec.bmp_to_iyuv(b.data, w, h, bits) == oracle.bmp_to_iyuv(b.data, w, h, bits)


@pytest.mark.gpu
@pytest.mark.parametrize("sw,sh", ORIENTS)
def test_gpu_vs_oracle_4k(codec, oracle, sw, sh):
    b = synth(sw * 4032, sh * 3008, 32, 7)
    assert codec.bmp_to_iyuv(b.data, b.width, b.height, 32) == oracle.bmp_to_iyuv(b.data, b.width, b.height, 32)


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,bits,code", [(6, -2, 32, 15), (-4, -2, 32, 16), (4, -3, 32, 17), (4, -2, 16, 17)])
def test_gpu_errors(codec, w, h, bits, code):
    import myyuv_hip

    with pytest.raises(myyuv_hip.CodecError) as e:
        codec.bmp_to_iyuv(bytes(abs(w) * abs(h) * 4), w, h, bits)
    assert e.value.code == code


@pytest.mark.gpu
def test_gpu_device_then_compress(codec, golden):
    """HBM-resident chain: BMP pixels -> K7 -> IYUV -> DCT q50 compress; the
    stream equals the reference's chef-with-trumpet-DCT-50 payload."""
    import torch
    import myyuv_hip

    b = chef_bmp()
    dev = torch.device("cuda", 0)
    d_bmp = torch.frombuffer(bytearray(b.data), dtype=torch.uint8).to(dev)
    n = 992 * 736 * 3 // 2
    d_iyuv = torch.empty(n, dtype=torch.uint8, device=dev)
    codec.bmp_to_iyuv_device(d_bmp.data_ptr(), b.width, b.height, 32, d_iyuv.data_ptr(),
                             torch.cuda.current_stream(dev).cuda_stream)
    cap = myyuv_hip.payload_bound(992, 736)
    d_pay = torch.empty(cap, dtype=torch.uint8, device=dev)
    d_sz = torch.zeros(1, dtype=torch.int32, device=dev)
    codec.compress_device(d_iyuv.data_ptr(), 992, 736, (50, 50, 50), d_pay.data_ptr(), cap, d_sz.data_ptr(),
                          torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    want = golden("chef-with-trumpet-DCT-50.myyuv")
    assert bytes(d_iyuv.cpu().numpy()) == golden("chef-with-trumpet.myyuv").data
    assert bytes(d_pay[: int(d_sz.item())].cpu().numpy()) == want.data
