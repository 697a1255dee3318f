"""The C-ABI library (the drop-in boundary) loads and exports every entry point
include/myyuv_hip.h declares; host-side logic that needs no GPU."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import PKG, ROOT

HEADER = os.path.join(ROOT, "include", "myyuv_hip.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\*?\s+\*?(myyuv_[a-z_0-9]+)\s*\(", src, re.M)))


def test_header_declares_the_abi():
    names = declared_functions()
    assert "myyuv_gpu_dct_compress" in names and "myyuv_gpu_dct_decompress" in names
    assert len(names) >= 14


def test_library_exports_every_declared_symbol():
    import myyuv_hip
    lib = ctypes.CDLL(myyuv_hip.LIB_PATH)
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert sorted(myyuv_hip.EXPORTS) == sorted(declared_functions())


def test_exported_symbols_are_plain_c():
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(PKG, "libmyyuv_hip.so")],
                         capture_output=True, text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    for name in declared_functions():
        assert name in exported, name  # unmangled: extern "C"


def test_kernel_ids_match_the_header():
    """myyuv_hip.KERNELS / K_* (profile and skip masks) follow MYYUV_K_* of the header."""
    import myyuv_hip
    ids = {m.group(1): int(m.group(2)) for m in
           re.finditer(r"^#define MYYUV_K_([A-Z0-9_]+)\s+(\d+)", open(HEADER).read(), re.M)}
    assert ids.pop("COUNT") == len(myyuv_hip.KERNELS)
    for name, kid in ids.items():
        assert getattr(myyuv_hip, "K_" + name) == kid, name


def test_error_strings_are_the_reference_messages():
    import myyuv_hip
    assert myyuv_hip.strerror(2) == "Level of quality must be between 1 and 100"
    assert myyuv_hip.strerror(3) == "Error. width % 8 must be 0"
    assert myyuv_hip.strerror(4) == "Error. height % 8 must be 0"
    assert myyuv_hip.strerror(6) == "DCTYUV load bad size"
    assert myyuv_hip.strerror(7) == "DCTYUVPlane load bad size"
    assert myyuv_hip.strerror(8) == "DCTYUVPlane load chunks_sizes_size bad size"
    assert myyuv_hip.strerror(9) == "DCTYUVPlane load content_size bad size"
    assert myyuv_hip.strerror(10) == "Huffman bad code"
    assert myyuv_hip.strerror(11) == "Huffman unknown symbol"


def test_payload_bound_covers_worst_case(oracle):
    import myyuv_hip
    for w, h in ((16, 16), (992, 736), (4032, 3008), (8192, 8192)):
        assert myyuv_hip.payload_bound(w, h) >= oracle.lib().oracle_payload_bound(w, h)
        assert myyuv_hip.payload_bound(w, h) % 4 == 0


def test_no_cpu_fallback_without_gpu():
    """On a machine without a GPU the product path fails loudly (no silent CPU
    fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    import myyuv_hip
    with pytest.raises(myyuv_hip.CodecError) as e:
        myyuv_hip.Codec(0)
    assert e.value.code == myyuv_hip.E_NO_DEVICE


def test_host_library_and_cli_are_built():
    for f in ("libmyyuv_hip.so", "libmyyuv_amd.so", "myyuv_cli"):
        assert os.path.exists(os.path.join(PKG, f)), f
    out = subprocess.run(["nm", "-DC", "--defined-only", os.path.join(PKG, "libmyyuv_amd.so")],
                         capture_output=True, text=True, check=True).stdout
    for sym in ("myyuvDCT::compress_DCT_planar", "myyuvDCT::decompress_DCT_planar",
                "myyuv::YUV::compress_map", "myyuv::YUV::decompress_map", "myyuv::YUV::load",
                "myyuv::YUV::dump"):
        assert sym in out, sym


def test_into_calls_check_their_buffers():
    """compress_into / decompress_into hand the caller's arrays to the C ABI
    as raw pointers: short, strided, non-uint8 or read-only buffers are refused
    before any call (no GPU needed: the checks precede it)."""
    import numpy as np
    import myyuv_hip
    c = myyuv_hip.Codec.__new__(myyuv_hip.Codec)
    c._h = None
    w, h = 16, 16
    fb = w * h * 3 // 2
    good = np.zeros(fb, np.uint8)
    out = np.zeros(4096, np.uint8)
    bad_inputs = [np.zeros(fb - 1, np.uint8),                 # short frame
                  np.zeros(2 * fb, np.uint8)[::2],           # strided
                  np.zeros(fb, np.int16),                    # not uint8
                  bytes(fb)]                                 # not an ndarray
    for a in bad_inputs:
        with pytest.raises(ValueError):
            c.compress_into(a, w, h, (50, 50, 50), out)
    ro = np.zeros(4096, np.uint8)
    ro.flags.writeable = False
    for o in (np.zeros(8192, np.uint8)[::2], np.zeros(4096, np.uint16), ro):
        with pytest.raises(ValueError):
            c.compress_into(good, w, h, (50, 50, 50), o)
    with pytest.raises(ValueError):
        c.decompress_into(np.zeros(64, np.uint8), w, h, (50, 50, 50), np.zeros(fb - 1, np.uint8))
    with pytest.raises(ValueError):
        c.decompress_into(np.zeros(128, np.uint8)[::2], w, h, (50, 50, 50), np.zeros(fb, np.uint8))
