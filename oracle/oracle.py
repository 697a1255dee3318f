"""ctypes wrapper for the CPU restatement (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product path.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
        L = ctypes.CDLL(path)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.oracle_compress.argtypes = [u8p, ctypes.c_uint32, ctypes.c_uint32, u8p, u8p,
                                      ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
        L.oracle_decompress.argtypes = [u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                        u8p, u8p]
        L.oracle_payload_bound.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        L.oracle_payload_bound.restype = ctypes.c_uint32
        L.oracle_qtable.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
        L.oracle_fdct_block.argtypes = [u8p, ctypes.POINTER(ctypes.c_float),
                                        ctypes.POINTER(ctypes.c_int16)]
        L.oracle_idct_block.argtypes = [ctypes.POINTER(ctypes.c_int16),
                                        ctypes.POINTER(ctypes.c_float), u8p]
        L.oracle_huff_encode_block.argtypes = [ctypes.POINTER(ctypes.c_int16), u8p]
        L.oracle_huff_decode_block.argtypes = [u8p, ctypes.c_int, ctypes.POINTER(ctypes.c_int16)]
        L.oracle_set_num_threads.argtypes = [ctypes.c_int]
        _LIB = L
    return _LIB


def _p(a, t=ctypes.c_uint8):
    return a.ctypes.data_as(ctypes.POINTER(t))


def compress(iyuv, w, h, q):
    """IYUV bytes -> DCTYUV payload bytes (App. A). Raises RuntimeError(code)."""
    src = np.ascontiguousarray(np.frombuffer(bytes(iyuv), np.uint8) if not isinstance(iyuv, np.ndarray) else iyuv, np.uint8)
    qa = np.array(q, np.uint8)
    cap = lib().oracle_payload_bound(w, h)
    out = np.empty(cap, np.uint8)
    size = ctypes.c_uint32(0)
    rc = lib().oracle_compress(_p(src), w, h, _p(qa), _p(out), cap, ctypes.byref(size))
    if rc:
        raise RuntimeError(rc)
    return out[: size.value].tobytes()


def decompress(payload, w, h, q):
    src = np.frombuffer(bytes(payload), np.uint8)
    qa = np.array(q, np.uint8)
    out = np.zeros(w * h * 3 // 2, np.uint8)
    rc = lib().oracle_decompress(_p(src), len(src), w, h, _p(qa), _p(out))
    if rc:
        raise RuntimeError(rc)
    return out.tobytes()


def qtable(q, chroma):
    out = np.empty(64, np.float32)
    lib().oracle_qtable(int(q), int(chroma), _p(out, ctypes.c_float))
    return out


def fdct_block(px, Q):
    px = np.ascontiguousarray(px, np.uint8).reshape(64)
    out = np.empty(64, np.int16)
    lib().oracle_fdct_block(_p(px), _p(np.ascontiguousarray(Q, np.float32), ctypes.c_float),
                            _p(out, ctypes.c_int16))
    return out


def idct_block(coef, Q):
    coef = np.ascontiguousarray(coef, np.int16).reshape(64)
    out = np.empty(64, np.uint8)
    lib().oracle_idct_block(_p(coef, ctypes.c_int16),
                            _p(np.ascontiguousarray(Q, np.float32), ctypes.c_float), _p(out))
    return out


def huff_encode_block(coef):
    coef = np.ascontiguousarray(coef, np.int16).reshape(64)
    out = np.zeros(160, np.uint8)
    n = lib().oracle_huff_encode_block(_p(coef, ctypes.c_int16), _p(out))
    return out[:n].tobytes()


def huff_decode_block(chunk):
    src = np.frombuffer(bytes(chunk), np.uint8).copy()
    out = np.empty(64, np.int16)
    rc = lib().oracle_huff_decode_block(_p(src), len(src), _p(out, ctypes.c_int16))
    if rc:
        raise RuntimeError(rc)
    return out


def set_num_threads(n):
    lib().oracle_set_num_threads(int(n))


def num_threads():
    return lib().oracle_num_threads()


def bmp_to_iyuv(bmp_data, width, height, bit_count):
    """BMP::data (as stored) -> IYUV bytes (myyuv_yuv.cpp:88-128 over
    myyuv_bmp.cpp:77-101).  Raises RuntimeError(code) as the C ABI does."""
    src = np.frombuffer(bytes(bmp_data), np.uint8).copy()
    W, H = abs(width), abs(height)
    out = np.zeros(max(1, W * H * 3 // 2), np.uint8)
    L = lib()
    L.oracle_bmp_to_iyuv.argtypes = [ctypes.POINTER(ctypes.c_uint8), ctypes.c_int32, ctypes.c_int32,
                                     ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint8)]
    rc = L.oracle_bmp_to_iyuv(_p(src), int(width), int(height), int(bit_count), _p(out))
    if rc:
        raise RuntimeError(rc)
    return out[: W * H * 3 // 2].tobytes()
