"""ctypes wrapper for oracle/_ref/libmyyuv_ref_{serial,omp}.so — the reference
library compiled from its own sources (oracle/Makefile `ref`) plus
oracle/ref_harness.cpp.

TEST INFRASTRUCTURE ONLY (checker + cpu_baseline "reference" leg).
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIBS = {}


def path(variant="omp"):
    return os.path.join(_HERE, "_ref", f"libmyyuv_ref_{variant}.so")


def available(variant="omp"):
    return os.path.exists(path(variant))


def lib(variant="omp"):
    if variant not in _LIBS:
        L = ctypes.CDLL(path(variant))
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.ref_compress.argtypes = [u8p, ctypes.c_uint32, ctypes.c_uint32, u8p, u8p, ctypes.c_uint32,
                                   ctypes.POINTER(ctypes.c_uint32)]
        L.ref_decompress.argtypes = [u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, u8p, u8p]
        L.ref_bench.argtypes = [u8p, ctypes.c_uint32, ctypes.c_uint32, u8p, ctypes.c_int,
                                ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
        L.ref_last_error.restype = ctypes.c_char_p
        _LIBS[variant] = L
    return _LIBS[variant]


def _p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


class RefError(RuntimeError):
    pass


def compress(iyuv, w, h, q, variant="omp"):
    src = np.frombuffer(bytes(iyuv), np.uint8).copy()
    qa = np.array(q, np.uint8)
    cap = 12 + 24 + (w * h * 3 // 2) // 64 * 161
    out = np.empty(cap, np.uint8)
    size = ctypes.c_uint32(0)
    L = lib(variant)
    rc = L.ref_compress(_p(src), w, h, _p(qa), _p(out), cap, ctypes.byref(size))
    if rc == 1:
        raise RefError(L.ref_last_error().decode())
    if rc:
        raise RuntimeError(f"ref_compress rc={rc}")
    return out[: size.value].tobytes()


def decompress(payload, w, h, q, variant="omp"):
    src = np.frombuffer(bytes(payload), np.uint8).copy()
    qa = np.array(q, np.uint8)
    out = np.zeros(w * h * 3 // 2, np.uint8)
    L = lib(variant)
    rc = L.ref_decompress(_p(src), len(src), w, h, _p(qa), _p(out))
    if rc == 1:
        raise RefError(L.ref_last_error().decode())
    return out.tobytes()


def bench(iyuv, w, h, q, iters, variant="omp"):
    """Median (compress_ms, decompress_ms) over `iters` in-process calls."""
    src = np.frombuffer(bytes(iyuv), np.uint8).copy()
    qa = np.array(q, np.uint8)
    tc, td = ctypes.c_double(0), ctypes.c_double(0)
    L = lib(variant)
    rc = L.ref_bench(_p(src), w, h, _p(qa), int(iters), ctypes.byref(tc), ctypes.byref(td))
    if rc:
        raise RefError(L.ref_last_error().decode())
    return tc.value, td.value


def bmp_to_iyuv(path, variant="serial"):
    """myyuv::BMP(path) -> YUV(bmp, IYUV) of the reference (ref_harness.cpp);
    returns (width, height, iyuv bytes)."""
    L = lib(variant)
    L.ref_bmp_to_iyuv.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint8), ctypes.c_uint32,
                                  ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]
    cap = max(1, os.path.getsize(path))  # the IYUV frame is smaller than the BMP file
    out = np.zeros(cap, np.uint8)
    w, h = ctypes.c_uint32(0), ctypes.c_uint32(0)
    rc = L.ref_bmp_to_iyuv(os.fsencode(path), _p(out), cap, ctypes.byref(w), ctypes.byref(h))
    if rc == 1:
        raise RefError(L.ref_last_error().decode())
    if rc:
        raise RuntimeError(f"ref_bmp_to_iyuv rc={rc}")
    return w.value, h.value, out[: w.value * h.value * 3 // 2].tobytes()
