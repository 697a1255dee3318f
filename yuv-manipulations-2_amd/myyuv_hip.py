"""ctypes binding of the C ABI (include/myyuv_hip.h) of the gfx950 DCT codec.

This is the Python view of the product path: every call goes to
libmyyuv_hip.so (HIP kernels).  There is no CPU fallback — if the library or
a GPU is missing, calls raise.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# MYYUV_HIP_LIB selects a diagnostic build (e.g. build/stamps/libmyyuv_hip.so)
LIB_PATH = os.environ.get("MYYUV_HIP_LIB") or os.path.join(_HERE, "libmyyuv_hip.so")

OK = 0
E_ARG, E_QUALITY, E_WIDTH, E_HEIGHT, E_CAPACITY = 1, 2, 3, 4, 5
E_DCTYUV_SIZE, E_PLANE_SIZE, E_PLANE_NBLK, E_PLANE_CONTENT = 6, 7, 8, 9
E_BAD_CODE, E_UNKNOWN_SYMBOL, E_BAD_CHUNK, E_HIP, E_NO_DEVICE = 10, 11, 12, 13, 14
E_BMP_INVALID, E_BMP_SIGN, E_BMP_UNSUPPORTED = 15, 16, 17

KERNELS = ["fdct_quant", "huff_encode", "scan_tiles", "stream_out", "encode_tile", "huff_decode",
           "dequant_idct", "huff_encode_wide", "huff_encode_r16", "huff_encode_wave", "bmp_to_iyuv",
           "fdct_fix"]
# ids: MYYUV_K_* of include/myyuv_hip.h, in KERNELS order (tests/test_cabi.py checks both)
(K_FDCT, K_HUFF_ENC, K_SCAN, K_COMPACT, K_ENCODE_TILE, K_HUFF_DEC, K_IDCT, K_HUFF_WIDE,
 K_HUFF_R16, K_HUFF_WAVE, K_BMP, K_FDCT_FIX) = range(len(KERNELS))

# the exported symbols include/myyuv_hip.h declares (checked by the CPU tests)
EXPORTS = [
    "myyuv_hip_create", "myyuv_hip_destroy", "myyuv_hip_strerror", "myyuv_dct_payload_bound",
    "myyuv_gpu_dct_compress", "myyuv_gpu_dct_decompress", "myyuv_hip_reserve",
    "myyuv_gpu_dct_compress_device", "myyuv_gpu_dct_decompress_device", "myyuv_hip_sync_status",
    "myyuv_hip_profile", "myyuv_hip_profile_kernels", "myyuv_hip_kernel_stats", "myyuv_gpu_fdct_blocks",
    "myyuv_gpu_huff_encode_blocks", "myyuv_hip_reserve_batch", "myyuv_gpu_dct_compress_batch_device",
    "myyuv_gpu_dct_decompress_batch_device", "myyuv_gpu_bmp_to_iyuv", "myyuv_gpu_bmp_to_iyuv_device",
    "myyuv_gpu_dct_compress_batch", "myyuv_gpu_dct_compress_frames", "myyuv_gpu_dct_decompress_frames",
    "myyuv_gpu_dct_decompress_batch",
]

_lib = None
# myyuv_payload_alloc_fn
PAYLOAD_ALLOC = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32)


class CodecError(RuntimeError):
    """A MYYUV_E_* failure; .code is the number, str() the reference's message."""

    def __init__(self, code, bad_block=-1):
        self.code = code
        self.bad_block = bad_block
        super().__init__(strerror(code) if _lib is not None else f"error {code}")


def _share_hip_runtime_with_torch():
    """torch ships its own libamdhip64 with the same soname (libamdhip64.so.7)
    as /opt/rocm's.  Two copies in one process means two HIP/HSA runtimes and
    the second one finds no GPU.  When torch is importable, load it first so
    this library binds to the runtime torch already mapped (the loader matches
    our NEEDED libamdhip64.so.7 against it); without torch the library uses
    /opt/rocm's runtime through its RUNPATH."""
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def load():
    global _lib
    if _lib is not None:
        return _lib
    if os.environ.get("MYYUV_NO_TORCH_RUNTIME") != "1":
        _share_hip_runtime_with_torch()
    if not os.path.exists(LIB_PATH):
        raise FileNotFoundError(f"{LIB_PATH} missing: build it with `make -C yuv-manipulations-2_amd`"
                                " or __graft_entry__.build()")
    L = ctypes.CDLL(LIB_PATH)
    u8p = ctypes.POINTER(ctypes.c_uint8)
    vp = ctypes.c_void_p
    u32 = ctypes.c_uint32
    L.myyuv_hip_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.myyuv_hip_destroy.argtypes = [vp]
    L.myyuv_hip_destroy.restype = None
    L.myyuv_hip_strerror.argtypes = [ctypes.c_int]
    L.myyuv_hip_strerror.restype = ctypes.c_char_p
    L.myyuv_dct_payload_bound.argtypes = [u32, u32]
    L.myyuv_dct_payload_bound.restype = u32
    L.myyuv_gpu_dct_compress.argtypes = [vp, u8p, u32, u32, u8p, u8p, u32, ctypes.POINTER(u32)]
    L.myyuv_gpu_dct_decompress.argtypes = [vp, u8p, u32, u32, u32, u8p, u8p,
                                           ctypes.POINTER(ctypes.c_int64)]
    L.myyuv_hip_reserve.argtypes = [vp, u32, u32]
    L.myyuv_gpu_dct_compress_device.argtypes = [vp, vp, u32, u32, u8p, vp, u32, vp, vp]
    L.myyuv_gpu_dct_decompress_device.argtypes = [vp, vp, vp, u32, u32, u32, u8p, vp, vp]
    L.myyuv_hip_reserve_batch.argtypes = [vp, u32, u32, u32]
    L.myyuv_gpu_dct_compress_batch_device.argtypes = [vp, vp, u32, u32, u32, u8p, vp, u32, vp, vp]
    L.myyuv_gpu_dct_decompress_batch_device.argtypes = [vp, vp, vp, u32, u32, u32, u32, u8p, vp, vp]
    L.myyuv_hip_sync_status.argtypes = [vp, vp, ctypes.POINTER(ctypes.c_int64)]
    L.myyuv_hip_profile.argtypes = [vp, ctypes.c_int]
    L.myyuv_hip_profile_kernels.argtypes = [vp, ctypes.c_uint32]
    L.myyuv_hip_kernel_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_double),
                                         ctypes.POINTER(ctypes.c_int64)]
    L.myyuv_gpu_fdct_blocks.argtypes = [vp, u8p, u32, ctypes.POINTER(ctypes.c_float),
                                        ctypes.POINTER(ctypes.c_int16)]
    L.myyuv_gpu_huff_encode_blocks.argtypes = [vp, ctypes.POINTER(ctypes.c_int16), u32, u8p, u8p]
    i32 = ctypes.c_int32
    L.myyuv_gpu_bmp_to_iyuv.argtypes = [vp, u8p, i32, i32, ctypes.c_uint16, u8p]
    L.myyuv_gpu_bmp_to_iyuv_device.argtypes = [vp, vp, i32, i32, ctypes.c_uint16, vp, vp]
    L.myyuv_gpu_dct_compress_batch.argtypes = [vp, u8p, u32, u32, u32, u8p, u8p, u32, ctypes.POINTER(u32)]
    L.myyuv_gpu_dct_decompress_batch.argtypes = [vp, u8p, ctypes.POINTER(u32), u32, u32, u32, u32, u8p, u8p,
                                                 ctypes.POINTER(ctypes.c_int64)]
    L.myyuv_gpu_dct_decompress_frames.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(u32), u32, u32, u32, u8p,
                                                  ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_int64)]
    L.myyuv_gpu_dct_compress_frames.argtypes = [vp, ctypes.POINTER(vp), u32, u32, u32, u8p, PAYLOAD_ALLOC, vp,
                                                ctypes.POINTER(u32)]
    L.myyuv_debug_tinfo_guard.argtypes = [vp, u32, ctypes.c_int, ctypes.POINTER(u32)]  # diagnostic
    _lib = L
    return L


def strerror(code):
    return load().myyuv_hip_strerror(int(code)).decode()


def payload_bound(w, h):
    return load().myyuv_dct_payload_bound(w, h)


def batch_tiles(w, h):
    """K2's 256-block tiles per frame (FrameGeom::tcum[3]): per plane
    ceil(blocks / 256), Y then U and V."""
    y = (w // 8) * (h // 8)
    c = (w // 16) * (h // 16)
    return -(-y // 256) + 2 * -(-c // 256)


def _u8(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def _u8_array(a, name, writable=False):
    """The caller's buffer as-is (no copy): a C-contiguous uint8 ndarray, else
    ValueError (a strided or wider-typed array would hand the C ABI the wrong
    bytes, and a copy of `out` would drop the result)."""
    if not isinstance(a, np.ndarray) or a.dtype != np.uint8 or not a.flags.c_contiguous:
        raise ValueError(f"{name}: a C-contiguous numpy uint8 array is required")
    if writable and not a.flags.writeable:
        raise ValueError(f"{name}: read-only array")
    return a


def _q(q):
    return np.ascontiguousarray(np.array(q, dtype=np.int64).astype(np.uint8))


class Codec:
    """One context (HIP stream + workspace) on one device."""

    def __init__(self, device=0):
        L = load()
        h = ctypes.c_void_p()
        rc = L.myyuv_hip_create(int(device), ctypes.byref(h))
        if rc:
            raise CodecError(rc)
        self._h = h
        self.device = device

    def close(self):
        if self._h:
            load().myyuv_hip_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- host-buffer API (what YUV::compress_map / decompress_map call) --
    def compress(self, iyuv, w, h, q):
        """IYUV bytes -> DCTYUV payload bytes."""
        src = np.ascontiguousarray(np.frombuffer(memoryview(iyuv).cast("B"), np.uint8))
        if src.size < w * h * 3 // 2:
            raise ValueError("frame smaller than W*H*3/2")
        qa = _q(q)
        cap = payload_bound(w, h)
        out = np.empty(cap, np.uint8)
        size = ctypes.c_uint32(0)
        rc = load().myyuv_gpu_dct_compress(self._h, _u8(src), w, h, _u8(qa), _u8(out), cap,
                                           ctypes.byref(size))
        if rc:
            raise CodecError(rc)
        return out[: size.value].tobytes()

    def decompress(self, payload, w, h, q):
        src = np.ascontiguousarray(np.frombuffer(memoryview(payload).cast("B"), np.uint8))
        qa = _q(q)
        out = np.empty(w * h * 3 // 2, np.uint8)
        bad = ctypes.c_int64(-1)
        rc = load().myyuv_gpu_dct_decompress(self._h, _u8(src), src.size, w, h, _u8(qa),
                                             _u8(out), ctypes.byref(bad))
        if rc:
            raise CodecError(rc, bad.value)
        return out.tobytes()

    def compress_into(self, iyuv, w, h, q, out):
        """IYUV numpy buffer -> payload written into the caller's numpy buffer
        `out` (no per-call allocation); returns the payload size.  Both must be
        C-contiguous uint8 arrays: `iyuv` at least W*H*3/2 bytes, `out` sized
        by its byte count (a short `out` fails with E_CAPACITY)."""
        src = _u8_array(iyuv, "iyuv")
        dst = _u8_array(out, "out", writable=True)
        if src.nbytes < w * h * 3 // 2:
            raise ValueError("frame smaller than W*H*3/2")
        size = ctypes.c_uint32(0)
        rc = load().myyuv_gpu_dct_compress(self._h, _u8(src), w, h, _u8(_q(q)), _u8(dst), dst.nbytes,
                                           ctypes.byref(size))
        if rc:
            raise CodecError(rc)
        return size.value

    def decompress_into(self, payload, w, h, q, out):
        """payload numpy buffer -> IYUV frame written into the caller's numpy
        buffer `out` (at least W*H*3/2 bytes); both C-contiguous uint8."""
        src = _u8_array(payload, "payload")
        dst = _u8_array(out, "out", writable=True)
        if dst.nbytes < w * h * 3 // 2:
            raise ValueError("output smaller than W*H*3/2")
        bad = ctypes.c_int64(-1)
        rc = load().myyuv_gpu_dct_decompress(self._h, _u8(src), src.nbytes, w, h, _u8(_q(q)), _u8(dst),
                                             ctypes.byref(bad))
        if rc:
            raise CodecError(rc, bad.value)

    def compress_batch(self, frames, w, h, q):
        """Host-buffer batch: a list of IYUV frames of one geometry -> their
        DCTYUV payloads (one launch per kernel for the batch)."""
        n = len(frames)
        fb = w * h * 3 // 2
        for i, f in enumerate(frames):
            if len(memoryview(f).cast("B")) != fb:
                raise ValueError(f"frame {i}: {len(memoryview(f).cast('B'))} bytes, a {w}x{h} IYUV frame has {fb}")
        src = np.ascontiguousarray(np.frombuffer(b"".join(bytes(f) for f in frames), np.uint8))
        cap = (payload_bound(w, h) + 3) & ~3
        out = np.empty(n * cap, np.uint8)
        sizes = (ctypes.c_uint32 * n)()
        rc = load().myyuv_gpu_dct_compress_batch(self._h, _u8(src), n, w, h, _u8(_q(q)), _u8(out), cap, sizes)
        if rc:
            raise CodecError(rc)
        return [out[i * cap: i * cap + sizes[i]].tobytes() for i in range(n)]

    def compress_frames(self, frames, w, h, q):
        """Host-buffer batch through the pointer-array entry point: each
        payload is written into a buffer sized once its length is known."""
        n = len(frames)
        fb = w * h * 3 // 2
        srcs = [np.frombuffer(bytes(f), np.uint8) for f in frames]
        for i, a in enumerate(srcs):
            if a.size != fb:
                raise ValueError(f"frame {i}: {a.size} bytes, a {w}x{h} IYUV frame has {fb}")
        ptrs = (ctypes.c_void_p * n)(*[a.ctypes.data for a in srcs])
        outs = [None] * n

        def alloc(_user, f, size):
            outs[f] = np.empty(max(size, 1), np.uint8)
            return outs[f].ctypes.data

        cb = PAYLOAD_ALLOC(alloc)
        sizes = (ctypes.c_uint32 * n)()
        rc = load().myyuv_gpu_dct_compress_frames(self._h, ptrs, n, w, h, _u8(_q(q)), cb, None, sizes)
        if rc:
            raise CodecError(rc)
        return [outs[i][: sizes[i]].tobytes() for i in range(n)]

    def decompress_batch(self, payloads, w, h, q):
        """Host-buffer batch decompress (pipelined): a list of DCTYUV
        payloads of one geometry and quality -> their IYUV frames."""
        n = len(payloads)
        fb = w * h * 3 // 2
        cap = max(len(p) for p in payloads)
        src = np.zeros(n * cap, np.uint8)
        sizes = (ctypes.c_uint32 * n)()
        for i, p in enumerate(payloads):
            src[i * cap: i * cap + len(p)] = np.frombuffer(bytes(p), np.uint8)
            sizes[i] = len(p)
        out = np.empty(n * fb, np.uint8)
        bad = ctypes.c_int64(-1)
        rc = load().myyuv_gpu_dct_decompress_batch(self._h, _u8(src), sizes, cap, n, w, h, _u8(_q(q)), _u8(out),
                                                   ctypes.byref(bad))
        if rc:
            raise CodecError(rc, bad.value)
        return [out[i * fb:(i + 1) * fb].tobytes() for i in range(n)]

    def decompress_frames(self, payloads, w, h, q):
        """The pointer-array form of decompress_batch."""
        n = len(payloads)
        fb = w * h * 3 // 2
        srcs = [np.frombuffer(bytes(p), np.uint8) for p in payloads]
        outs = [np.empty(fb, np.uint8) for _ in range(n)]
        ip = (ctypes.c_void_p * n)(*[a.ctypes.data for a in srcs])
        op = (ctypes.c_void_p * n)(*[a.ctypes.data for a in outs])
        sizes = (ctypes.c_uint32 * n)(*[a.size for a in srcs])
        bad = ctypes.c_int64(-1)
        rc = load().myyuv_gpu_dct_decompress_frames(self._h, ip, sizes, n, w, h, _u8(_q(q)), op, ctypes.byref(bad))
        if rc:
            raise CodecError(rc, bad.value)
        return [o.tobytes() for o in outs]

    def bmp_to_iyuv(self, bmp_data, width, height, bit_count):
        """BMP::data (as stored; signed header width/height) -> IYUV bytes,
        as YUV(const BMP&, IYUV) (myyuv_yuv.cpp:88-128)."""
        src = np.ascontiguousarray(np.frombuffer(memoryview(bmp_data).cast("B"), np.uint8))
        W, H = abs(int(width)), abs(int(height))
        if src.size < W * H * (bit_count // 8):
            raise ValueError("pixel array smaller than |w|*|h|*bit_count/8")
        out = np.empty(max(1, W * H * 3 // 2), np.uint8)
        rc = load().myyuv_gpu_bmp_to_iyuv(self._h, _u8(src), int(width), int(height), int(bit_count),
                                          _u8(out))
        if rc:
            raise CodecError(rc)
        return out[: W * H * 3 // 2].tobytes()

    def bmp_to_iyuv_device(self, d_bmp, width, height, bit_count, d_iyuv, stream=None):
        rc = load().myyuv_gpu_bmp_to_iyuv_device(self._h, d_bmp, int(width), int(height),
                                                 int(bit_count), d_iyuv, stream)
        if rc:
            raise CodecError(rc)

    # -- device-resident API (pointers are device addresses, e.g. torch data_ptr) --
    def reserve(self, w, h):
        rc = load().myyuv_hip_reserve(self._h, w, h)
        if rc:
            raise CodecError(rc)

    def compress_device(self, d_iyuv, w, h, q, d_payload, cap, d_size, stream=None):
        rc = load().myyuv_gpu_dct_compress_device(self._h, d_iyuv, w, h, _u8(_q(q)), d_payload,
                                                  cap, d_size, stream)
        if rc:
            raise CodecError(rc)

    def decompress_device(self, d_payload, d_size, cap, w, h, q, d_iyuv, stream=None):
        rc = load().myyuv_gpu_dct_decompress_device(self._h, d_payload, d_size, cap, w, h,
                                                    _u8(_q(q)), d_iyuv, stream)
        if rc:
            raise CodecError(rc)

    # batches: frame f at d_iyuv + f*W*H*3/2, payload f at d_payload + f*cap,
    # its size at d_sizes[f] (u32)
    def reserve_batch(self, w, h, nframes):
        rc = load().myyuv_hip_reserve_batch(self._h, w, h, nframes)
        if rc:
            raise CodecError(rc)

    def compress_batch_device(self, d_iyuv, nframes, w, h, q, d_payload, cap, d_sizes, stream=None):
        rc = load().myyuv_gpu_dct_compress_batch_device(self._h, d_iyuv, nframes, w, h, _u8(_q(q)),
                                                        d_payload, cap, d_sizes, stream)
        if rc:
            raise CodecError(rc)

    def decompress_batch_device(self, d_payload, d_sizes, cap, nframes, w, h, q, d_iyuv, stream=None):
        rc = load().myyuv_gpu_dct_decompress_batch_device(self._h, d_payload, d_sizes, cap, nframes, w,
                                                          h, _u8(_q(q)), d_iyuv, stream)
        if rc:
            raise CodecError(rc)

    def sync_status(self, stream=None):
        bad = ctypes.c_int64(-1)
        rc = load().myyuv_hip_sync_status(self._h, stream, ctypes.byref(bad))
        return rc, bad.value

    def profile(self, enable, kernels=None):
        """Per-kernel event stamping: all kernels, or only the named ones."""
        if kernels is None:
            rc = load().myyuv_hip_profile(self._h, 1 if enable else 0)
        else:
            mask = sum(1 << KERNELS.index(k) for k in kernels) if enable else 0
            rc = load().myyuv_hip_profile_kernels(self._h, mask)
        if rc:
            raise CodecError(rc)

    def kernel_stats(self):
        ms = (ctypes.c_double * len(KERNELS))()
        n = (ctypes.c_int64 * len(KERNELS))()
        rc = load().myyuv_hip_kernel_stats(self._h, ms, n)
        if rc:
            raise CodecError(rc)
        return {KERNELS[i]: (ms[i], n[i]) for i in range(len(KERNELS))}

    def tinfo_guard(self, ntiles, arm):
        """Diagnostic (not in include/myyuv_hip.h): arm=True writes a canary
        into the tile-info words past batch tile ntiles; arm=False returns how
        many of them a kernel overwrote since."""
        n = ctypes.c_uint32(0)
        rc = load().myyuv_debug_tinfo_guard(self._h, int(ntiles), 1 if arm else 0, ctypes.byref(n))
        if rc:
            raise CodecError(rc)
        return n.value

    # -- block-level known-answer entry points --
    def fdct_blocks(self, px, qtable):
        px = np.ascontiguousarray(px, np.uint8).reshape(-1, 64)
        qt = np.ascontiguousarray(qtable, np.float32).reshape(64)
        out = np.empty((px.shape[0], 64), np.int16)
        rc = load().myyuv_gpu_fdct_blocks(self._h, _u8(px), px.shape[0],
                                          qt.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                          out.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)))
        if rc:
            raise CodecError(rc)
        return out

    def huff_encode_blocks(self, coef_zz):
        c = np.ascontiguousarray(coef_zz, np.int16).reshape(-1, 64)
        n = c.shape[0]
        chunks = np.zeros((n, 160), np.uint8)
        sizes = np.zeros(n, np.uint8)
        rc = load().myyuv_gpu_huff_encode_blocks(
            self._h, c.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)), n, _u8(chunks), _u8(sizes))
        if rc:
            raise CodecError(rc)
        return [chunks[i, : sizes[i]].tobytes() for i in range(n)]
