"""The .myyuv container on the Python side (tests, bench, batch driver).

Mirrors the parts of myyuv::YUV the DCT path uses (myyuv_yuv.hpp:17-28,
myyuv_yuv.cpp:374-423, 485-536) and the header rewrites of
compress_DCT_planar / decompress_DCT_planar (DCT.cpp:389-396, 446-453).
The C++ mirror of the same API is csrc/host/myyuv_yuv.{hpp,cpp}.
"""
import struct

HEADER = struct.Struct("<2sIIHIIIII32s")  # 64 bytes, #pragma pack(1)
IYUV = 0x56555949
NONE, DCT = 0, 1


class YUVFile:
    def __init__(self, fourcc=IYUV, width=0, height=0, compression=NONE, params=b"", data=b"",
                 unused=b"\0" * 32):
        self.fourcc = fourcc
        self.width = width
        self.height = height
        self.compression = compression
        self.params = bytes(params)
        self.data = bytes(data)
        self.unused = bytes(unused)

    # YUV::getImageSize (myyuv_yuv.cpp:374-381): IYUV = 8 + 2 + 2 bits/pixel
    def image_size(self):
        return self.width * self.height * 3 // 2

    @classmethod
    def load(cls, path_or_bytes):
        """YUV::load (myyuv_yuv.cpp:485-510), including its normalisation of
        params_pos / data_pos and of data_size for raw images."""
        b = path_or_bytes if isinstance(path_or_bytes, (bytes, bytearray)) else open(path_or_bytes, "rb").read()
        (typ, fourcc, data_size, comp, psz, ppos, w, h, dpos, unused) = HEADER.unpack(b[:64])
        if typ != b"YU" or fourcc != IYUV or w == 0 or h == 0 or dpos < 64 + psz or data_size == 0:
            raise ValueError("Error bad header")
        params = bytes(b[ppos:ppos + psz]) if psz else b""
        if comp == NONE:
            data_size = w * h * 3 // 2
        data = bytes(b[dpos:dpos + data_size])
        return cls(fourcc, w, h, comp, params, data, unused)

    def header_bytes(self):
        psz = len(self.params)
        return HEADER.pack(b"YU", self.fourcc, len(self.data), self.compression, psz,
                           64 if psz else 0, self.width, self.height, 64 + psz, self.unused)

    def dumps(self):
        """YUV::dump (myyuv_yuv.cpp:525-536): header + params + data."""
        return self.header_bytes() + self.params + self.data

    def dump(self, path):
        with open(path, "wb") as f:
            f.write(self.dumps())

    def planes(self):
        w, h = self.width, self.height
        d = self.data
        return d[: w * h], d[w * h: w * h * 5 // 4], d[w * h * 5 // 4: w * h * 3 // 2]

    # header rewrites of compress_DCT_planar (DCT.cpp:389-396)
    def compressed(self, q, payload):
        return YUVFile(self.fourcc, self.width, self.height, DCT, bytes(q), payload, self.unused)

    # ... and of decompress_DCT_planar (DCT.cpp:446-453)
    def decompressed(self, iyuv):
        return YUVFile(self.fourcc, self.width, self.height, NONE, b"", iyuv, self.unused)


# ---- BMP input (myyuv_bmp.hpp:8-39, myyuv_bmp.cpp:141-166) ----
BMP_HEADER = struct.Struct("<2sIHHIIiiHHIIiiII")  # 54 bytes, #pragma pack(1)
BMP_COLOR = struct.Struct("<IIIII64s")            # 84 bytes (BMPColorHeader)


class BMPFile:
    """BMP::load: the 54-byte header, the colour header for 32-bit images,
    then imageSize() = |w|*|h|*bit_count/8 bytes from data_pos."""

    def __init__(self, width, height, bit_count, data, header=None, color=None):
        self.width, self.height, self.bit_count = width, height, bit_count
        self.data = bytes(data)
        self.header = header
        self.color = color or (0x00FF0000, 0x0000FF00, 0x000000FF, 0xFF000000, 0x73524742)

    @classmethod
    def load(cls, path_or_bytes):
        b = path_or_bytes if isinstance(path_or_bytes, (bytes, bytearray)) else open(path_or_bytes, "rb").read()
        hdr = BMP_HEADER.unpack(b[:54])
        (typ, _fsz, _r1, _r2, dpos, hsz, w, h, _pl, bits, comp, _sz, _xp, _yp, cu, ci) = hdr
        color = None
        if bits == 32:
            color = BMP_COLOR.unpack(b[54:54 + 84])[:5]
        size = abs(w) * abs(h) * bits // 8
        return cls(w, h, bits, b[dpos:dpos + size], hdr, color)

    def is_valid_header(self):
        """BMP::isValidHeader (myyuv_bmp.cpp:125-139)."""
        typ, hsz, comp, cu, ci = (self.header[0], self.header[5], self.header[10], self.header[14],
                                  self.header[15]) if self.header else (b"BM", 40, 0, 0, 0)
        r, g, bl, a, cs = self.color
        return (typ == b"BM" and self.width % 4 == 0 and self.bit_count > 0 and hsz > 0
                and comp in (0, 3) and cu == 0 and ci == 0 and r == 0x00FF0000 and g == 0x0000FF00
                and bl == 0x000000FF and a in (0xFF000000, 0) and cs == 0x73524742)

    def dumps(self):
        """BMP::dump layout (myyuv_bmp.cpp:168-179), for synthetic test images."""
        bits = self.bit_count
        dpos = 54 + (84 if bits == 32 else 0)
        size = len(self.data)
        out = BMP_HEADER.pack(b"BM", dpos + size, 0, 0, dpos, 124 if bits == 32 else 40, self.width,
                              self.height, 1, bits, 3 if bits == 32 else 0, 0, 0, 0, 0, 0)
        if bits == 32:
            out += BMP_COLOR.pack(*self.color, b"\0" * 64)
        return out + self.data
