// k_color.hip — K7: BMP (BGR / BGRA) -> IYUV 4:2:0, the step before compress
// (SURVEY.md §8f row 3).  Replaces YUV(const BMP&, IYUV): bmp_to_yuv_map[IYUV]
// (myyuv_lib/myyuv_yuv.cpp:88-128) over BMP::colorData (myyuv_bmp.cpp:77-101),
// getYUV444FromRGB2x2 (myyuv_yuv.cpp:34-52) and divide_roundnearest<uint8_t>
// (:20-27).
//
// Pure streaming: 3 or 4 B read + 1.5 B written per pixel, no reuse, so the
// bound is HBM.  A lane converts a 4x2 pixel tile (two 2x2 chroma quads):
// one 16-B (BGRA) or 12-B (BGR) load per pixel row — consecutive lanes read
// consecutive tiles, and width % 4 == 0 (BMP::isValidHeader) keeps every load
// dword aligned — then a 4-B luma store per row and a 2-B store per chroma
// plane.  colorData's re-orientation is folded into the source addressing
// (no flipped copy of the image).
//
// Numerics are the reference x86-64 build's (checked against it and against
// the golden chef-with-trumpet.myyuv in tests/test_color.py): fp32
// Y = 0.299 R + 0.587 G + 0.114 B, products and sums left to right, no FMA
// (-ffp-contract=off); float -> uint8_t casts truncate through a 32-bit
// integer (cvttss2si) and keep the low byte (the +128 offset of a negative
// chroma value wraps through it); the 4-term chroma sum wraps mod 256, so a
// saturated-blue quad has Cb 0, as the reference's has.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "codec_common.hpp"

namespace myyuv_gpu {

namespace {

__device__ __forceinline__ uint32_t trunc_u8(float x) { return (uint32_t)(int32_t)x & 0xFFu; }

// getYUV444FromRGB2x2's per-pixel step; returns Y and the two chroma values
// already divided by 4 with round-to-nearest (divide_roundnearest(c, 4)).
__device__ __forceinline__ void pixel(uint32_t b, uint32_t g, uint32_t r, uint32_t& y,
                                      uint32_t& cb4, uint32_t& cr4) {
  const float B = (float)b, G = (float)g, R = (float)r;
  const float Y = 0.299f * R + 0.587f * G + 0.114f * B;
  y = trunc_u8(Y);
  cb4 = (((trunc_u8((B - Y) * 0.564f) + 128u) & 0xFFu) + 2u) >> 2;
  cr4 = (((trunc_u8((R - Y) * 0.713f) + 128u) & 0xFFu) + 2u) >> 2;
}

// byte k of a little-endian word array (k static after unrolling)
template <int N>
__device__ __forceinline__ uint32_t byte_at(const uint32_t (&w)[N], int k) {
  return (w[k >> 2] >> ((k & 3) * 8)) & 0xFFu;
}

// Four consecutive source pixels starting at pixel index `pix` (pix % 4 == 0).
template <int BPP>
__device__ __forceinline__ void load4(const uint8_t* __restrict__ src, size_t pix,
                                      uint32_t (&w)[BPP]) {
  const uint32_t* p = reinterpret_cast<const uint32_t*>(src + pix * BPP);
  if constexpr (BPP == 4) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    w[0] = v.x, w[1] = v.y, w[2] = v.z, w[3] = v.w;
  } else {
#pragma unroll
    for (int i = 0; i < BPP; i++) w[i] = p[i];
  }
}

}  // namespace

// One lane per 4x2 tile, grid-stride.  orient: 0 = rows as stored (width > 0,
// height < 0), 1 = pixel order reversed (width < 0, height > 0), 2 = rows
// bottom-up (width > 0, height > 0): the three cases of BMP::colorData.
template <int BPP>
__global__ __launch_bounds__(256) void k_bmp_to_iyuv(const uint8_t* __restrict__ src, uint32_t W,
                                                     uint32_t H, uint32_t orient,
                                                     uint8_t* __restrict__ dst) {
  const uint32_t tiles_x = W / 4;
  const uint32_t ntiles = tiles_x * (H / 2);
  const size_t npx = (size_t)W * H;
  uint8_t* __restrict__ u = dst + npx;
  uint8_t* __restrict__ v = u + npx / 4;
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < ntiles; t += gridDim.x * blockDim.x) {
    const uint32_t ty = t / tiles_x, tx = t - ty * tiles_x;
    const uint32_t r = 2 * ty, c = 4 * tx;
    uint32_t Y[2] = {0, 0}, cb[2] = {0, 0}, cr[2] = {0, 0};
#pragma unroll
    for (int dr = 0; dr < 2; dr++) {
      const size_t lin = (size_t)(r + dr) * W + c;  // colorData pixel index of the tile row
      size_t base;
      if (orient == 0)
        base = lin;
      else if (orient == 1)
        base = npx - 4 - lin;  // pixels lin..lin+3 are source npx-1-lin .. npx-4-lin
      else
        base = (size_t)(H - 1 - (r + dr)) * W + c;
      uint32_t w[BPP];
      load4<BPP>(src, base, w);
#pragma unroll
      for (int k = 0; k < 4; k++) {
        uint32_t b, g, rr;
        if (orient == 1) {  // uniform branch: both orders keep static byte indices
          b = byte_at(w, (3 - k) * BPP), g = byte_at(w, (3 - k) * BPP + 1), rr = byte_at(w, (3 - k) * BPP + 2);
        } else {
          b = byte_at(w, k * BPP), g = byte_at(w, k * BPP + 1), rr = byte_at(w, k * BPP + 2);
        }
        uint32_t y, cb4, cr4;
        pixel(b, g, rr, y, cb4, cr4);
        Y[dr] |= y << (8 * k);
        cb[k >> 1] += cb4;
        cr[k >> 1] += cr4;
      }
    }
    *reinterpret_cast<uint32_t*>(dst + (size_t)r * W + c) = Y[0];
    *reinterpret_cast<uint32_t*>(dst + (size_t)(r + 1) * W + c) = Y[1];
    const size_t k = (size_t)ty * (W / 2) + 2 * tx;
    *reinterpret_cast<uint16_t*>(u + k) = (uint16_t)((cb[0] & 0xFFu) | (cb[1] & 0xFFu) << 8);
    *reinterpret_cast<uint16_t*>(v + k) = (uint16_t)((cr[0] & 0xFFu) | (cr[1] & 0xFFu) << 8);
  }
}

template __global__ void k_bmp_to_iyuv<3>(const uint8_t*, uint32_t, uint32_t, uint32_t, uint8_t*);
template __global__ void k_bmp_to_iyuv<4>(const uint8_t*, uint32_t, uint32_t, uint32_t, uint8_t*);

}  // namespace myyuv_gpu
