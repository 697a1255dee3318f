// k_transform.hip — K1 fdct_quant_zz and K6 dequant_idct for gfx950.
//
// Both are HBM-bound streaming kernels: K1 reads 1 B/sample
// (u8 pixel) and writes 2 B/sample (int16 coefficient, zig-zag order); K6 the
// reverse.  Geometry: one wave = one "group" of 8 consecutive 8x8 blocks of one
// block-row.  Lane l = (row-or-column r = l>>3, block b = l&7):
//   load    lane (r,b) fetches row r of block b (8 B; the wave reads 8 rows x
//           64 contiguous bytes),
//   stage 1 lane (j,b) owns column j of block b: T = D·X (column transform),
//   stage 2 lane (i,b) owns row i of block b: Y = T·Dᵀ (row transform),
// with two 8x8 transposes through a per-wave LDS tile (block stride 68 floats:
// conflict-free for the column reads and writes).
//
// Bit-exactness (SURVEY.md §7 hard part 1, App. C): the reference computes
// each output as a straight k-ascending sum of fp32-rounded products
// (DCT.cpp:232-266), then an IEEE divide and roundf.  This file is compiled
// with -ffp-contract=off (no v_fma / v_pk_fma), the sums keep the reference's
// order, division is the correctly rounded HIP default, and roundf is
// half-away-from-zero.  No butterflies, no MFMA (an MFMA f32 product is an fma
// chain, which rounds differently).
#include "codec_common.hpp"

namespace myyuv_gpu {

__constant__ uint8_t c_zigzag[64] = MYYUV_ZIGZAG;
__constant__ uint8_t c_izigzag[64];  // filled on the host: izz[zigzag[z]] = z

namespace {

// Compile-time basis: folded into instruction literals (a __constant__ array
// would be re-read through the scalar cache on every use).
constexpr float c_dct[64] = MYYUV_DCT_MATRIX;

constexpr int kTileStride = 68;  // floats per block in the LDS tile
constexpr int kGroupBlocks = 8;

__device__ __forceinline__ void wave_sync() { __builtin_amdgcn_wave_barrier(); }

// Locate the wave's group: plane, block-row, first block of the group.
struct GroupPos {
  int p;
  uint32_t by, bx0, g0;  // g0 = global index of block (by, bx0)
  bool valid;
};

__device__ __forceinline__ GroupPos locate_group(const FrameGeom& G, uint32_t group) {
  GroupPos r;
  r.valid = group < G.gcum[3];
  r.p = group >= G.gcum[1] ? (group >= G.gcum[2] ? 2 : 1) : 0;
  uint32_t local = group - G.gcum[r.p];
  r.by = local / G.gpr[r.p];
  r.bx0 = (local - r.by * G.gpr[r.p]) * kGroupBlocks;
  r.g0 = G.cum[r.p] + r.by * G.bw[r.p] + r.bx0;
  return r;
}

}  // namespace

// K1: u8 planes -> int16 coefficients, zig-zag order, block-interleaved words.
// DCT.cpp:297-306 (gather, -128), :269-277 (applyDCTBlock), Huffman.cpp:176-182
// (zig-zag gather).
__global__ __launch_bounds__(256) void k_fdct_quant_zz(const uint8_t* __restrict__ frame,
                                                      FrameGeom G,
                                                      const QTables* __restrict__ qt,
                                                      uint32_t* __restrict__ coefw,
                                                      uint8_t* __restrict__ mszs) {
  __shared__ float tile_all[4][kGroupBlocks * kTileStride];
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  float* tile = tile_all[wave];
  const GroupPos gp = locate_group(G, blockIdx.x * 4 + wave);
  if (!gp.valid) return;  // whole wave exits together
  const int r = lane >> 3, b = lane & 7;
  const uint32_t bx = gp.bx0 + b;
  const bool live = bx < G.bw[gp.p];
  const uint32_t pw = G.pw[gp.p];

  // ---- load row r of block b, x - 128 (DCT.cpp:303) -> tile[b][r][0..7]
  uint2 raw = make_uint2(0x80808080u, 0x80808080u);
  if (live) {
    const uint8_t* src = frame + G.poff[gp.p] + (size_t)(gp.by * 8 + r) * pw + bx * 8;
    raw = *reinterpret_cast<const uint2*>(src);
  }
  {
    float4 lo, hi;
    lo.x = (float)((raw.x >> 0) & 0xFFu) - 128.0f;
    lo.y = (float)((raw.x >> 8) & 0xFFu) - 128.0f;
    lo.z = (float)((raw.x >> 16) & 0xFFu) - 128.0f;
    lo.w = (float)((raw.x >> 24) & 0xFFu) - 128.0f;
    hi.x = (float)((raw.y >> 0) & 0xFFu) - 128.0f;
    hi.y = (float)((raw.y >> 8) & 0xFFu) - 128.0f;
    hi.z = (float)((raw.y >> 16) & 0xFFu) - 128.0f;
    hi.w = (float)((raw.y >> 24) & 0xFFu) - 128.0f;
    float4* dst = reinterpret_cast<float4*>(tile + b * kTileStride + r * 8);
    dst[0] = lo;
    dst[1] = hi;
  }
  wave_sync();

  // ---- stage 1: lane (j=r, b) column j.  T[i][j] = sum_k D[i][k] * X[k][j]
  // (squareMatrixMul<8>(DCT, X), DCT.cpp:232-242, k ascending).
  {
    const int j = r;
    float x[8];
#pragma unroll
    for (int k = 0; k < 8; k++) x[k] = tile[b * kTileStride + k * 8 + j];
    float t[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      float s = c_dct[i * 8 + 0] * x[0];
#pragma unroll
      for (int k = 1; k < 8; k++) s = s + c_dct[i * 8 + k] * x[k];
      t[i] = s;
    }
    wave_sync();
#pragma unroll
    for (int i = 0; i < 8; i++) tile[b * kTileStride + i * 8 + j] = t[i];
  }
  wave_sync();

  // ---- stage 2: lane (i=r, b) row i.  Y[i][v] = sum_k T[i][k] * D[v][k]
  // (squareMatrixMulT<8>(T, DCT), DCT.cpp:244-254), then /Q, roundf, int16
  // (DCT.cpp:273-276).
  {
    const int i = r;
    const float4* trow = reinterpret_cast<const float4*>(tile + b * kTileStride + i * 8);
    const float4 t0 = trow[0], t1 = trow[1];
    const float t[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
    const float4* qrow = reinterpret_cast<const float4*>(&qt->q[gp.p][i * 8]);
    const float4 q0 = qrow[0], q1 = qrow[1];
    const float q[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
    const uint2 izz = *reinterpret_cast<const uint2*>(&c_izigzag[i * 8]);
    int c[8];
#pragma unroll
    for (int v = 0; v < 8; v++) {
      float s = t[0] * c_dct[v * 8 + 0];
#pragma unroll
      for (int k = 1; k < 8; k++) s = s + t[k] * c_dct[v * 8 + k];
      c[v] = (int)roundf(s / q[v]);
    }
    wave_sync();
    // scatter into zig-zag order: int16 view of the block's tile area
    int16_t* zz = reinterpret_cast<int16_t*>(tile + b * kTileStride);
#pragma unroll
    for (int v = 0; v < 8; v++) {
      const uint32_t word = v < 4 ? izz.x : izz.y;
      const int z = (word >> (8 * (v & 3))) & 0xFF;
      zz[z] = (int16_t)c[v];
    }
  }
  wave_sync();

  // ---- store: lane (s=r, b) writes zig-zag words 4s..4s+3 of block b into
  // the block-interleaved layout K2 reads (word w of block g at
  // ((g>>6)*32 + w)*64 + (g&63)), and the message length msz (1 + index of
  // the last nonzero zig-zag coefficient, Huffman.cpp:176-190) per block.
  {
    const uint4 v = *reinterpret_cast<const uint4*>(
        reinterpret_cast<const int16_t*>(tile + b * kTileStride) + r * 8);
    const uint32_t w8[4] = {v.x, v.y, v.z, v.w};
    int last = -1;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (w8[k] & 0xFFFFu) last = r * 8 + 2 * k;
      if (w8[k] >> 16) last = r * 8 + 2 * k + 1;
    }
    last = max(last, __shfl_xor(last, 8, 64));
    last = max(last, __shfl_xor(last, 16, 64));
    last = max(last, __shfl_xor(last, 32, 64));
    if (live) {
      const uint32_t g = gp.g0 + b;
      uint32_t* dst = coefw + (size_t)(g >> 6) * 32 * 64 + (g & 63);
#pragma unroll
      for (int k = 0; k < 4; k++) dst[(r * 4 + k) * 64] = w8[k];
      if (r == 0) mszs[g] = (uint8_t)(last + 1);
    }
  }
}

// K6: int16 zig-zag coefficients (block-interleaved words) -> u8 planes.
// DCT.cpp:330-334 (dequant, squareMatrixMulT2, squareMatrixMul), :358-362
// (roundf, +128, clamp).
__global__ __launch_bounds__(256) void k_dequant_idct(const uint32_t* __restrict__ coefw,
                                                     FrameGeom G,
                                                     const QTables* __restrict__ qt,
                                                     uint8_t* __restrict__ frame) {
  __shared__ float tile_all[4][kGroupBlocks * kTileStride];
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  float* tile = tile_all[wave];
  const GroupPos gp = locate_group(G, blockIdx.x * 4 + wave);
  if (!gp.valid) return;
  const int r = lane >> 3, b = lane & 7;
  const uint32_t bx = gp.bx0 + b;
  const bool live = bx < G.bw[gp.p];

  // ---- load zig-zag coefficients r*8..r*8+7 of block b, dequantise, and
  // scatter them to their natural positions in the tile.
  {
    uint4 raw = make_uint4(0, 0, 0, 0);
    if (live) {
      const uint32_t g = gp.g0 + b;
      const uint32_t* src = coefw + (size_t)(g >> 6) * 32 * 64 + (g & 63) + (r * 4) * 64;
      raw = make_uint4(src[0], src[64], src[128], src[192]);
    }
    const uint2 zz = *reinterpret_cast<const uint2*>(&c_zigzag[r * 8]);
    const float4* qrow = reinterpret_cast<const float4*>(&qt->qzz[gp.p][r * 8]);
    const float4 q0 = qrow[0], q1 = qrow[1];
    const float q[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
    const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
    for (int t = 0; t < 8; t++) {
      const int16_t cv = (int16_t)((w[t >> 1] >> (16 * (t & 1))) & 0xFFFF);
      const uint32_t zw = t < 4 ? zz.x : zz.y;
      const int n = (zw >> (8 * (t & 3))) & 0xFF;
      tile[b * kTileStride + n] = (float)cv * q[t];  // DCT.cpp:331
    }
  }
  wave_sync();

  // ---- stage 1: lane (j=r, b) column j.  U[i][j] = sum_k D[k][i] * Z[k][j]
  // (squareMatrixMulT2<8>(DCT, Z), DCT.cpp:256-266).
  {
    const int j = r;
    float z[8];
#pragma unroll
    for (int k = 0; k < 8; k++) z[k] = tile[b * kTileStride + k * 8 + j];
    float u[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      float s = c_dct[0 * 8 + i] * z[0];
#pragma unroll
      for (int k = 1; k < 8; k++) s = s + c_dct[k * 8 + i] * z[k];
      u[i] = s;
    }
    wave_sync();
#pragma unroll
    for (int i = 0; i < 8; i++) tile[b * kTileStride + i * 8 + j] = u[i];
  }
  wave_sync();

  // ---- stage 2: lane (i=r, b) row i.  R[i][v] = sum_k U[i][k] * D[k][v]
  // (squareMatrixMul<8>(U, DCT)), then clamp(roundf(R) + 128) and store the
  // 8-pixel row directly (the wave writes 8 rows x 64 contiguous bytes).
  {
    const int i = r;
    const float4* urow = reinterpret_cast<const float4*>(tile + b * kTileStride + i * 8);
    const float4 u0 = urow[0], u1 = urow[1];
    const float u[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
    uint32_t packed[2] = {0, 0};
#pragma unroll
    for (int v = 0; v < 8; v++) {
      float s = u[0] * c_dct[0 * 8 + v];
#pragma unroll
      for (int k = 1; k < 8; k++) s = s + u[k] * c_dct[k * 8 + v];
      int px = (int)roundf(s) + 128;
      px = px < 0 ? 0 : (px > 255 ? 255 : px);
      packed[v >> 2] |= (uint32_t)px << (8 * (v & 3));
    }
    if (live) {
      uint8_t* dst = frame + G.poff[gp.p] + (size_t)(gp.by * 8 + i) * G.pw[gp.p] + bx * 8;
      *reinterpret_cast<uint2*>(dst) = make_uint2(packed[0], packed[1]);
    }
  }
}

}  // namespace myyuv_gpu
