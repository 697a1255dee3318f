// k_transform.hip — K1 fdct_quant and K6 dequant_idct for gfx950.
//
// Streaming kernels: K1 reads 1 B/sample (u8 pixel) and writes 2 B/sample
// (int16 coefficient), K6 the reverse (3 B/sample each).  The
// bit-exact transform is 8 fp32 products + 7 sums per output per stage in a
// fixed order (~30 VALU per sample); at the 8 TB/s ridge the budget is ~10
// lane-ops per byte, so the arithmetic sets the pace and the code is shaped
// by the issue rates measured on this chip (tools/ubench/valu_mix.hip,
// profiles/r01_ubench_valu_mix.txt):
//   * independent VOP2 f32 ops with an inline literal issue every ~1.0 ns per
//     SIMD; packed v_pk_* ops do two lanes of work in ~1.9 ns but take no
//     literals — the per-use s_mov of the basis into SGPRs costs more than the
//     packing gains — so the transform is scalar, with the basis as literals;
//   * dependent chains are what slows issue (a v_add waiting on its v_mul):
//     every stage keeps 16 independent accumulators per lane and advances
//     them together;
//   * quantisation by multiply-by-reciprocal and the 1.5*2^23 magic add, with
//     a cheap test that routes the rare near-tie samples to the IEEE divide
//     (below); K6 rounds with the same magic add;
//   * no zig-zag here: coefficients are stored in natural order (the
//     permutation is free where they are consumed/produced, K2/K5);
//   * pixels move in whole 512-byte rows: a workgroup's 64 blocks are
//     64 x 8 B of each of 8 pixel rows, loaded/stored 8 B per lane through an
//     LDS image (2-byte per-lane accesses measured ~40 % slower).
//
// Geometry: four lanes per 8x8 block, 16 blocks per wave, 64 consecutive
// blocks of one plane per 256-thread workgroup (waves never straddle planes,
// so the tables are uniform per workgroup).  Lane (b, q), q = lane & 3:
//   stage 1 owns columns 2q, 2q+1 (T[i][2q], T[i][2q+1] for i = 0..7),
//   stage 2 owns rows 2q, 2q+1    (Y[2q][v], Y[2q+1][v] for v = 0..7),
// and the 8x8 transpose between them goes through a per-block LDS tile
// (tix()).  The lane's two output rows are coefficient quads 2q, 2q+1 of the
// block (codec_common.hpp layout).  The per-quality tables (QTables) are a
// device buffer; each lane loads its 16 reciprocals / quantisers.
//
// Bit-exactness (SURVEY.md §7 hard part 1, App. C): each output is the
// reference's straight k-ascending sum of fp32-rounded products
// (DCT.cpp:232-266; stage 1 accumulates row k at a time, which is still
// k-ascending for every output); -ffp-contract=off keeps products and sums
// separately rounded (the only fma is the explicit near-tie test).
//   K1 /Q + roundf: t = y * fl(1/Q) is within |t| * 1.5 * 2^-23 of fl(y/Q)
//     (two roundings of relative error 2^-24 plus fl(y/Q)'s own), so
//     roundf(fl(y/Q)) == rint(t) unless a half-integer lies within
//     |t| * 2^-21 of t.  rint(t) comes from u = t + 1.5*2^23 (|t| < 2^22:
//     the sum rounds to an integer, half-even; its low 16 bits are the int16
//     two's complement), e = t - (u - 1.5*2^23) is exact, and the distance
//     to the nearest half-integer is 0.5 - |e|.  The lane tests
//     e*e + (W - 0.25) >= 0 with W >= 2 * Ymax * 2^-21 / Q over its 16
//     positions (QTables::near) — true whenever 0.5 - |e| <= |t| * 2^-21
//     (|t| <= Ymax / Q) — and then recomputes its outputs with the
//     reference's divide and roundf.  tests/test_numerics.py checks the rule
//     against the divide around every half-integer for every Q.
//   K6 roundf + clamp: s' = med3(s, -128, 127) then u = s' + (1.5*2^23 + 128)
//     rounds half-even to an integer whose low byte is the pixel; only exact
//     ties (|s' - rint(s')| == 0.5, where roundf goes away from zero) differ,
//     and the lane redoes those with truncf(x + copysignf(0.49999997f, x))
//     == roundf(x) (exhaustively checked for all 2^32 floats).
// No butterflies and no MFMA (an MFMA f32 product is an fma chain).
#include "codec_common.hpp"

#ifndef MYYUV_ALIAS
#define MYYUV_ALIAS 0
#endif
#ifndef MYYUV_EXP
#define MYYUV_EXP 0  // diagnostic ablations (tools/kab.sh builds); 0 = the product
#endif

namespace myyuv_gpu {

namespace {

constexpr float c_dct[64] = MYYUV_DCT_MATRIX;  // row u = basis u (DCT.cpp:221-230)
constexpr int kTile = 72;  // floats per block in the transpose tile; (i, j) at tix(i, j)
constexpr int kPix = 72;   // bytes per block in the pixel image (8 rows x 8 B + pad; 8-aligned)
constexpr float kMagic = 0x1.8p23f;             // 1.5 * 2^23
constexpr float kMagicPx = 0x1.8p23f + 128.0f;  // ... + 128: low byte = pixel
constexpr float kHalfDown = 0x1.fffffep-2f;     // largest float below 0.5

// Transpose tile: rows i = 2m, 2m+1 interleaved, so the pair a stage-2 lane
// needs, (M[2q][k], M[2q+1][k]), is one 8-byte read; block stride 72 makes
// those reads bank-conflict-free (the column-pair writes are 2-way).
__device__ __forceinline__ constexpr int tix(int i, int j) { return (i >> 1) * 18 + 2 * j + (i & 1); }

__device__ __forceinline__ uint32_t bits(float x) { return __builtin_bit_cast(uint32_t, x); }

__device__ __forceinline__ void wave_sync() { __builtin_amdgcn_wave_barrier(); }

// Keeps 16 accumulators' updates in round-robin order (the scheduler would
// otherwise serialise them chain by chain to save registers).
__device__ __forceinline__ void fence16(float (&a)[16]) {
  asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
               "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]),
               "+v"(a[12]), "+v"(a[13]), "+v"(a[14]), "+v"(a[15]));
}

// The workgroup's plane and first block.
struct Group {
  int p;           // plane (uniform)
  uint32_t first;  // local index (inside the plane) of the group's block 0
  uint32_t nb;     // blocks in the plane
};

__device__ __forceinline__ Group group_of(const FrameGeom& G) {
  Group r;
  const uint32_t w = blockIdx.x;
  r.p = w >= G.wcum[1] ? (w >= G.wcum[2] ? 2 : 1) : 0;
  r.first = (w - G.wcum[r.p]) * 64u;
  r.nb = G.cum[r.p + 1] - G.cum[r.p];
  return r;
}

// Byte offset in the frame of pixel row r of the group's block bl (bl < 64),
// or ~0u past the plane's end.
__device__ __forceinline__ uint32_t block_row_offset(const FrameGeom& G, const Group& gr, uint32_t bl,
                                                     uint32_t r) {
  const uint32_t local = gr.first + bl;
  if (local >= gr.nb) return ~0u;
  const uint32_t by = block_row(G, gr.p, local);
  const uint32_t bx = local - by * G.bw[gr.p];
  return G.poff[gr.p] + (by * 8u + r) * G.pw[gr.p] + bx * 8u;  // frames < 4 GiB
}

// Stage 2 of either transform for one lane's row pair: out[2v + h] =
// sum_k P[2k + h] * B(v, k) (h = row 2q + h), k ascending, with
// B(v, k) = D[v][k] (forward: T * D^T) or D[k][v] (inverse: U * D).
template <bool kInverse>
__device__ __forceinline__ void dot_rows(const float (&P)[16], float (&out)[16]) {
#pragma unroll
  for (int k = 0; k < 8; k++) {
    float pr[16];
#pragma unroll
    for (int v = 0; v < 8; v++) {
      const float d = c_dct[kInverse ? k * 8 + v : v * 8 + k];
      pr[2 * v] = P[2 * k] * d;
      pr[2 * v + 1] = P[2 * k + 1] * d;
    }
#pragma unroll
    for (int j = 0; j < 16; j++) out[j] = k == 0 ? pr[j] : out[j] + pr[j];
    fence16(out);
  }
}

__device__ __forceinline__ float sbyte(uint32_t w, int k) {  // byte k of w, sign-extended
  return (float)(int)(int8_t)(uint8_t)(w >> (8 * k));
}

}  // namespace

// K1: u8 planes -> int16 coefficients (natural order, quad layout).
// DCT.cpp:297-306 (gather, x - 128), :269-277 (applyDCTBlock).
__global__ __launch_bounds__(256) void k_fdct_quant(const uint8_t* __restrict__ frame, FrameGeom G,
                                                   const QTables* __restrict__ qt,
                                                   uint4* __restrict__ coef) {
  __shared__ float tile[64 * kTile];
#if MYYUV_ALIAS
  uint32_t* pix = reinterpret_cast<uint32_t*>(tile);
#else
  __shared__ uint32_t pix[64 * kPix / 4];
#endif
  const Group gr = group_of(G);
  const uint32_t t = threadIdx.x;
  const uint32_t q = t & 3u, b = t >> 2;  // quarter, block in the group
  const uint32_t local = gr.first + b;
  const bool live = local < gr.nb;
  const uint32_t g = G.cum[gr.p] + (live ? local : gr.nb - 1);

  // ---- pixel rows in: wave w loads rows w and w + 4 of the 64 blocks (8 B
  // per lane, 512 contiguous bytes per instruction within a block-row)
#pragma unroll
  for (int j = 0; j < 2; j++) {
    const uint32_t r = (t >> 6) + 4u * j, bl = t & 63u;
    const uint32_t off = block_row_offset(G, gr, bl, r);
    uint2 v = make_uint2(0x80808080u, 0x80808080u);
#if MYYUV_EXP != 2
    if (off != ~0u) v = *reinterpret_cast<const uint2*>(frame + off);
#else  // diagnostic: compute only
    v = make_uint2(off * 2654435761u, off ^ 0x5bd1e995u);
#endif
    *reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(pix) + bl * kPix + r * 8u) = v;
  }
  // reciprocals of rows 2q, 2q+1 (natural n0 .. n0 + 15), and the near-tie
  // threshold: in flight during the barrier and stage 1
  const uint32_t n0 = 16u * q;
  const float4* R4 = reinterpret_cast<const float4*>(qt->r[gr.p] + n0);
  const float4 r0 = R4[0], r1 = R4[1], r2 = R4[2], r3 = R4[3];
  const float rr[16] = {r0.x, r2.x, r0.y, r2.y, r0.z, r2.z, r0.w, r2.w,
                        r1.x, r3.x, r1.y, r3.y, r1.z, r3.z, r1.w, r3.w};  // [2v + h]
  const float nw = qt->near[gr.p][q];
  __syncthreads();

  // ---- columns 2q, 2q+1 of the block's 8 rows; x ^ 0x80 is x - 128 as a
  // signed byte (DCT.cpp:303)
  const uint8_t* pb = reinterpret_cast<const uint8_t*>(pix) + b * kPix + 2u * q;
  uint32_t xr[4];  // rows 2m (low half), 2m+1 (high half)
#pragma unroll
  for (int m = 0; m < 4; m++)
    xr[m] = (*reinterpret_cast<const uint16_t*>(pb + 16 * m) |
             ((uint32_t)*reinterpret_cast<const uint16_t*>(pb + 16 * m + 8) << 16)) ^ 0x80808080u;

#if MYYUV_EXP == 1  // diagnostic: memory only (same loads and stores, no transform)
  if (live) {
    const uint32_t h = (xr[0] ^ xr[1] ^ xr[2] ^ xr[3] ^ bits(nw) ^ bits(rr[q])) & 0x00010001u;
    const uint4 m = make_uint4(h, 0, 0, 0);  // small symbols: K2/K5 stay valid
    coef[coef_quad(g, 2 * q)] = m;
    coef[coef_quad(g, 2 * q + 1)] = m;
  }
  return;
#endif

#if MYYUV_ALIAS
  __syncthreads();  // every pixel read done before the tile is overwritten
#endif
  // ---- stage 1: T[i][j] = sum_k D[i][k] * X[k][j], j in {2q, 2q+1}
  // (squareMatrixMul<8>(DCT, X), DCT.cpp:232-242); T[2i + c] = T[i][2q + c]
  float T[16];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const float x0 = sbyte(xr[k >> 1], 2 * (k & 1)), x1 = sbyte(xr[k >> 1], 2 * (k & 1) + 1);
    float pr[16];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      pr[2 * i] = c_dct[i * 8 + k] * x0;
      pr[2 * i + 1] = c_dct[i * 8 + k] * x1;
    }
#pragma unroll
    for (int j = 0; j < 16; j++) T[j] = k == 0 ? pr[j] : T[j] + pr[j];
    fence16(T);
  }

  // ---- transpose: columns (2q, 2q+1) in, rows (2q, 2q+1) out
  float* tb = tile + b * kTile;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    tb[tix(i, 2 * q)] = T[2 * i];
    tb[tix(i, 2 * q + 1)] = T[2 * i + 1];
  }
  wave_sync();
  float P[16];  // P[2k + h] = T[2q + h][k]
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const float2 v = *reinterpret_cast<const float2*>(tb + tix(2 * q, k));
    P[2 * k] = v.x;
    P[2 * k + 1] = v.y;
  }

  // ---- stage 2: Y[i][v] = sum_k T[i][k] * D[v][k] (squareMatrixMulT<8>(T, DCT),
  // DCT.cpp:244-254); coef = (int16)roundf(Y / Q) (DCT.cpp:273-276)
  float Y[16];  // Y[2v + h] = Y[2q + h][v]
  dot_rows<false>(P, Y);
  uint32_t c[16];
  uint32_t allfar = ~0u;  // sign bit: every sample of the lane is far from a tie
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const float tq = Y[j] * rr[j];
    const float u = tq + kMagic;
    const float e = tq - (u - kMagic);
    allfar &= bits(__builtin_fmaf(e, e, nw));
    c[j] = bits(u);
  }
  if ((int)allfar >= 0) {  // a near-tie in the lane: the reference's divide for all 16
    const float* Qt = qt->q[gr.p] + n0;
#pragma unroll
    for (int j = 0; j < 16; j++) c[j] = (uint32_t)(int)roundf(Y[j] / Qt[(j >> 1) + 8 * (j & 1)]);
  }

  // ---- store rows 2q, 2q+1 = coefficient quads 2q, 2q+1 of the block
  if (live) {
    uint4 lo, hi;
    lo.x = (c[0] & 0xFFFFu) | (c[2] << 16);
    lo.y = (c[4] & 0xFFFFu) | (c[6] << 16);
    lo.z = (c[8] & 0xFFFFu) | (c[10] << 16);
    lo.w = (c[12] & 0xFFFFu) | (c[14] << 16);
    hi.x = (c[1] & 0xFFFFu) | (c[3] << 16);
    hi.y = (c[5] & 0xFFFFu) | (c[7] << 16);
    hi.z = (c[9] & 0xFFFFu) | (c[11] << 16);
    hi.w = (c[13] & 0xFFFFu) | (c[15] << 16);
    coef[coef_quad(g, 2 * q)] = lo;
    coef[coef_quad(g, 2 * q + 1)] = hi;
  }
}

// K6: int16 coefficients (natural order, quad layout) -> u8 planes.
// DCT.cpp:330-334 (dequant, squareMatrixMulT2, squareMatrixMul), :358-362
// (roundf, +128, clamp).
__global__ __launch_bounds__(256) void k_dequant_idct(const uint4* __restrict__ coef, FrameGeom G,
                                                     const QTables* __restrict__ qt,
                                                     uint8_t* __restrict__ frame) {
  __shared__ float tile[64 * kTile];
  __shared__ uint32_t pix[64 * kPix / 4];
  const Group gr = group_of(G);
  const uint32_t t = threadIdx.x;
  const uint32_t q = t & 3u, b = t >> 2;
  const uint32_t local = gr.first + b;
  const uint32_t g = G.cum[gr.p] + (local < gr.nb ? local : gr.nb - 1);
  float* tb = tile + b * kTile;

  // ---- rows 2q, 2q+1 of coefficients in (256-B runs), with the quantisers
  // of columns 2q, 2q+1
#if MYYUV_EXP == 2  // diagnostic: compute only (no coefficient loads)
  const uint32_t hh = g * 2654435761u + q;
  const uint4 a = make_uint4(hh & 0x000F000Fu, hh >> 28, 0, hh & 3), c = make_uint4(hh >> 30, 0, 0, 0);
#else
  const uint4 a = coef[coef_quad(g, 2 * q)];
  const uint4 c = coef[coef_quad(g, 2 * q + 1)];
#endif
  const float* Qt = qt->q[gr.p];
  float qk[16];  // qk[2k + h] = Q[k][2q + h]
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const float2 v = *reinterpret_cast<const float2*>(Qt + k * 8 + 2 * q);
    qk[2 * k] = v.x;
    qk[2 * k + 1] = v.y;
  }

#if MYYUV_EXP == 1  // diagnostic: memory only
  {
    const uint32_t m = a.x ^ a.y ^ a.z ^ a.w ^ c.x ^ c.y ^ c.z ^ c.w ^ bits(qk[q]);
    uint8_t* pbw = reinterpret_cast<uint8_t*>(pix) + b * kPix + 16u * q;
    *reinterpret_cast<uint2*>(pbw) = make_uint2(m, m + 1);
    *reinterpret_cast<uint2*>(pbw + 8) = make_uint2(m + 2, m + 3);
  }
#else
  // ---- through LDS: the block's int16 image (first 32 dwords of its tile),
  // then (Z[k][2q], Z[k][2q+1]) = word k*4 + q
  uint32_t* tw = reinterpret_cast<uint32_t*>(tb);
  *reinterpret_cast<uint4*>(tw + 8 * q) = a;
  *reinterpret_cast<uint4*>(tw + 8 * q + 4) = c;
  wave_sync();
  uint32_t zc[8];
#pragma unroll
  for (int k = 0; k < 8; k++) zc[k] = tw[k * 4 + q];
  wave_sync();

  // ---- dequantise (DCT.cpp:331) and stage 1: U[i][j] = sum_k D[k][i] * Z[k][j],
  // j in {2q, 2q+1} (squareMatrixMulT2<8>(DCT, Z), DCT.cpp:256-266)
  float U[16];  // U[2i + h] = U[i][2q + h]
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const float z0 = (float)(int16_t)zc[k] * qk[2 * k];
    const float z1 = (float)(int16_t)(zc[k] >> 16) * qk[2 * k + 1];
    float pr[16];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      pr[2 * i] = c_dct[k * 8 + i] * z0;
      pr[2 * i + 1] = c_dct[k * 8 + i] * z1;
    }
#pragma unroll
    for (int j = 0; j < 16; j++) U[j] = k == 0 ? pr[j] : U[j] + pr[j];
    fence16(U);
  }

  // ---- transpose (the float tile reuses the block's LDS)
#pragma unroll
  for (int i = 0; i < 8; i++) {
    tb[tix(i, 2 * q)] = U[2 * i];
    tb[tix(i, 2 * q + 1)] = U[2 * i + 1];
  }
  wave_sync();
  float P[16];  // P[2k + h] = U[2q + h][k]
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const float2 v = *reinterpret_cast<const float2*>(tb + tix(2 * q, k));
    P[2 * k] = v.x;
    P[2 * k + 1] = v.y;
  }

  // ---- stage 2: R[i][v] = sum_k U[i][k] * D[k][v] (squareMatrixMul<8>(U, DCT)),
  // then clamp(roundf(R) + 128) (DCT.cpp:358-362)
  float S[16];  // S[2v + h] = R[2q + h][v]
  dot_rows<true>(P, S);
  uint32_t px[16];  // low byte = pixel
  float mt = 0.0f;  // max |s' - rint(s')| of the lane: 0.5 means an exact tie
#pragma unroll
  for (int j = 0; j < 16; j++) {
    S[j] = __builtin_amdgcn_fmed3f(S[j], -128.0f, 127.0f);
    const float u = S[j] + kMagicPx;
    mt = __builtin_fmaxf(mt, __builtin_fabsf(S[j] - (u - kMagicPx)));
    px[j] = bits(u);
  }
  if (mt >= 0.5f) {  // an exact .5 somewhere in the lane: roundf goes away from zero
#pragma unroll
    for (int j = 0; j < 16; j++)
      px[j] = (uint32_t)((int)__builtin_truncf(S[j] + __builtin_copysignf(kHalfDown, S[j])) + 128);
  }
  // rows 2q, 2q+1 of the block into the pixel image
  {
    uint8_t* pbw = reinterpret_cast<uint8_t*>(pix) + b * kPix + 16u * q;
    *reinterpret_cast<uint2*>(pbw) =
        make_uint2((px[0] & 0xFFu) | ((px[2] & 0xFFu) << 8) | ((px[4] & 0xFFu) << 16) | (px[6] << 24),
                   (px[8] & 0xFFu) | ((px[10] & 0xFFu) << 8) | ((px[12] & 0xFFu) << 16) | (px[14] << 24));
    *reinterpret_cast<uint2*>(pbw + 8) =
        make_uint2((px[1] & 0xFFu) | ((px[3] & 0xFFu) << 8) | ((px[5] & 0xFFu) << 16) | (px[7] << 24),
                   (px[9] & 0xFFu) | ((px[11] & 0xFFu) << 8) | ((px[13] & 0xFFu) << 16) | (px[15] << 24));
  }
#endif
  __syncthreads();

  // ---- pixel rows out: wave w stores rows w and w + 4 of the 64 blocks
#pragma unroll
  for (int j = 0; j < 2; j++) {
    const uint32_t r = (t >> 6) + 4u * j, bl = t & 63u;
    const uint32_t off = block_row_offset(G, gr, bl, r);
    if (off != ~0u)
      *reinterpret_cast<uint2*>(frame + off) =
          *reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(pix) + bl * kPix + r * 8u);
  }
}

}  // namespace myyuv_gpu
