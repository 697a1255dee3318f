// xform_common.hpp — the 8x8 block transforms of K1 (fdct_quant) and K6
// (dequant_idct), shared by k_transform.hip and the fused encoder
// (k_huff_encode.hip, k_encode_tile).  See k_transform.hip for the design and
// the bit-exactness argument (DCT.cpp:232-277, :325-335).
#pragma once
#include <stddef.h>

#include "codec_common.hpp"
#include "fdct_bfly.h"

namespace myyuv_gpu {
namespace xf {

constexpr float c_dct[64] = MYYUV_DCT_MATRIX;  // row u = basis u (DCT.cpp:221-230)
constexpr int kTile = 72;  // floats per block in the transpose tile; (i, j) at tix(i, j)
constexpr int kXfTile16 = 16 * kTile;  // a 16-block unit's tile (floats)
constexpr float kMagic = 0x1.8p23f;             // 1.5 * 2^23
constexpr float kMagicPx = 0x1.8p23f + 128.0f;  // ... + 128: low byte = pixel
constexpr float kHalfDown = 0x1.fffffep-2f;     // largest float below 0.5

// Transpose tile: rows i = 2m, 2m+1 interleaved, so the pair a stage-2 lane
// needs, (M[2q][k], M[2q+1][k]), is one 8-byte read; block stride 72 makes
// those reads bank-conflict-free (the column-pair writes are 2-way).
__device__ __forceinline__ constexpr int tix(int i, int j) { return (i >> 1) * 18 + 2 * j + (i & 1); }

__device__ __forceinline__ uint32_t bits(float x) { return __builtin_bit_cast(uint32_t, x); }

// Hand-off between a wave's lanes through LDS: a wave's LDS accesses execute
// in program order, so no wait is needed, but the compiler must not move LDS
// stores and loads across this point (wave-scope release/acquire: no
// instructions, a compiler memory barrier).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Exchanges inside a block's four lanes (a DPP quad: lanes 4b .. 4b+3).  The
// callers run with the whole wave active (K1's loop, k_fdct_fix's, the fused
// encoder's phase 1: every branch around them is wave-uniform), so every
// source lane is active.
template <int kCtrl>  // quad_perm control
__device__ __forceinline__ uint32_t quad_perm(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, kCtrl, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t quad_xor1(uint32_t v) { return quad_perm<0xB1>(v); }   // [1, 0, 3, 2]
__device__ __forceinline__ uint32_t quad_xor2(uint32_t v) { return quad_perm<0x4E>(v); }   // [2, 3, 0, 1]
__device__ __forceinline__ uint32_t quad_lane0(uint32_t v) { return quad_perm<0x00>(v); }  // [0, 0, 0, 0]

// Keeps 16 accumulators' updates in round-robin order (the scheduler would
// otherwise serialise them chain by chain to save registers).
__device__ __forceinline__ void fence16(float (&a)[16]) {
  asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
               "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]),
               "+v"(a[12]), "+v"(a[13]), "+v"(a[14]), "+v"(a[15]));
}

// A 16-block unit of one plane, with the plane's geometry (wave-uniform;
// selected from the kernel-argument fields by static index, so everything
// stays in SGPRs with no scalar loads in the loop).
struct Unit {
  int p;            // plane
  uint32_t local0;  // local index (inside the plane) of the unit's block 0
  uint32_t nb;      // blocks in the plane
  uint32_t cum;     // global index of the plane's block 0
  uint32_t poff;    // byte offset of the plane in the frame
  uint32_t pw;      // plane width (bytes per pixel row)
  uint32_t bw;      // blocks per block-row
  uint64_t bmag;    // FrameGeom::bmag of the plane
};

template <class T>
__device__ __forceinline__ T pick(bool p1, bool p2, T a0, T a1, T a2) {
  return p2 ? a2 : (p1 ? a1 : a0);
}

__device__ __forceinline__ Unit unit_of(const FrameGeom& G, uint32_t u) {
  const bool p1 = u >= G.ucum[1], p2 = u >= G.ucum[2];
  Unit r;
  r.p = p2 ? 2 : (p1 ? 1 : 0);
  r.local0 = (u - pick(p1, p2, G.ucum[0], G.ucum[1], G.ucum[2])) * kXfUnit;
  r.cum = pick(p1, p2, G.cum[0], G.cum[1], G.cum[2]);
  r.nb = pick(p1, p2, G.cum[1], G.cum[2], G.cum[3]) - r.cum;
  r.poff = pick(p1, p2, G.poff[0], G.poff[1], G.poff[2]);
  r.pw = pick(p1, p2, G.pw[0], G.pw[1], G.pw[2]);
  r.bw = pick(p1, p2, G.bw[0], G.bw[1], G.bw[2]);
  r.bmag = pick(p1, p2, G.bmag[0], G.bmag[1], G.bmag[2]);
  return r;
}

// Byte offset in the frame of pixel row r of block `local` of the unit's
// plane (block_row() with the plane's magic, codec_common.hpp).
__device__ __forceinline__ uint32_t block_row_offset(const Unit& U, uint32_t local, uint32_t r) {
  uint32_t by = local;
  if (U.bmag != 0) {
    const uint64_t lo = (uint64_t)local * (uint32_t)U.bmag;
    const uint64_t hi = (uint64_t)local * (uint32_t)(U.bmag >> 32) + (lo >> 32);
    by = (uint32_t)(hi >> 32);
  }
  const uint32_t bx = local - by * U.bw;
  return U.poff + (by * 8u + r) * U.pw + bx * 8u;  // frames < 4 GiB
}

// The wave's first unit and stride (wave-uniform, in SGPRs).
__device__ __forceinline__ uint32_t first_unit() {
  return __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
}
__device__ __forceinline__ uint32_t unit_stride() { return gridDim.x * 4u; }

// Stage 2 of either transform for one lane's row pair: out[2v + h] =
// sum_k P[2k + h] * B(v, k) (h = row 2q + h), k ascending, with
// B(v, k) = D[v][k] (forward: T * D^T) or D[k][v] (inverse: U * D).
// kSkip: a step k whose P[2k], P[2k+1] are zero in every lane of the wave is
// skipped (the sums start at +0 and a +-0 product leaves a sum unchanged, so
// the result is bit-identical; see K6).  kFence: the accumulators' updates
// kept in round-robin order (fence16); across the skip branches the fence
// pins the accumulators to registers that the two paths do not share, which
// costs a copy of them at every join (the fused decoder leaves it out).
// The fused decoder's transform runs its first kAlwaysSteps steps without the
// skip test: a 16-block unit of the bench frame needs rows / columns 0, 1, 2
// in 100 / 98 / 87-91 % of the cases, and a skip branch costs the compiler a
// copy of the 16 accumulators at its join (the +0 products of a step that
// turns out zero leave the sums unchanged, as in the skipped case).
constexpr int kAlwaysSteps = 3;
template <bool kInverse, bool kSkip = false, bool kFence = true>
__device__ __forceinline__ void dot_rows(const float (&P)[16], float (&out)[16]) {
  if (kSkip) {
#pragma unroll
    for (int j = 0; j < 16; j++) out[j] = 0.0f;
  }
#pragma unroll
  for (int k = 0; k < 8; k++) {
    if (kSkip && (kFence || k >= kAlwaysSteps) && !__any(P[2 * k] != 0.0f || P[2 * k + 1] != 0.0f)) continue;
    float pr[16];
#pragma unroll
    for (int v = 0; v < 8; v++) {
      const float d = c_dct[kInverse ? k * 8 + v : v * 8 + k];
      pr[2 * v] = P[2 * k] * d;
      pr[2 * v + 1] = P[2 * k + 1] * d;
    }
#pragma unroll
    for (int j = 0; j < 16; j++) out[j] = (k == 0 && !kSkip) ? pr[j] : out[j] + pr[j];
    if (kFence) fence16(out);
  }
}

// Column pairs (2q, 2q+1) of a block's 8x8 tile in the per-wave tile after
// stage 1, read back as row pairs (2q, 2q+1): P[2k + h] = M[2q + h][k].
__device__ __forceinline__ void transpose_tile(float* tb, uint32_t q, const float (&M)[16],
                                               float (&P)[16]) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    tb[tix(i, 2 * q)] = M[2 * i];
    tb[tix(i, 2 * q + 1)] = M[2 * i + 1];
  }
  wave_sync();
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const float2 v = *reinterpret_cast<const float2*>(tb + tix(2 * q, k));
    P[2 * k] = v.x;
    P[2 * k + 1] = v.y;
  }
}

__device__ __forceinline__ float sbyte(uint32_t w, int k) {  // byte k of w, sign-extended
  return (float)(int)(int8_t)(uint8_t)(w >> (8 * k));
}

// Pixel rows 2q, 2q+1 of the lane's block in unit u (x/y: row 2q, z/w: row
// 2q+1).  Lanes past the plane's end read the plane's last block (their
// results go to the sink): the loads are unconditional and their values are
// not touched until the next iteration, so the wave does not wait for them.
__device__ __forceinline__ uint4 load_rows(const uint8_t* __restrict__ frame, const FrameGeom& G,
                                           uint32_t ua, uint32_t b, uint32_t q) {
  const uint32_t f = div_magic(ua, G.umag);
  const Unit U = unit_of(G, ua - f * G.ucum[3]);
  const uint32_t local = U.local0 + b;
  const uint32_t off = block_row_offset(U, local < U.nb ? local : U.nb - 1, 2u * q);
  const uint8_t* fr = frame + (size_t)f * G.fbytes;
  const uint2 r0 = *reinterpret_cast<const uint2*>(fr + off);
  const uint2 r1 = *reinterpret_cast<const uint2*>(fr + off + U.pw);
  return make_uint4(r0.x, r0.y, r1.x, r1.y);
}

// The quality tables a kernel needs, staged once per workgroup into LDS.
template <int kWords>
__device__ __forceinline__ void stage_tables(const float* __restrict__ src, float* dst) {
  static_assert(kWords <= 512, "two words per thread of the 256-thread workgroup");
#pragma unroll
  for (uint32_t i = threadIdx.x; i < 512u; i += 256u)
    if (i < (uint32_t)kWords) dst[i] = src[i];
  __syncthreads();
}

__device__ __forceinline__ uint32_t unit_block(const FrameGeom& G, uint32_t ua, uint32_t b) {
  const uint32_t f = div_magic(ua, G.umag);
  const Unit U = unit_of(G, ua - f * G.ucum[3]);
  const uint32_t local = U.local0 + b;
  return f * G.cum[3] + U.cum + (local < U.nb ? local : U.nb - 1);
}

// Quads 2q, 2q+1 of block g; rows whose mask bit is clear read a zero quad
// (always issued: unconditional loads keep the vmcnt pipelining)
__device__ __forceinline__ void load_quads(const uint4* __restrict__ coef, const uint4* __restrict__ zq,
                                           uint32_t g, uint32_t q, uint32_t m, uint4& a, uint4& c) {
  const uint4* pa = (m >> (2 * q)) & 1u ? coef + coef_quad(g, 2 * q) : zq;
  const uint4* pc = (m >> (2 * q + 1)) & 1u ? coef + coef_quad(g, 2 * q + 1) : zq;
  a = *pa;
  c = *pc;
}


// Stage 1 of the forward transform for lane (b, q), the reference's order
// and roundings: T[2i + c] = T[i][2q + c] = sum_k D[i][k] * X[k][2q + c]
// (squareMatrixMul<8>(DCT, X), DCT.cpp:232-242) from the lane's pixel
// columns xr (unsigned bytes, row pairs; x - 128 as the signed byte x ^ 0x80,
// DCT.cpp:303).
__device__ __forceinline__ void fdct_stage1_exact(const uint32_t (&xr)[4], float (&T)[16]) {
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const uint32_t w = xr[k >> 1] ^ 0x80808080u;
    const float x0 = sbyte(w, 2 * (k & 1)), x1 = sbyte(w, 2 * (k & 1) + 1);
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const float d = c_dct[i * 8 + k];
      const float p0 = d * x0, p1 = d * x1;
      T[2 * i] = k == 0 ? p0 : T[2 * i] + p0;
      T[2 * i + 1] = k == 0 ? p1 : T[2 * i + 1] + p1;
    }
    fence16(T);
  }
}

// Forward transform + quantisation of lane (b, q)'s part of one block of a
// 16-block unit (K1's per-unit body, DCT.cpp:269-277, :297-306), in three
// pieces: fdct_load (the lane's pixel columns from the block's 8 x 8 B image
// img, which aliases its transpose tile tb), fdct_fast and fdct_exact.  The
// lane's 16 coefficients go to emit(c): c[2v + h] holds, in its low 16 bits,
// the int16 coefficient of row 2q + h, column v.  sqr: the Q tables, their
// reciprocals and the fast path's row bounds (QTables layout), p the plane.
//
// Fast path (round 5): both stages as even/odd butterflies over a nominal
// basis (fdct_bfly.h: 4.5 instructions per output and stage against round
// 4's 8-term FMA chains and the reference's 15 operations), then t = Y *
// fl(1/Q) rounded with the magic add.  fdct_bfly.h bounds |t - fl(Y_ref /
// Q)| by beta_h = A * kb[row] (A: the block's sum of |x - 128|); every output
// further than beta_h from the nearest half-integer rounds to the reference's
// coefficient.  If any output of the wave's unit is closer, fdct_fast emits
// nothing and returns false (wave-uniform), and the unit goes through
// fdct_exact: the reference's order, quantised as before (the near-tie lanes
// with the reference's divide).  On the bench frame (4032x3008, q=50) 14 of
// 17,766 units take the exact path (0.08 %; 20 % at q=90, 52 % at q=100;
// tools/diag/fdct_bfly_check.cpp, which also checks every passing unit
// against the reference transform).

// The lane's columns 2q, 2q+1 of the block's 8 rows, as unsigned pixels:
// xr[m] = rows 2m (low half), 2m+1 (high half).  The image may be overwritten
// after this (the wave_sync).
__device__ __forceinline__ void fdct_load(const uint8_t* img, uint32_t q, uint32_t (&xr)[4]) {
#pragma unroll
  for (int m = 0; m < 4; m++)
    xr[m] = *reinterpret_cast<const uint16_t*>(img + 16 * m + 2 * q) |
            ((uint32_t)*reinterpret_cast<const uint16_t*>(img + 16 * m + 8 + 2 * q) << 16);
  wave_sync();
}

// QTables offsets in the staged LDS copy (sqr): q, r, kb
constexpr int kSqR = 3 * 64, kSqKb = 2 * 3 * 64, kSqWords = 2 * 3 * 64 + 3 * 8;

// Returns 0 when every output of the unit is proven (all emitted), else the
// ballot of the lanes whose BLOCK has an unproven output: with kPerBlock the
// proven blocks are emitted (emit(c, keep): keep false for the others, whose
// lanes must store nothing), without it nothing is emitted.
template <bool kPerBlock, class Emit>
__device__ __forceinline__ uint64_t fdct_fast(const uint32_t (&xr)[4], float* tb, uint32_t q, const float* sqr, int p,
                                              Emit&& emit) {
  // ---- A = sum |x - 128| over the block (exact: byte SADs against 128, the
  // block's four lanes summed)
  uint32_t a = 0;
#pragma unroll
  for (int m = 0; m < 4; m++) a = __builtin_amdgcn_sad_u8(xr[m], 0x80808080u, a);
  a += quad_xor1(a);
  a += quad_xor2(a);
  // ---- stage 1: the lane's two columns (exact integer butterflies, then
  // the basis products), T[2i + c] = T[i][2q + c]
  float T[16];
#pragma unroll
  for (int c = 0; c < 2; c++) {
    float px[8], t[8];
#pragma unroll
    for (int m = 0; m < 8; m++) px[m] = (float)((xr[m >> 1] >> (8 * (2 * (m & 1) + c))) & 0xFFu);
    myyuv_bfly::bfly_cols(px, t);
#pragma unroll
    for (int i = 0; i < 8; i++) T[2 * i + c] = t[i];
  }
  float P[16];  // P[2k + h] = T[2q + h][k]
  transpose_tile(tb, q, T, P);
  // ---- stage 2: the lane's two rows, each quantised as it is done:
  // coef = (int16)roundf(Y / Q) (DCT.cpp:273-276) as rint(Y * fl(1/Q)) where
  // no output lies within beta_h of a half-integer
  const float af = (float)a;
  const float* Rq = sqr + kSqR + p * 64 + 16u * q;  // reciprocals of rows 2q, 2q+1
  uint32_t c[16];
  float mx = 0.0f;  // max over the lane's rows of max |e| + beta_h: >= 0.5 when an output may round otherwise
#pragma unroll
  for (int h = 0; h < 2; h++) {
    float x[8], y[8];
#pragma unroll
    for (int k = 0; k < 8; k++) x[k] = P[2 * k + h];
    myyuv_bfly::bfly_rows(x, y);
    float em = 0.0f;
#pragma unroll
    for (int v = 0; v < 8; v++) {
      const float t = y[v] * Rq[8 * h + v];
      const float u = t + kMagic;
      const float e = t - (u - kMagic);
      em = __builtin_fmaxf(em, __builtin_fabsf(e));
      c[2 * v + h] = bits(u);
    }
    mx = __builtin_fmaxf(mx, __builtin_fmaf(af, sqr[kSqKb + p * 8 + 2 * q + h], em));
  }
  const uint64_t bad = __builtin_amdgcn_ballot_w64(mx >= 0.5f);
  if (bad == 0) {
    emit(c, true);  // every output clears the bound: its rounded t is the reference's coefficient
    return 0;
  }
  if (!kPerBlock) return bad;
  // (bad != 0 is wave-uniform: the whole wave runs the quad exchanges) a
  // block is unproven when any of its four lanes is; the bound is per block
  // (A and the row factors are the block's own), so the other blocks' outputs
  // are the reference's
  uint32_t fb = mx >= 0.5f ? 1u : 0u;
  fb |= quad_xor1(fb);
  fb |= quad_xor2(fb);
  emit(c, fb == 0u);
  return __builtin_amdgcn_ballot_w64(fb != 0u);
}

// The unit in the reference's order (the tile tb is rewritten: callers
// wave_sync between a fast attempt and this).
template <class Emit>
__device__ __forceinline__ void fdct_exact(const uint32_t (&xr)[4], float* tb, uint32_t q, const float* sqr, int p,
                                           Emit&& emit) {
  const uint32_t n0 = 16u * q;
  float T[16];
  fdct_stage1_exact(xr, T);
  float P[16];  // P[2k + h] = T[2q + h][k]
  transpose_tile(tb, q, T, P);
  float Y[16];  // Y[2v + h] = Y[2q + h][v]
  dot_rows<false>(P, Y);
  // reciprocals of rows 2q, 2q+1 (natural n0 .. n0 + 15)
  const float4* R4 = reinterpret_cast<const float4*>(sqr + kSqR + p * 64 + n0);
  const float4 r0 = R4[0], r1 = R4[1], r2 = R4[2], r3 = R4[3];
  const float rr[16] = {r0.x, r2.x, r0.y, r2.y, r0.z, r2.z, r0.w, r2.w,
                        r1.x, r3.x, r1.y, r3.y, r1.z, r3.z, r1.w, r3.w};  // [2v + h]
  uint32_t c[16];
  float mx = 0.0f;  // max over the lane of |e| + |t| * 2^-21: >= 0.5 near a tie
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const float tq = Y[j] * rr[j];
    const float uu = tq + kMagic;
    const float e = tq - (uu - kMagic);
    mx = __builtin_fmaxf(mx, __builtin_fmaf(__builtin_fabsf(tq), kNearRel, __builtin_fabsf(e)));
    c[j] = bits(uu);
  }
  if (mx >= 0.5f) {  // a near-tie in the lane: the reference's divide for all 16
    const float* Qt = sqr + p * 64 + n0;
#pragma unroll
    for (int j = 0; j < 16; j++) c[j] = (uint32_t)(int)roundf(Y[j] / Qt[(j >> 1) + 8 * (j & 1)]);
  }
  emit(c);
}

// Both in one pass (the fused encoder): the fast path, else the exact one.
template <class Emit>
__device__ __forceinline__ void fdct_core(const uint8_t* img, float* tb, uint32_t q, const float* sqr, int p,
                                          Emit&& emit) {
  uint32_t xr[4];
  fdct_load(img, q, xr);
  if (__builtin_expect(fdct_fast<false>(xr, tb, q, sqr, p, emit) != 0, 0)) {
    wave_sync();
    fdct_exact(xr, tb, q, sqr, p, [&](const uint32_t (&c)[16]) { emit(c, true); });
  }
}

// Rows 2q, 2q+1 of the block as two coefficient quads (codec_common.hpp
// layout) and the block's row mask (bit c: row c has a nonzero coefficient),
// from its four lanes (lanes 4b .. 4b+3 of the wave).
__device__ __forceinline__ void pack_quads(const uint32_t (&c)[16], uint32_t q, uint4& lo, uint4& hi,
                                           uint32_t& rm) {
  lo.x = __builtin_amdgcn_perm(c[2], c[0], 0x05040100u);
  lo.y = __builtin_amdgcn_perm(c[6], c[4], 0x05040100u);
  lo.z = __builtin_amdgcn_perm(c[10], c[8], 0x05040100u);
  lo.w = __builtin_amdgcn_perm(c[14], c[12], 0x05040100u);
  hi.x = __builtin_amdgcn_perm(c[3], c[1], 0x05040100u);
  hi.y = __builtin_amdgcn_perm(c[7], c[5], 0x05040100u);
  hi.z = __builtin_amdgcn_perm(c[11], c[9], 0x05040100u);
  hi.w = __builtin_amdgcn_perm(c[15], c[13], 0x05040100u);
  const bool nzl = (lo.x | lo.y | lo.z | lo.w) != 0u, nzh = (hi.x | hi.y | hi.z | hi.w) != 0u;
  rm = (nzl ? 1u << (2 * q) : 0u) | (nzh ? 2u << (2 * q) : 0u);
  rm |= quad_xor1(rm);
  rm |= quad_xor2(rm);
}

// K6's body for lane (b, q) of a 16-block unit (DCT.cpp:325-335, :358-362):
// the block's int16 coefficient image (natural order, word w = coefficients
// 2w, 2w+1) is the first 32 dwords of its transpose tile tb; Qt: the plane's
// Q table (natural order).  Out: pixel rows 2q (w0) and 2q+1 (w1), 8 bytes
// each.  Shared by k_dequant_idct and the fused decoder (k_decode_idct).
// The int16 image of block slot b sits at word img_word(b) of its tile
// region (the float tile at word 0): slots b and b + 4 of a 32-lane group
// then start on different banks (72 b mod 32 repeats every 4 slots), so the
// image's 16-B writes and idct_rows' word reads are conflict-free.
__device__ __forceinline__ constexpr uint32_t img_word(uint32_t b) { return 4u * ((b >> 2) & 1u); }

__device__ __forceinline__ void idct_rows(float* tb, uint32_t q, uint32_t b, const float* Qt, uint2& w0,
                                          uint2& w1) {
  const uint32_t* tw = reinterpret_cast<const uint32_t*>(tb) + img_word(b);
  // (Z[k][2q], Z[k][2q+1]) = word k*4 + q
  uint32_t zc[8];
#pragma unroll
  for (int k = 0; k < 8; k++) zc[k] = tw[k * 4 + q];
  wave_sync();
  // the quantisers of columns 2q, 2q+1: qk[2k + h] = Q[k][2q + h]
  float qk[16];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const float2 v = *reinterpret_cast<const float2*>(Qt + k * 8 + 2 * q);
    qk[2 * k] = v.x;
    qk[2 * k + 1] = v.y;
  }

  // ---- dequantise (DCT.cpp:331) and stage 1: U[i][j] = sum_k D[k][i] * Z[k][j],
  // j in {2q, 2q+1} (squareMatrixMulT2<8>(DCT, Z), DCT.cpp:256-266)
  // Quantised blocks are sparse: a coefficient row k that is zero in all 16
  // blocks of the unit (61 % of the (unit, k) pairs of the bench frame)
  // contributes only +-0 products, and a sum that starts at +0 (as the
  // reference's does, DCT.cpp:259-263) is unchanged by them — so the wave
  // skips that step outright, bit-exactly.  Stage 2 skips the zero columns
  // of Z the same way (U's column k is zero exactly when Z's is).
  float Um[16];  // Um[2i + h] = U[i][2q + h]
#pragma unroll
  for (int j = 0; j < 16; j++) Um[j] = 0.0f;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    if (k >= kAlwaysSteps && !__any(zc[k] != 0u)) continue;
    const float z0 = (float)(int16_t)zc[k] * qk[2 * k];
    const float z1 = (float)(int16_t)(zc[k] >> 16) * qk[2 * k + 1];
    float pr[16];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      pr[2 * i] = c_dct[k * 8 + i] * z0;
      pr[2 * i + 1] = c_dct[k * 8 + i] * z1;
    }
#pragma unroll
    for (int j = 0; j < 16; j++) Um[j] = Um[j] + pr[j];
    // (no fence16 here: across the skip branches it costs a copy of the
    // accumulators at every join, see dot_rows)
  }

  // ---- transpose (the float tile reuses the block's LDS)
  float P[16];  // P[2k + h] = U[2q + h][k]
  transpose_tile(tb, q, Um, P);

  // ---- stage 2: R[i][v] = sum_k U[i][k] * D[k][v] (squareMatrixMul<8>(U, DCT)),
  // then clamp(roundf(R) + 128) (DCT.cpp:358-362)
  float S[16];  // S[2v + h] = R[2q + h][v]
  dot_rows<true, true, false>(P, S);
  uint32_t px[16];  // low byte = pixel
  bool tie = false;  // an exact .5 in the lane: fract(s') == 0.5 (exact for |s'| <= 128)
#pragma unroll
  for (int j = 0; j < 16; j++) {
    S[j] = __builtin_amdgcn_fmed3f(S[j], -128.0f, 127.0f);
    const float uu = S[j] + kMagicPx;
    tie = tie || __builtin_amdgcn_fractf(S[j]) == 0.5f;
    px[j] = bits(uu);
  }
  if (tie) {  // an exact .5 somewhere in the lane: roundf goes away from zero
#pragma unroll
    for (int j = 0; j < 16; j++)
      px[j] = (uint32_t)((int)__builtin_truncf(S[j] + __builtin_copysignf(kHalfDown, S[j])) + 128);
  }
  // rows 2q (even j) and 2q+1 (odd j): bytes v = 0..7 of each
  w0 = make_uint2(__builtin_amdgcn_perm(__builtin_amdgcn_perm(px[6], px[4], 0x0c0c0400u),
                                                    __builtin_amdgcn_perm(px[2], px[0], 0x0c0c0400u),
                                                    0x05040100u),
                              __builtin_amdgcn_perm(__builtin_amdgcn_perm(px[14], px[12], 0x0c0c0400u),
                                                    __builtin_amdgcn_perm(px[10], px[8], 0x0c0c0400u),
                                                    0x05040100u));
  w1 = make_uint2(__builtin_amdgcn_perm(__builtin_amdgcn_perm(px[7], px[5], 0x0c0c0400u),
                                                    __builtin_amdgcn_perm(px[3], px[1], 0x0c0c0400u),
                                                    0x05040100u),
                              __builtin_amdgcn_perm(__builtin_amdgcn_perm(px[15], px[13], 0x0c0c0400u),
                                                    __builtin_amdgcn_perm(px[11], px[9], 0x0c0c0400u),
                                                    0x05040100u));
}

// The same transform on 8-block units, eight lanes per block (the fused
// decoder's last 1-8 blocks of a group): lane (b, r) computes column r of U
// in stage 1 and row r of R in stage 2, one pixel row per lane.  A step costs
// 8 products and sums per lane instead of 16, so the last unit of a group
// costs about two thirds of a 16-block one when it has 8 blocks or fewer
// (half the VALU, the same LDS round trips).  All-8-block units measured
// slower: 4.2 units per 64-block group instead of 2.3 (16.3 + 15.8 steps
// instead of 10.0 + 9.6, tools/diag/idct_units.py), and each unit's fixed
// round trips outweigh the halved steps (transform phase +22 %,
// profiles/r5ai_*).  Slot b's region: kTile8 floats, its int16 image
// (natural order) at word 0, the float tile over it after the image is read;
// row stride 8, slot stride 72 (= 8 mod 32: the column writes of four slots
// fall on distinct banks).  qc[k] = Q[k][r].
constexpr int kTile8 = 72;
#ifndef MYYUV_ALWAYS8
#define MYYUV_ALWAYS8 2
#endif
constexpr int kAlways8 = MYYUV_ALWAYS8;  // steps run without the skip test (row / column 0, 1: 100 / 97 % of the units)
__device__ __forceinline__ uint2 idct_row8(float* tb, uint32_t r, const float (&qc)[8]) {
  const int16_t* im = reinterpret_cast<const int16_t*>(tb);
  int zk[8];  // Z[k][r]
#pragma unroll
  for (int k = 0; k < 8; k++) zk[k] = im[8 * k + r];
  wave_sync();
  // ---- dequantise (DCT.cpp:331) and stage 1, U[i][r] = sum_k D[k][i] * Z[k][r]
  // (squareMatrixMulT2<8>(DCT, Z), DCT.cpp:256-266), k ascending; a row k
  // that is zero in every block of the unit adds only +-0 products to sums
  // that start at +0, so the wave skips it (bit-exact, see idct_rows)
  float Um[8];
#pragma unroll
  for (int i = 0; i < 8; i++) Um[i] = 0.0f;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    if (k >= kAlways8 && !__any(zk[k] != 0)) continue;
    const float z = (float)zk[k] * qc[k];
#pragma unroll
    for (int i = 0; i < 8; i++) Um[i] = Um[i] + c_dct[k * 8 + i] * z;
  }
  // ---- transpose through the slot's tile: column r out, row r back
#pragma unroll
  for (int i = 0; i < 8; i++) tb[8 * i + r] = Um[i];
  wave_sync();
  const float4 p0 = *reinterpret_cast<const float4*>(tb + 8 * r);
  const float4 p1 = *reinterpret_cast<const float4*>(tb + 8 * r + 4);
  const float P[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};  // U[r][k]
  // ---- stage 2: R[r][v] = sum_k U[r][k] * D[k][v] (squareMatrixMul<8>(U, DCT)),
  // skipping the columns that are zero in every block, then
  // clamp(roundf(R) + 128) (DCT.cpp:358-362)
  float S[8];
#pragma unroll
  for (int v = 0; v < 8; v++) S[v] = 0.0f;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    if (k >= kAlways8 && !__any(P[k] != 0.0f)) continue;
#pragma unroll
    for (int v = 0; v < 8; v++) S[v] = S[v] + P[k] * c_dct[k * 8 + v];
  }
  uint32_t px[8];
  bool tie = false;
#pragma unroll
  for (int v = 0; v < 8; v++) {
    S[v] = __builtin_amdgcn_fmed3f(S[v], -128.0f, 127.0f);
    tie = tie || __builtin_amdgcn_fractf(S[v]) == 0.5f;
    px[v] = bits(S[v] + kMagicPx);
  }
  if (tie) {
#pragma unroll
    for (int v = 0; v < 8; v++)
      px[v] = (uint32_t)((int)__builtin_truncf(S[v] + __builtin_copysignf(kHalfDown, S[v])) + 128);
  }
  return make_uint2(__builtin_amdgcn_perm(__builtin_amdgcn_perm(px[3], px[2], 0x0c0c0400u),
                                          __builtin_amdgcn_perm(px[1], px[0], 0x0c0c0400u), 0x05040100u),
                    __builtin_amdgcn_perm(__builtin_amdgcn_perm(px[7], px[6], 0x0c0c0400u),
                                          __builtin_amdgcn_perm(px[5], px[4], 0x0c0c0400u), 0x05040100u));
}

}  // namespace xf
}  // namespace myyuv_gpu
