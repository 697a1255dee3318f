// k_transform.hip — K1 fdct_quant and K6 dequant_idct for gfx950.
//
// Streaming kernels: K1 reads 1 B/sample (u8 pixel) and writes 2 B/sample
// (int16 coefficient), K6 the reverse (3 B/sample each).  The
// bit-exact transform is 8 fp32 products + 7 sums per output per stage in a
// fixed order (~30 VALU per sample); at the 8 TB/s ridge the budget is ~10
// lane-ops per byte, so the arithmetic and the memory stream both set the
// pace, and the code is shaped to overlap them:
//   * persistent waves: each wave strides over 16-block units of the frame
//     and issues the NEXT unit's loads (pixel rows / coefficient quads)
//     before transforming the current one, so HBM latency hides behind the
//     wave's own arithmetic; every wave is independent (no workgroup
//     barrier; all LDS traffic is wave-local);
//   * issue rates measured on this chip (tools/ubench/valu_mix.hip,
//     profiles/r01_ubench_valu_mix.txt): independent VOP2 f32 ops with an
//     inline literal issue every ~1.0 ns per SIMD; packed v_pk_* ops do two
//     lanes of work in ~1.9 ns but take no literals, so the transform is
//     scalar with the basis as literals;
//   * dependent chains slow issue (a v_add waiting on its v_mul): every stage
//     keeps 16 independent accumulators per lane and advances them together;
//   * quantisation by multiply-by-reciprocal and the 1.5*2^23 magic add, with
//     a cheap test that routes the rare near-tie samples to the IEEE divide
//     (below); K6 rounds with the same magic add;
//   * no zig-zag here: coefficients are stored in natural order (the
//     permutation is free where they are consumed/produced, K2/K5).
//
// Geometry: four lanes per 8x8 block, 16 blocks (a "unit", never straddling
// planes, so the tables are uniform per unit) per wave.  Lane (b, q),
// q = lane & 3:
//   stage 1 owns columns 2q, 2q+1 (T[i][2q], T[i][2q+1] for i = 0..7),
//   stage 2 owns rows 2q, 2q+1    (Y[2q][v], Y[2q+1][v] for v = 0..7),
// and the 8x8 transposes (pixel rows -> columns, stage 1 -> stage 2) go
// through a per-wave LDS tile (tix()).  Lane (b, q) loads / stores the
// block's pixel rows 2q, 2q+1 directly (8 B each; 16 blocks x 8 B = 128 B
// runs per row) and its two coefficient quads 2q, 2q+1 (codec_common.hpp
// layout; 256 B runs).  The per-quality tables (QTables) are a device buffer.
// A launch covers a batch of frames (FrameGeom::nframes): the waves stride
// over the units of all of them, frame f's unit u being f * ucum[3] + u.
//
// Bit-exactness (SURVEY.md §7 hard part 1, App. C).  K1's fast path
// (fdct_fast, xform_common.hpp) is an even/odd BUTTERFLY over a nominal
// basis N (the literal DCT_matrix8 of DCT.cpp:221-230 made exactly symmetric,
// fdct_bfly.h): it does not reproduce the reference's operation order, so
// each 16-block unit carries a proof instead.  With A = sum |x - 128| over the
// block, |Y_fast - Y_ref| <= kappa * A (Higham gamma_k bounds on both
// evaluations plus max|N - D|; fdct_bfly.h), and a row whose every
// t = Y_fast * fl(1/Q) stays further than A * kb[row] from a half-integer
// quantises to the reference's roundf(fl(Y_ref / Q)).  A unit where any row
// fails is listed and recomputed by k_fdct_fix in the reference's order: the
// straight k-ascending sums of fp32-rounded products (DCT.cpp:232-266),
// -ffp-contract=off (fdct_exact; its only fma is the near-tie test below).
// tools/diag/fdct_bfly_check.cpp (tests/test_numerics.py) replays the fast
// arithmetic on the host and checks every proven unit equals the reference.
// K6 keeps the reference's order throughout.
//   exact path /Q + roundf: t = y * fl(1/Q) is within |t| * 1.5 * 2^-23 of fl(y/Q)
//     (two roundings of relative error 2^-24 plus fl(y/Q)'s own), so
//     roundf(fl(y/Q)) == rint(t) unless a half-integer lies within
//     |t| * 2^-21 of t.  rint(t) comes from u = t + 1.5*2^23 (|t| < 2^22:
//     the sum rounds to an integer, half-even; its low 16 bits are the int16
//     two's complement), e = t - (u - 1.5*2^23) is exact, and the distance
//     to the nearest half-integer is 0.5 - |e|.  Each sample's
//     x = fma(|t|, 2^-21, |e|) is >= 0.5 whenever 0.5 - |e| <= |t| * 2^-21
//     (fma rounds once and 0.5 is a float, so no near-tie is missed; exact
//     ties, where rint and roundf disagree, give x >= 0.5 too); a lane whose
//     max x reaches 0.5 recomputes its 16 outputs with the reference's divide
//     and roundf.  tools/check_numerics.c (tests/test_numerics.py) checks the
//     rule against the divide around every half-integer for every Q (a 2^-24
//     window already fails it).
//   K6 roundf + clamp: s' = med3(s, -128, 127) then u = s' + (1.5*2^23 + 128)
//     rounds half-even to an integer whose low byte is the pixel; only exact
//     ties (fract(s') == 0.5: v_fract_f32 is exact here, and a non-tie never
//     has a fractional part of exactly 0.5), where roundf goes away from zero,
//     differ, and the lane redoes those with truncf(x + copysignf(0.49999997f,
//     x)) == roundf(x) (exhaustively checked for all 2^32 floats).
// No MFMA: this is not a dense contraction, and the bound above admits only
// evaluations whose every operation rounds once to nearest.
#include <stddef.h>

#include "codec_common.hpp"
#include "xform_common.hpp"

// K1: 8 waves per SIMD (its LDS allows 8 workgroups per CU); the compiler
// otherwise settles at 69 VGPRs (7 waves) with the block-info computation
#ifndef MYYUV_K1_OCC
#define MYYUV_K1_OCC 8
#endif
#define MYYUV_K1_ATTR __attribute__((amdgpu_waves_per_eu(MYYUV_K1_OCC, MYYUV_K1_OCC)))

namespace myyuv_gpu {

using namespace xf;

// K1: u8 planes -> int16 coefficients (natural order, quad layout).
// DCT.cpp:297-306 (gather, x - 128), :269-277 (applyDCTBlock).
typedef unsigned short k1_us2 __attribute__((ext_vector_type(2)));

// Rows 2q, 2q+1 of lane (b, q)'s block (coefficient quads 2q, 2q+1), the
// block's row mask (bit c: row c has a nonzero coefficient, from the block's
// four lanes) and its K2 info word (binfo_word: row mask, msz, class, DC),
// which lets K2 classify its blocks from 4 B each instead of their rows.  An
// all-zero row is not stored (K2 reads masked-off rows from a zero buffer),
// which saves most of the 128 B per block of a q=50 frame twice (this write,
// K2's read).  Every lane still issues its four stores (the sink takes the
// skipped ones and those of lanes past the plane's end).  zq: the lane's
// eight (zig-zag index + 1) pairs, kZzPairs.v[8q .. 8q+7].
__device__ __forceinline__ void store_block_rows(const uint32_t (&c)[16], uint32_t q, uint32_t lane, bool live,
                                                 uint32_t g, uint4* dlo, uint4* dhi, uint8_t* __restrict__ rmask,
                                                 uint32_t* __restrict__ binfo, const uint4* zq,
                                                 uint4* __restrict__ sink) {
  uint4 lo, hi;
  uint32_t rm;
  pack_quads(c, q, lo, hi, rm);
  // nonzero count and msz of the lane's natural pairs 8q .. 8q+7 (lo: row
  // 2q, hi: row 2q+1) in packed 16-bit arithmetic, as K2's block_class_msz:
  // flag = min(v, 1) per half, count += flag, max of (0 - flag) & (index + 1)
  const uint4 z0 = zq[0], z1 = zq[1];
  const uint32_t wv[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  const uint32_t zv[8] = {z0.x, z0.y, z0.z, z0.w, z1.x, z1.y, z1.z, z1.w};
  k1_us2 cnt = {0, 0}, mx = {0, 0};
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint32_t fu, m16;
    asm("v_pk_min_u16 %0, %1, %2" : "=v"(fu) : "v"(wv[i]), "s"(0x00010001u));
    cnt += __builtin_bit_cast(k1_us2, fu);
    // flag * (index + 1): the indices are VGPRs here, so the packed multiply takes them
    asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(m16) : "v"(fu), "v"(zv[i]));
    mx = __builtin_elementwise_max(mx, __builtin_bit_cast(k1_us2, m16));
  }
  // the block's four lanes: counts add, msz is the maximum (one shuffle per
  // step carries both)
  uint32_t nnz = (uint32_t)cnt.x + (uint32_t)cnt.y;
  uint32_t msz = mx.x > mx.y ? (uint32_t)mx.x : (uint32_t)mx.y;
#pragma unroll
  for (int d = 1; d < 4; d <<= 1) {
    const uint32_t o = d == 1 ? quad_xor1(nnz | (msz << 16)) : quad_xor2(nnz | (msz << 16));
    nnz += o & 0xFFFFu;
    msz = max(msz, o >> 16);
  }
  const bool nzl = (rm >> (2 * q)) & 1u, nzh = (rm >> (2 * q + 1)) & 1u;
  *(live ? rmask + g : reinterpret_cast<uint8_t*>(sink + 128) + lane) = (uint8_t)rm;
  // the block's four lanes store the same word (lane 4b holds row 0: the DC
  // is the low half of its lo.x)
  const uint32_t dc = quad_lane0(lo.x);
  *(live ? binfo + g : reinterpret_cast<uint32_t*>(sink + 132) + lane) = binfo_word(rm, msz, class_of(nnz, msz), dc);
  *(nzl ? dlo : sink + lane) = lo;
  *(nzh ? dhi : sink + 64 + lane) = hi;
}

// K1's stores as buffer stores (1; 0: flat stores with per-lane pointers):
// 32-bit offsets from wave-uniform descriptors, and a store that must not
// happen (a zero row, a lane past the plane's end, a block left to the exact
// path) gets an offset past the descriptor's range, which the hardware drops.
// The flat form selects a sink pointer per store instead: two 64-bit selects
// and a 64-bit add, each a VOP3 instruction (half the issue rate of the VOP2
// forms on gfx950, tools/ubench/iforms.hip).  The launch's coefficient image
// must stay below 4 GiB (make_geom / the batch split guarantee it).
#ifndef MYYUV_K1_BUF
#define MYYUV_K1_BUF 1
#endif
typedef unsigned int k1_v4u __attribute__((ext_vector_type(4)));
constexpr uint32_t kOob = 0xFFFFFFFFu;  // a buffer offset past every range: the store is dropped

struct K1Rsrc {
  __amdgpu_buffer_rsrc_t coef, rmask, binfo;
};
// descriptors of the launch's coefficient image, row masks and block words
// (from kernel arguments only: wave-uniform)
__device__ __forceinline__ K1Rsrc k1_rsrc(uint4* coef, uint8_t* rmask, uint32_t* binfo, const FrameGeom& G) {
  const uint32_t nblk = G.cum[3] * G.nframes;
  K1Rsrc r;
  r.coef = __builtin_amdgcn_make_buffer_rsrc(coef, 0, (int)(((nblk + 63u) / 64u) * (kCoefQuadsPerWave * 16u)),
                                             0x00020000);
  r.rmask = __builtin_amdgcn_make_buffer_rsrc(rmask, 0, (int)nblk, 0x00020000);
  r.binfo = __builtin_amdgcn_make_buffer_rsrc(binfo, 0, (int)(nblk * 4u), 0x00020000);
  return r;
}

// store_block_rows through the descriptors: the same bytes, the skipped
// stores dropped by an out-of-range offset instead of a sink
__device__ __forceinline__ void store_block_rows_buf(const uint32_t (&c)[16], uint32_t q, bool live, uint32_t g,
                                                     const K1Rsrc& R, const uint4* zq) {
  uint4 lo, hi;
  uint32_t rm;
  pack_quads(c, q, lo, hi, rm);
  const uint4 z0 = zq[0], z1 = zq[1];
  const uint32_t wv[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  const uint32_t zv[8] = {z0.x, z0.y, z0.z, z0.w, z1.x, z1.y, z1.z, z1.w};
  k1_us2 cnt = {0, 0}, mx = {0, 0};
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint32_t fu, m16;
    asm("v_pk_min_u16 %0, %1, %2" : "=v"(fu) : "v"(wv[i]), "s"(0x00010001u));
    cnt += __builtin_bit_cast(k1_us2, fu);
    asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(m16) : "v"(fu), "v"(zv[i]));
    mx = __builtin_elementwise_max(mx, __builtin_bit_cast(k1_us2, m16));
  }
  uint32_t nnz = (uint32_t)cnt.x + (uint32_t)cnt.y;
  uint32_t msz = mx.x > mx.y ? (uint32_t)mx.x : (uint32_t)mx.y;
#pragma unroll
  for (int d = 1; d < 4; d <<= 1) {
    const uint32_t o = d == 1 ? quad_xor1(nnz | (msz << 16)) : quad_xor2(nnz | (msz << 16));
    nnz += o & 0xFFFFu;
    msz = max(msz, o >> 16);
  }
  const bool nzl = (rm >> (2 * q)) & 1u, nzh = (rm >> (2 * q + 1)) & 1u;
  const uint32_t dc = quad_lane0(lo.x);
  __builtin_amdgcn_raw_buffer_store_b8((uint8_t)rm, R.rmask, live ? g : kOob, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b32(binfo_word(rm, msz, class_of(nnz, msz), dc), R.binfo, live ? 4u * g : kOob,
                                        0, 0);
  const uint32_t qo = coef_quad(g, 2 * q) * 16u;  // quad 2q + 1 is 64 quads further
  __builtin_amdgcn_raw_buffer_store_b128(k1_v4u{lo.x, lo.y, lo.z, lo.w}, R.coef, live && nzl ? qo : kOob, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b128(k1_v4u{hi.x, hi.y, hi.z, hi.w}, R.coef, live && nzh ? qo + 1024u : kOob, 0,
                                         0);
}

// The zig-zag pair table in LDS (kZzPairs; before the tables' barrier)
__device__ __forceinline__ void stage_zz(uint4* szz) {
  if (threadIdx.x < 32) reinterpret_cast<uint32_t*>(szz)[threadIdx.x] = kZzPairs.v[threadIdx.x];
}

// K1's exact path out of line: a unit whose fast result is not provably the
// reference's is appended by K1 to one of kFixLists lists (unit ua to list
// ua % kFixLists, fix_count / fix_list in codec_common.hpp; each launch uses
// the counts of its parity `par`) and transformed by k_fdct_fix, which runs
// next in the stream.  Kept in K1, the exact path's code raised K1 from 64 to
// 99 VGPRs (7 -> 5 waves per SIMD) and cost it 15 % (profiles/r4g_*).  One
// count for all units serialised the appends on one address (at q90, 18 % of
// the units: 47k atomics per 8192x8192 frame, K1 83 -> 215 us); a per-wave
// register list flushed 64 at a time fixed that but cost K1 4 % at q50
// (profiles/r4r_*).

__global__ __launch_bounds__(256) MYYUV_K1_ATTR void k_fdct_quant(const uint8_t* __restrict__ frame, FrameGeom G,
                                                   const QTables* __restrict__ qt,
                                                   uint4* __restrict__ coef, uint8_t* __restrict__ rmask,
                                                   uint32_t* __restrict__ binfo, uint4* __restrict__ sink,
                                                   uint32_t* __restrict__ k2ctl, uint32_t* __restrict__ fix,
                                                   uint32_t par) {
  // K2's overflow count for the launch that follows in the stream (nullptr: none)
  if (k2ctl != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *k2ctl = 0u;
  __shared__ float tile[4][kXfUnit * kTile];
  __shared__ float sqr[kSqWords];  // QTables::q, r, kb
  __shared__ uint4 szz[8];
  static_assert(offsetof(QTables, r) == sizeof(float) * kSqR && offsetof(QTables, kb) == sizeof(float) * kSqKb,
                "layout");
  stage_zz(szz);
  stage_tables<kSqWords>(qt->q[0], sqr);
  if (kSinkSlots > 1) sink += (size_t)((blockIdx.x * 4u + (threadIdx.x >> 6)) % kSinkSlots) * kSinkQuads;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t q = lane & 3u, b = lane >> 2;  // quarter, block in the unit
  float* tb = tile[threadIdx.x >> 6] + b * kTile;
  uint8_t* img = reinterpret_cast<uint8_t*>(tb);  // the block's 8 x 8 B pixel image (aliases tb)
#if MYYUV_K1_BUF
  const K1Rsrc rs = k1_rsrc(coef, rmask, binfo, G);
#endif
  // batch units: unit u of frame f is ua = f * ucum[3] + u
  const uint32_t nall = G.ucum[3] * G.nframes, stride = unit_stride();
  uint32_t ua = first_unit();
  uint4 nx = ua < nall ? load_rows(frame, G, ua, b, q) : make_uint4(0, 0, 0, 0);
  // two stores behind the first loads, as every iteration has behind its
  // prefetch: the loop top then waits with vmcnt(2) on every path
  sink[lane] = make_uint4(0, 0, 0, 0);
  sink[64 + lane] = make_uint4(0, 0, 0, 0);
  reinterpret_cast<uint8_t*>(sink + 128)[lane] = 0;

  for (; ua < nall; ua += stride) {
    const uint32_t f = div_magic(ua, G.umag);
    const Unit U = unit_of(G, ua - f * G.ucum[3]);
    const uint32_t local = U.local0 + b;
    const bool live = local < U.nb;
    const uint32_t g = f * G.cum[3] + U.cum + local;
    // ---- this unit's rows 2q, 2q+1 into the block's image; the next unit's
    // rows in flight behind this unit's arithmetic
    *reinterpret_cast<uint2*>(img + 16u * q) = make_uint2(nx.x, nx.y);
    *reinterpret_cast<uint2*>(img + 16u * q + 8u) = make_uint2(nx.z, nx.w);
    // (the last unit reloads itself: an unconditional load keeps the
    // in-order vmcnt accounting exact, so the loop top waits for these two
    // loads only, not for the stores behind them)
    nx = load_rows(frame, G, ua + stride < nall ? ua + stride : ua, b, q);
    wave_sync();

    // stores of lanes past the plane's end, and of blocks left to the exact
    // path, go to the sink (no branch: see load_rows)
    auto store = [&](const uint32_t (&c)[16], bool keep) {
      const bool lv = live && keep;
#if MYYUV_K1_BUF
      store_block_rows_buf(c, q, lv, g, rs, szz + 2 * q);
#else
      uint4* dlo = lv ? coef + coef_quad(g, 2 * q) : sink + lane;
      uint4* dhi = lv ? coef + coef_quad(g, 2 * q + 1) : sink + 64 + lane;
      store_block_rows(c, q, lane, lv, g, dlo, dhi, rmask, binfo, szz + 2 * q, sink);
#endif
    };
    uint32_t xr[4];
    fdct_load(img, q, xr);
    const uint64_t bad = fdct_fast<true>(xr, tb, q, sqr, U.p, store);
    if (bad != 0) {  // (wave-uniform) the unproven blocks, listed by their lane 4b
      const bool mine = ((bad >> lane) & 1u) && q == 0 && live;
      const uint64_t m = __ballot(mine);
      const uint32_t c = ua % kFixLists;
      uint32_t base = 0;
      // (a launch lists each block at most once, so a count below the list's
      // capacity is guaranteed while k_fdct_fix resets the counts; the clamp
      // keeps a stale count, e.g. a diagnostic skip of the fix kernel, in bounds)
      if (lane == 0 && m != 0) base = atomicAdd(fix_count(fix, par, c), (uint32_t)__popcll(m));
      base = __builtin_amdgcn_readfirstlane(base);
      const uint32_t idx = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (mine && idx < fix_list_cap(nall)) fix_list(fix, G, c)[idx] = ua * kXfUnit + b;
    }
  }
}

// K1's exact path for the blocks K1 listed (kFixLists lists, the counts of
// parity par; entry ua * 16 + b: block slot b of unit ua): a wave takes 16
// listed blocks at a time, in any planes and frames (lane (b, q) takes
// entry b: its geometry, plane and Q tables per lane), the reference's order
// (fdct_exact), the same stores.  Wave w takes list w % kFixLists (the grid's
// waves are a multiple of kFixLists).  Workgroup 0 zeroes the other parity's
// counts, which the next K1 fills (the previous fix launch, their reader, is
// done: stream order).  Per block rather than per unit: at q90 on the bench
// frame 20 % of the units but 1.8 % of the blocks are unproven
// (tools/diag/fdct_bfly_check.cpp).
__global__ __launch_bounds__(64 * kFixWaves) void k_fdct_fix(const uint8_t* __restrict__ frame, FrameGeom G,
                                                  const QTables* __restrict__ qt, uint4* __restrict__ coef,
                                                  uint8_t* __restrict__ rmask, uint32_t* __restrict__ binfo,
                                                  uint4* __restrict__ sink,
                                                  uint32_t* __restrict__ fix, uint32_t par) {
  __shared__ float tile[kFixWaves][kXfUnit * kTile];
  __shared__ float sqr[2 * 3 * 64];
  __shared__ uint4 szz[8];
  __shared__ uint32_t s_any;
  if (blockIdx.x == 0 && threadIdx.x < kFixLists) *fix_count(fix, par ^ 1u, threadIdx.x) = 0u;
  if (threadIdx.x == 0) s_any = 0u;
  __syncthreads();
  const uint32_t gw = blockIdx.x * kFixWaves + (threadIdx.x >> 6), nw = gridDim.x * kFixWaves;
  const uint32_t c = gw % kFixLists;
  const uint32_t n = __builtin_amdgcn_readfirstlane(*fix_count(fix, par, c));
  if ((threadIdx.x & 63u) == 0 && gw / kFixLists * kXfUnit < n) s_any = 1u;
  __syncthreads();
  if (s_any == 0u) return;  // (uniform over the workgroup)
  stage_zz(szz);
#pragma unroll
  for (uint32_t i = threadIdx.x; i < 2u * 3u * 64u; i += 64u * kFixWaves) sqr[i] = qt->q[0][i];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t q = lane & 3u, b = lane >> 2;
  float* tb = tile[threadIdx.x >> 6] + b * kTile;
  uint8_t* img = reinterpret_cast<uint8_t*>(tb);
  const uint32_t* list = fix_list(fix, G, c);
#if MYYUV_K1_BUF
  const K1Rsrc rs = k1_rsrc(coef, rmask, binfo, G);
#endif
  for (uint32_t i = gw / kFixLists * kXfUnit; i < n; i += nw / kFixLists * kXfUnit) {
    // lanes past the list's end redo entry i (a real block) into the sink
    const bool real = i + b < n;
    const uint32_t ent = list[real ? i + b : i];
    const uint32_t ua = ent / kXfUnit, bb = ent % kXfUnit;
    const uint32_t f = div_magic(ua, G.umag);
    const Unit U = unit_of(G, ua - f * G.ucum[3]);
    const uint32_t g = f * G.cum[3] + U.cum + U.local0 + bb;
    const uint4 r = load_rows(frame, G, ua, bb, q);
    wave_sync();  // (the previous blocks' tile reads are done)
    *reinterpret_cast<uint2*>(img + 16u * q) = make_uint2(r.x, r.y);
    *reinterpret_cast<uint2*>(img + 16u * q + 8u) = make_uint2(r.z, r.w);
    wave_sync();
    uint32_t xr[4];
    fdct_load(img, q, xr);
#if MYYUV_K1_BUF
    fdct_exact(xr, tb, q, sqr, U.p, [&](const uint32_t (&cc)[16]) { store_block_rows_buf(cc, q, real, g, rs, szz + 2 * q); });
#else
    uint4* dlo = real ? coef + coef_quad(g, 2 * q) : sink + lane;
    uint4* dhi = real ? coef + coef_quad(g, 2 * q + 1) : sink + 64 + lane;
    fdct_exact(xr, tb, q, sqr, U.p,
               [&](const uint32_t (&cc)[16]) {
                 store_block_rows(cc, q, lane, real, g, dlo, dhi, rmask, binfo, szz + 2 * q, sink);
               });
#endif
  }
}

// K6: int16 coefficients (natural order, quad layout) -> u8 planes.
// DCT.cpp:330-334 (dequant, squareMatrixMulT2, squareMatrixMul), :358-362
// (roundf, +128, clamp).
__global__ __launch_bounds__(256) void k_dequant_idct(const uint4* __restrict__ coef,
                                                     const uint8_t* __restrict__ rmask,
                                                     const uint4* __restrict__ zq, FrameGeom G,
                                                     const QTables* __restrict__ qt,
                                                     uint8_t* __restrict__ frame, uint4* __restrict__ sink) {
  __shared__ float tile[4][kXfUnit * kTile];
  __shared__ float sq[3 * 64];  // QTables::q
  stage_tables<3 * 64>(qt->q[0], sq);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t q = lane & 3u, b = lane >> 2;
  float* tb = tile[threadIdx.x >> 6] + b * kTile;
  uint32_t* tw = reinterpret_cast<uint32_t*>(tb);  // the block's int16 image (aliases tb)
  const uint32_t nall = G.ucum[3] * G.nframes, stride = unit_stride();
  uint32_t ua = first_unit();
  uint4 na = make_uint4(0, 0, 0, 0), nc = na;
  uint32_t un = ua + stride < nall ? ua + stride : ua, nm = 0;
  if (ua < nall) {
    const uint32_t g0 = unit_block(G, ua, b);
    load_quads(coef, zq, g0, q, rmask[g0], na, nc);
    nm = rmask[unit_block(G, un, b)];
  }
  sink[lane] = make_uint4(0, 0, 0, 0);  // see K1
  sink[64 + lane] = make_uint4(0, 0, 0, 0);

  for (; ua < nall; ua += stride) {
    const uint32_t f = div_magic(ua, G.umag);
    const Unit U = unit_of(G, ua - f * G.ucum[3]);
    const uint32_t local = U.local0 + b;
    // ---- rows 2q, 2q+1 of coefficients into the block's image (first 32
    // dwords of its tile); the next unit's quads in flight
    *reinterpret_cast<uint4*>(tw + 8 * q) = na;
    *reinterpret_cast<uint4*>(tw + 8 * q + 4) = nc;
    load_quads(coef, zq, unit_block(G, un, b), q, nm, na, nc);  // unconditional: see K1
    un = un + stride < nall ? un + stride : un;
    nm = rmask[unit_block(G, un, b)];
    wave_sync();
    // (Z[k][2q], Z[k][2q+1]) = word k*4 + q
    uint32_t zc[8];
#pragma unroll
    for (int k = 0; k < 8; k++) zc[k] = tw[k * 4 + q];
    wave_sync();
    // the quantisers of columns 2q, 2q+1: qk[2k + h] = Q[k][2q + h]
    const float* Qt = sq + U.p * 64;
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
      if (!__any(zc[k] != 0u)) continue;
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
      fence16(Um);
    }

    // ---- transpose (the float tile reuses the block's LDS)
    float P[16];  // P[2k + h] = U[2q + h][k]
    transpose_tile(tb, q, Um, P);

    // ---- stage 2: R[i][v] = sum_k U[i][k] * D[k][v] (squareMatrixMul<8>(U, DCT)),
    // then clamp(roundf(R) + 128) (DCT.cpp:358-362)
    float S[16];  // S[2v + h] = R[2q + h][v]
    dot_rows<true, true>(P, S);
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
    const uint2 w0 = make_uint2(__builtin_amdgcn_perm(__builtin_amdgcn_perm(px[6], px[4], 0x0c0c0400u),
                                                      __builtin_amdgcn_perm(px[2], px[0], 0x0c0c0400u),
                                                      0x05040100u),
                                __builtin_amdgcn_perm(__builtin_amdgcn_perm(px[14], px[12], 0x0c0c0400u),
                                                      __builtin_amdgcn_perm(px[10], px[8], 0x0c0c0400u),
                                                      0x05040100u));
    const uint2 w1 = make_uint2(__builtin_amdgcn_perm(__builtin_amdgcn_perm(px[7], px[5], 0x0c0c0400u),
                                                      __builtin_amdgcn_perm(px[3], px[1], 0x0c0c0400u),
                                                      0x05040100u),
                                __builtin_amdgcn_perm(__builtin_amdgcn_perm(px[15], px[13], 0x0c0c0400u),
                                                      __builtin_amdgcn_perm(px[11], px[9], 0x0c0c0400u),
                                                      0x05040100u));
    // ---- pixel rows 2q, 2q+1 of the block out (8 B each; lanes past the
    // plane's end write the sink)
    {
      const bool live = local < U.nb;
      const uint32_t off = block_row_offset(U, live ? local : 0u, 2u * q);
      uint8_t* fr = frame + (size_t)f * G.fbytes;
      uint2* d0 = live ? reinterpret_cast<uint2*>(fr + off) : reinterpret_cast<uint2*>(sink + lane);
      uint2* d1 = live ? reinterpret_cast<uint2*>(fr + off + U.pw)
                       : reinterpret_cast<uint2*>(sink + 64 + lane);
      *d0 = w0;
      *d1 = w1;
    }
  }
}

}  // namespace myyuv_gpu
