// k_huff_decode.hip — K5: per-block chunk parse + canonical Huffman decode on
// gfx950 (Huffman::fromDump, unpack11bit, decodeSymbol, decodeFromTreeData;
// myyuv_DCT/Huffman.cpp:243-277, :54-69, :106-154).
//
// One workgroup = one wave = up to 64 consecutive blocks of ONE plane, so the
// wave's chunks are one contiguous byte range of the plane's content[]; it is
// staged into LDS with 16-B loads issued together (the LDS image keeps the
// stream's 16-B grid; several rounds when it exceeds the 6 KiB stage), then
// each lane decodes its own block:
//   1. header: u16 nbits, u8 table_bytes;
//   2. table: one pass over the groups ((L-1)<<5 | (n-1)) + n x 11-bit values,
//      recording per length the code count and the bit address of its group.
//      No symbol table is unpacked: a decoded code's value is read in place
//      (11 bits at group_bit + 11 * rank), so the wave needs no LDS beyond
//      the stage;
//   3. symbols: the reference decodes bit-serially (puff style): at length L,
//      code = first L bits, match if code < first + count[L].  Here the next 8
//      bits are peeked from a 64-bit register window (refilled from LDS every
//      7 symbols, at most 56 bits apart) and:
//        * "regular" tables (every length in one group, first + count[L] <=
//          2^L: every table the reference writes) — the match conditions are
//          w8 < lim[L] with left-justified limits lim[L] = (first + count) <<
//          (8 - L), non-decreasing in L, so the matched length is 1 + #{L :
//          w8 >= lim[L]}: eight 16-bit compares in four SWAR subtractions;
//        * any other table (malformed or hand-made streams) — the bit-serial
//          conditions evaluated for L = 1..8 as the reference does (uint8
//          arithmetic of `first` kept), the value found by walking the groups
//          of that length in stream order (std::map<len, vector> append
//          semantics of tree_data).
//      Both give the reference's "bad code" / "unknown symbol" outcomes on
//      the same bit budget checks.
//   The symbol loop is unrolled over the 64 scan positions, so each decoded
//   value lands in a statically indexed register of the block's NATURAL-order
//   words (the de-zig-zag of Huffman.cpp:148-153 is free) and the block is
//   written as 8 quads of the codec_common.hpp layout that K6 reads.
#include "codec_common.hpp"
#include "k_stream.hpp"
#include "xform_common.hpp"

namespace myyuv_gpu {

namespace {

// 5 KiB stage: 80 B of chunk per block on average (a 4K frame at q=50 uses
// ~12 B); a wave whose chunks do not fit is staged in several rounds.
constexpr uint32_t kStageQuads = 320;
// One zero quad after the stage (zeroed at kernel start, never staged into):
// the symbol loop reads a lane's value from it when the lane takes none, so
// the value needs no select.
constexpr uint32_t kZeroBit = kStageQuads * 128u;
// after the zero quad: the table parse's per-lane value positions, 8 u32 per
// lane, length-major (decode_regular reads one per symbol, conflict-free:
// an LDS read instead of a select between 64-bit register pairs, a 64-bit
// shift and an add)
constexpr uint32_t kGposQuads = 8 * 64 * 4 / 16;

#ifndef MYYUV_K5_GROUP
#define MYYUV_K5_GROUP 2  // positions per "any lane left" test (1 / 2 / 4 / 8: 132.4 / 128.2 / 129.0 / 135.1 us per launch, tools/runs/r3n.sh)
#endif
// The symbol loop's arithmetic in full-rate forms (1; 0: as the compiler
// picks them): the value's stage bit by a 24-bit multiply-add (the code has
// at most 8 bits; written as a 32-bit product the compiler emits the 64-bit
// v_mad_u64_u32), and the message's bit count as a register of its own
// (left packed with the table size, every comparison with it is an SDWA
// form)
#ifndef MYYUV_K5_FORMS
#define MYYUV_K5_FORMS 1
#endif
#ifndef MYYUV_K5S_WAVES
#define MYYUV_K5S_WAVES 5  // the split decoder's K5
#endif
#ifndef MYYUV_K5_WAVES
#define MYYUV_K5_WAVES 5
#endif



struct ZzTable {
  uint8_t v[64];
  constexpr ZzTable() : v{} {
    constexpr uint8_t zz[64] = MYYUV_ZIGZAG;
    for (int i = 0; i < 64; i++) v[i] = zz[i];
  }
};
constexpr ZzTable kZz{};
constexpr const uint8_t* c_zz = kZz.v;
__constant__ uint8_t c_zz_dev[64] = MYYUV_ZIGZAG;

__device__ __forceinline__ void record_error(unsigned long long* err, uint64_t key, int code) {
  atomicMin(err, (unsigned long long)((key << 8) | (uint64_t)code));
}


// Inclusive sum over the wave's 64 lanes by DPP (rows of 16 by row_shr 1, 2,
// 4, 8, then row_bcast 15 / 31 across rows; lanes whose source is out of
// range add the old value 0).  Every lane must be active: under a partial
// EXEC, inactive lanes pass nothing on (the DPP rule).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return x;
}

__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t s) {
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (s & 31));
}

// One lane's chunk in the LDS stage (b0: its first byte).  Bits are in the
// stream's order: bit k of the chunk is bit k & 7 of byte k >> 3.
struct LdsChunk {
  const uint32_t* st;
  uint32_t b0;
  __device__ __forceinline__ uint32_t byte(uint32_t i) const {
    return reinterpret_cast<const uint8_t*>(st)[b0 + i];
  }
  __device__ __forceinline__ uint32_t bits32(uint32_t bit) const {
    const uint32_t P = 8 * b0 + bit, w = P >> 5;
    return funnel(st[w + 1], st[w], P);
  }
};

struct Table {
  uint32_t nbits = 0;   // symbol bits
  uint32_t sbit = 0;    // chunk bit of the first symbol bit
  uint32_t tb = 0;      // table bytes
  uint64_t cnt = 0;     // code count of length L in byte L-1
  uint32_t lim[4] = {0, 0, 0, 0};   // 16-bit fields: left-justified limit, lengths 2k+1, 2k+2
  bool regular = true;
};

// Header + table (Huffman::fromDump, Huffman.cpp:243-277).  Returns 0 or the
// MYYUV_E_* code (12: bad chunk).
template <class Chunk>
__device__ __forceinline__ int parse_table(const Chunk& c, uint32_t s, Table& T, uint32_t* gcol) {
  // (no early returns: a bad header only sets `bad`, and the walk and the
  // per-length pass run on whatever was read (inside the stage); each return
  // path would otherwise re-initialise the outputs at its branch level)
  // the chunk's first 20 bytes in registers, loaded together: the group walk
  // below is a chain of dependent byte reads, from registers for every table
  // that ends within them (at most 8 symbols always do), from LDS for the
  // rest in a second walk; both walks branch-free (a dynamic byte index as a
  // select chain compiled to nested EXEC branches, ~90 instructions a group)
  // (five named values, not an array: selects between an array's elements
  // are turned into a dynamically indexed scratch array)
  const uint32_t h0 = c.bits32(0), h1 = c.bits32(32), h2 = c.bits32(64), h3 = c.bits32(96), h4 = c.bits32(128);
  const uint32_t nbits = h0 & 0xFFFFu;
  const uint32_t tb = (h0 >> 16) & 0xFFu;
  const bool bad_hdr = s < 3 || nbits > 512 || 3 + tb + (nbits + 7) / 8 > s;
  auto reg_byte = [=](uint32_t i) -> uint32_t {  // i < 20
    const uint32_t k = i >> 2;
    const uint32_t w01 = (k & 1u) ? h1 : h0;
    const uint32_t w23 = (k & 1u) ? h3 : h2;
    const uint32_t w = k >= 4u ? h4 : ((k & 2u) ? w23 : w01);
    return (w >> (8u * (i & 3u))) & 0xFFu;
  };
  uint64_t cnt = 0, glo = 0, ghi = 0;
  uint32_t seen = 0, total = 0, i = 3;
  bool regular = true, bad = bad_hdr;
  auto group = [&](uint32_t info) {  // the group whose info byte is at i
    const uint32_t L = (info >> 5) + 1, n = (info & 31) + 1;
    const uint32_t nbytes = (n * 11 + 7) / 8;
    total += n;
    bad = bad || i + 1 + nbytes > 3 + tb || total > 64;
    cnt += (uint64_t)n << (8 * (L - 1));
    regular = regular && !(seen & (1u << L));
    seen |= 1u << L;
    const uint64_t gb = (uint64_t)(8 * (i + 1)) << (16 * ((L - 1) & 3));
    glo |= L <= 4 ? gb : 0ull;
    ghi |= L <= 4 ? 0ull : gb;
    i += 1 + nbytes;
  };
  if (3 + tb <= 20) {
    while (i - 3 < tb && !bad) group(reg_byte(i));
  } else {
    while (i - 3 < tb && !bad) group(c.byte(i));
  }
  uint32_t F = 0;
#pragma unroll
  for (int L = 0; L < 8; L++) {  // length L + 1
    const uint32_t cL = (uint32_t)(cnt >> (8 * L)) & 0xFF;
    if (F + cL > (2u << L)) regular = false;
    const uint32_t lim = ((F + cL) << (7 - L)) & 0xFFFF;
    const uint32_t gb = (uint32_t)((L < 4 ? glo : ghi) >> (16 * (L & 3))) & 0xFFFF;
    T.lim[L >> 1] |= lim << (16 * (L & 1));
    gcol[64 * L] = 8 * c.b0 + gb - 11 * F;  // (mod 2^32: the first value's stage bit is 8 b0 + gb)
    F = (F + cL) << 1;
  }
  uint32_t nb = nbits;
#if MYYUV_K5_FORMS
  asm volatile("" : "+v"(nb));  // (materialised: no WORD_0 selects on h0 in the symbol loop)
#endif
  T.nbits = nb;
  T.sbit = 8 * (3 + tb);
  T.tb = tb;
  T.cnt = cnt;
  T.regular = regular;
  return bad ? 12 : 0;
}

// Symbols of REGULAR tables (Huffman.cpp:106-154) into nw (natural-order
// int16 pairs, zeroed by the caller).  Returns true for an `act` lane whose
// message fails (no code matches, or a code runs past nbits): the caller
// re-decodes that block with decode_general, which gives the reference's
// exact outcome (10 bad code / 11 unknown symbol) — regular tables decode
// identically on both paths, so only the error code is taken from it.
//
// Fully unrolled over the 64 scan positions (each value lands in a statically
// indexed register), with a uniform "any lane left" exit before every
// position; the body is straight-line (state updates by select: divergent
// branches make the compiler shuffle the whole nw[] array at every join).
// A lane's state after it stops (bp, window) is dead, so it advances
// unconditionally; only the value store is predicated.  The 64-bit window is
// rebuilt every 7 positions (at most 56 bits consumed) from three stage
// words.  Per position: the length by SWAR compares, the value's 11 bits read
// in place from the table (group bit + 11 * rank), one predicated OR.
// (Prefetching the stage words a few positions ahead, or deferring each value
// read by one position, measured no faster on MI355X, and with the loads
// three positions ahead the decoded values came out wrong nondeterministically
// in long straight-line groups: both are deliberately not done.)
__device__ __forceinline__ bool decode_regular(const LdsChunk& c, const Table& T, const uint32_t* gcol, bool act,
                                               uint32_t (&nw)[32]) {
  bool bad = false;
  uint32_t bp = 0;
  uint64_t rwin = 0;  // MSB-first window: the next symbol's first bit at bit 63
  act = act && T.nbits > 0;
  const uint32_t P0 = 8 * c.b0 + T.sbit;  // stage bit of the first symbol bit
#pragma unroll
  for (int j0 = 0; j0 < 64; j0 += MYYUV_K5_GROUP) {
    if (__ballot(act) == 0) continue;
#pragma unroll
  for (int j = j0; j < j0 + MYYUV_K5_GROUP; j++) {
    if (j % 7 == 0) {
      const uint32_t P = act ? P0 + bp : P0, w = P >> 5;
      const uint32_t q0 = c.st[w], q1 = c.st[w + 1], q2 = c.st[w + 2];
      rwin = ((uint64_t)__brev(funnel(q1, q0, P)) << 32) | __brev(funnel(q2, q1, P));
    }
    const uint32_t w8 = (uint32_t)(rwin >> 56);  // next 8 bits, MSB-first
    // matched length - 1 = #{L : w8 >= lim[L]} (eight 16-bit fields)
    const uint32_t W = w8 * 0x10001u | 0x80008000u;
    const uint32_t n = __popc((W - T.lim[0]) & 0x80008000u) + __popc((W - T.lim[1]) & 0x80008000u) +
                       __popc((W - T.lim[2]) & 0x80008000u) + __popc((W - T.lim[3]) & 0x80008000u);
    const uint32_t bpn = bp + n + 1;
    const bool ok = n < 8 && bpn <= T.nbits;
    bad = bad || (act && !ok);
    const bool take = act && ok;
    // the value: the code's n + 1 bits times 11 plus length n + 1's entry of
    // the lane's column of the LDS table, the stage bit of its length's first
    // value less 11 times its first code (n = 8, no match: not taken)
    const uint32_t G = gcol[64 * (n & 7u)];
#if MYYUV_K5_FORMS
    uint32_t vbit;  // (code < 2^8: v_mad_u32_u24; the compiler turns a 32-bit product + G into v_mad_u64_u32)
    asm("v_mad_u32_u24 %0, %1, 11, %2" : "=v"(vbit) : "v"((uint32_t)(rwin >> 32) >> ((31u - n) & 31u)), "v"(G));
#else
    const uint32_t vbit = ((uint32_t)(rwin >> 32) >> ((31u - n) & 31u)) * 11u + G;
#endif
    const uint32_t P = take ? vbit : kZeroBit, w = P >> 5;  // (stage bits; kZeroBit: the zero quad)
    const uint32_t raw = funnel(c.st[w + 1], c.st[w], P);
    const uint32_t v = (uint32_t)(((int32_t)(raw << 21)) >> 21);
    const int z = c_zz[j];
    if (z & 1) nw[z >> 1] |= v << 16;
    else nw[z >> 1] |= v & 0xFFFFu;
    rwin <<= (n + 1) & 63;
    bp = bpn;
    act = take && bpn < T.nbits;
  }
  }
  return bad;
}

// Symbols of any table, bit-serial conditions as the reference evaluates them
// (uint8 arithmetic of `first` kept), values found by walking the groups of
// the matched length in stream order; int16 stores straight into the quad
// layout (slot `g`), zeros after the last symbol.  Only lanes whose table is
// not regular (malformed or hand-made streams) come here, after the wave's
// regular lanes, with the unrolled state dead.
__device__ __forceinline__ int decode_general(const LdsChunk c, const Table T, uint4* coef,
                                           uint32_t g) {
  uint16_t* out = reinterpret_cast<uint16_t*>(coef);
  int code = 0;
  uint32_t bp = 0, j = 0;
  while (bp < T.nbits && j < 64) {
    const uint32_t P = T.sbit + bp;
    const uint32_t x = c.byte(P >> 3) | (c.byte((P >> 3) + 1) << 8);
    const uint32_t w8 = __brev((x >> (P & 7)) & 0xFF) >> 24;  // next 8 bits, MSB-first
    uint32_t first = 0, mL = 0, r = 0;
    bool neg = false;
#pragma unroll
    for (uint32_t L = 1; L <= 8; L++) {
      const uint32_t cL = (uint32_t)(T.cnt >> (8 * (L - 1))) & 0xFF;
      const uint32_t cd = w8 >> (8 - L);
      if (mL == 0 && cd < cL + first) {
        mL = L;
        neg = cd < first;
        r = cd - first;
      }
      first = ((first + cL) << 1) & 0xFF;
    }
    if (mL == 0) {
      code = (bp + 8 > T.nbits) ? 10 : 11;
      break;
    }
    if (bp + mL > T.nbits || neg) {
      code = 10;
      break;
    }
    uint32_t i = 3, vbit = 0;
    while (i - 3 < T.tb) {
      const uint32_t info = c.byte(i);
      const uint32_t n = (info & 31) + 1;
      if ((info >> 5) + 1 == mL) {
        if (r < n) {
          vbit = 8 * (i + 1) + 11 * r;
          break;
        }
        r -= n;
      }
      i += 1 + (n * 11 + 7) / 8;
    }
    const uint32_t z = c_zz_dev[j];
    out[coef_quad(g, z >> 3) * 8 + (z & 7)] = (uint16_t)(((int32_t)(c.bits32(vbit) << 21)) >> 21);
    bp += mL;
    j++;
  }
  for (; j < 64; j++) {
    const uint32_t z = c_zz_dev[j];
    out[coef_quad(g, z >> 3) * 8 + (z & 7)] = 0;
  }
  return code;
}

}  // namespace

#ifdef MYYUV_STAMPS
// diagnostic build only (-DMYYUV_STAMPS): the fused decoder's wave cycles
// per phase, per wave (plain stores at the wave's end; contended atomics
// would distort the timing): g_dec_wstamps[wave][8] = [0] setup (sizes,
// scan, offsets), [1] staging, [2] table parse, [3] symbol loop, [5] the DC
// blocks and the transform, [6] rounds, [7] = 1 for a wave that ran
// (myyuv_debug_dec_stamps, tools/dec_phase.py)
__device__ uint32_t g_dec_wstamps[65536 * 8];
struct DStamps {
  unsigned long long prev;
  uint32_t acc[8];
};
#define DSTAMP(k)                                                \
  do {                                                           \
    if (ds != nullptr) {                                         \
      __builtin_amdgcn_sched_barrier(0);                         \
      const unsigned long long _t = __builtin_amdgcn_s_memtime(); \
      __builtin_amdgcn_sched_barrier(0);                         \
      ds->acc[k] += (uint32_t)(_t - ds->prev);                   \
      ds->prev = _t;                                             \
    }                                                            \
  } while (0)
#else
struct DStamps {};
#define DSTAMP(k) \
  do {            \
  } while (0)
#endif

// K5's decode of one wave's 64-block group (blockIdx.x) of frame blockIdx.y:
// the natural-order words of each lane's block in nw (or, for a table that is
// not "regular", written to coef by decode_general: *direct).  Returns false
// when the frame's stream header is bad (nothing decoded).
struct DecodeGroup {
  uint32_t f, gbase, g0, g1, g;
  int p;
  bool live;
};
__device__ __forceinline__ bool decode_group(const uint8_t* __restrict__ in, const uint32_t* __restrict__ in_size,
                                             uint32_t cap, const StreamDesc* __restrict__ desc,
                                             const uint32_t* __restrict__ local_off,
                                             const uint32_t* __restrict__ tile_pre, const FrameGeom& G,
                                             uint32_t tiles_p0, uint32_t tiles_p1, uint4* __restrict__ coef,
                                             unsigned long long* __restrict__ err, uint4* stq, DecodeGroup& D,
                                             uint32_t (&nw)[32], bool& direct, DStamps* ds = nullptr) {
  // frame blockIdx.y of the batch: its stream slot, descriptor and scan;
  // coefficients at batch-global block gbase + g
  const uint32_t f = blockIdx.y;
  const uint32_t nblk = G.cum[3];
  const uint32_t gbase = f * nblk;
  const uint32_t ntiles = (nblk + kScanTile - 1) / kScanTile;
  in += (size_t)f * cap;
  desc += f;
  local_off += gbase;
  tile_pre += (size_t)f * (ntiles + 1);
  const int lane = threadIdx.x;
  // the lanes' per-length value positions (stage bit of the length's first
  // value - 11 * its first code; length-major: lane l's length L at
  // [64 L + l]), after the stage and its zero quad
  uint32_t* gcol = reinterpret_cast<uint32_t*>(stq + kStageQuads + 1) + lane;
  const uint32_t t = blockIdx.x;
  const int p = t >= tiles_p0 ? (t >= tiles_p0 + tiles_p1 ? 2 : 1) : 0;
  // the plane's fields by static index (a dynamic index into the kernel
  // argument G, or into the descriptor once loaded, is a scalar load: one
  // more dependent round trip)
  auto sel3 = [p](uint32_t a0, uint32_t a1, uint32_t a2) { return p == 0 ? a0 : (p == 1 ? a1 : a2); };
  const uint32_t cum_p = sel3(G.cum[0], G.cum[1], G.cum[2]), cum_p1 = sel3(G.cum[1], G.cum[2], G.cum[3]);
  const uint32_t tile_in_plane = t - sel3(0u, tiles_p0, tiles_p0 + tiles_p1);
  const uint32_t g0 = cum_p + tile_in_plane * kWave;
  const uint32_t g1 = min(g0 + kWave, cum_p1);
  const uint32_t g = g0 + lane;
  const bool live = g < g1;
  // every scalar of the setup in one round trip: the descriptor, the payload
  // size, the scan at the plane's start and the group's ends.  No branch on
  // `bad` in front of them (it would hold the rest back by a round trip): a
  // bad frame decodes nothing (no lane is ok) and returns false below.
  const StreamDesc dsc = *desc;
  const uint32_t isz = in_size[f];
  const uint32_t g1c = min(g1, nblk - 1);
  const uint32_t lo_p = local_off[cum_p], tp_p = tile_pre[cum_p / kScanTile];
  const uint32_t lo_0 = local_off[g0], tp_0 = tile_pre[g0 / kScanTile];
  const uint32_t lo_1 = local_off[g1c], tp_1 = tile_pre[g1c / kScanTile];
  const uint32_t stot = tile_pre[ntiles];  // rel(nblk) = the total
  __builtin_amdgcn_sched_barrier(0);  // (all issued before the first use waits)
  const uint32_t plane_pre = lo_p + tp_p, s0 = lo_0 + tp_0, s1 = lo_1 + tp_1;
  const bool bad = dsc.bad != 0;
  const uint32_t limit = bad ? 0u : min(isz, cap);
  // end of the wave's chunk range from the scan alone
  const uint32_t end_scan = g1 == nblk ? stot : s1;
  const uint32_t cpos = sel3(dsc.content_pos[0], dsc.content_pos[1], dsc.content_pos[2]);
  const uint32_t csize = sel3(dsc.content_size[0], dsc.content_size[1], dsc.content_size[2]);
  const uint32_t spos = sel3(dsc.sizes_pos[0], dsc.sizes_pos[1], dsc.sizes_pos[2]);
  const uint32_t E = cpos + min(end_scan - plane_pre, csize);
  // Round 1 stages from the group's first chunk (lane 0's: g0 < g1, so lane
  // 0 is live; when it is not ok, no lane is and no round runs).  Its
  // position needs no size byte, so its loads go out together with the size
  // bytes' (issued just before them: the VMEM counter drains in order, so
  // the size bytes' wait covers them either way) instead of after the size
  // scan: one dependent load round trip less before the table parse.
  const uint32_t pre0 = s0 - plane_pre;
  auto window = [&](uint32_t A, uint32_t& aw, uint32_t& wend, uint32_t& nq, uint32_t& nfull) {
    aw = A & ~15u;
    wend = aw + 16 * (kStageQuads - 1);
    nq = E > aw ? (min(E, wend) - aw + 15) >> 4 : 0u;
    nfull = limit >= aw ? min(nq, (limit - aw) >> 4) : 0u;  // quads below limit
  };
  // the first 256 quads straight into the stage (LDS-DMA: quad 64m + lane
  // from instruction m), all in flight together and holding no registers.
  // Unconditional, at clamped addresses: the quads they write at or past
  // nfull are rewritten by stage() up to nq, and past nq nothing reads the
  // stage
  auto load4 = [&](uint32_t aw, uint32_t nfull) {
#pragma unroll
    for (int m = 0; m < 4; m++) {
      const uint8_t* src = nfull > 0 ? in + aw + 16 * min(lane + 64u * m, nfull - 1) : in;
      __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(stq + 64 * m),
                                       16, 0, 0);
    }
  };
  uint32_t aw, wend, nq, nfull;
  window(cpos + pre0, aw, wend, nq, nfull);
  load4(aw, nfull);
  __builtin_amdgcn_sched_barrier(0);  // (all four issued before the size bytes' load)
  const uint32_t gl = live ? g : g1 - 1;
  const uint32_t s = in[bad ? 0u : spos + (gl - cum_p)];
  // the chunk's offset: the group's (k_scan_chain keeps group starts only)
  // plus the wave's exclusive scan of the sizes
  // (by DPP, the whole wave active: six ds_bpermute round trips less)
  const uint32_t incl = wave_incl_scan(live ? s : 0u);
  const uint32_t rel = pre0 + incl - (live ? s : 0u);

  // plane-level check (DCT.cpp:21-33 reads past content_size otherwise):
  // the chunks must fit the declared content.
  bool ok = live && !bad;
  if (ok && rel + s > csize) {
    record_error(err, 2ull * ((uint64_t)G.fbase * nblk + gbase + cum_p), 9 /* MYYUV_E_PLANE_CONTENT */);
    ok = false;
  }

  int code = 0;
  direct = false;  // block written by decode_general

  // Rounds: stage the chunks of the first pending lane onwards (as many as
  // the stage holds, bytes at or past `limit` read as 0, one zero quad after),
  // decode the lanes whose chunks are inside.  Chunks are consecutive and at
  // most 255 B, so every round retires at least one lane; a 4K frame at q=50
  // needs one round per wave.
  uint64_t pending = __ballot(ok);
  DSTAMP(0);
  // the rest of one round's stage: the window past 256 quads, zeros at or
  // past `limit` and the slack quad
  auto stage = [&]() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // load4's LDS writes (before the zero quads)
    for (uint32_t k = lane + 256; k < nfull; k += 64)
      stq[k] = *reinterpret_cast<const uint4*>(in + aw + 16 * k);
    for (uint32_t k = nfull + lane; k <= nq; k += 64) {
      uint32_t v[4] = {0, 0, 0, 0};
      if (k < nq) {
#pragma unroll
        for (uint32_t b = 0; b < 16; b++) {
          const uint32_t a = aw + 16 * k + b;
          if (a < limit) v[b >> 2] |= (uint32_t)in[a] << (8 * (b & 3));
        }
      }
      stq[k] = make_uint4(v[0], v[1], v[2], v[3]);
    }
    __syncthreads();
  };
  if (pending) stage();
  while (pending) {
#ifdef MYYUV_STAMPS
    if (ds != nullptr) ds->acc[6] += 1;
#endif
    DSTAMP(1);

    const bool mine = ((pending >> lane) & 1) && cpos + rel + s <= wend;
    const LdsChunk lc{reinterpret_cast<const uint32_t*>(stq), mine ? cpos + rel - aw : 0u};
    Table T;
    // (every lane parses, the others as a bad header of size 0 at the stage's
    // start: no branch level around the parse, whose outputs the compiler
    // would re-initialise on the skipped path)
    const int pcode = parse_table(lc, mine ? s : 0u, T, gcol);
    const bool go = mine && pcode == 0;
    int dcode = 0;
    DSTAMP(2);
    const bool failed = decode_regular(lc, T, gcol, go && T.regular, nw);
    // tables the reference never writes, and failed messages (for the
    // reference's exact error code): the bit-serial path
    if (go && (!T.regular || failed)) {
      direct = true;
      dcode = decode_general(lc, T, coef, gbase + g);
    }
    if (mine) code = go ? dcode : pcode;
    pending &= ~__ballot(mine);
    DSTAMP(3);
    if (pending) {  // the next round, from the lowest pending lane's chunk
      __syncthreads();  // it overwrites the stage
      const int lo = __ffsll((long long)pending) - 1;
      window(cpos + __shfl(rel, lo, 64), aw, wend, nq, nfull);
      load4(aw, nfull);
      stage();
    }
  }
  // every LDS-DMA load has landed before the stage is reused or the wave
  // ends, whether or not a round ran (no lane ok: round 1's loads were still
  // issued)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (ok && code) record_error(err, 2ull * ((uint64_t)G.fbase * nblk + gbase + g) + 1, code);
  D.f = f;
  D.gbase = gbase;
  D.g0 = g0;
  D.g1 = g1;
  D.g = g;
  D.p = p;
  D.live = live;
  return !bad;
}

__global__ __launch_bounds__(64, MYYUV_K5S_WAVES) void k_huff_decode(const uint8_t* __restrict__ in,
                                                   const uint32_t* __restrict__ in_size,
                                                   uint32_t cap,
                                                   const StreamDesc* __restrict__ desc,
                                                   const uint32_t* __restrict__ local_off,
                                                   const uint32_t* __restrict__ tile_pre,
                                                   FrameGeom G, uint32_t tiles_p0,
                                                   uint32_t tiles_p1,
                                                   uint4* __restrict__ coef,
                                                   uint8_t* __restrict__ rmask,
                                                   unsigned long long* __restrict__ err) {
  __shared__ uint4 stq[kStageQuads + 1 + kGposQuads];
  if (threadIdx.x == 0) stq[kStageQuads] = make_uint4(0u, 0u, 0u, 0u);  // (ordered by decode_group's barrier)
  DecodeGroup D;
  uint32_t nw[32];
#pragma unroll
  for (int w = 0; w < 32; w++) nw[w] = 0;
  bool direct;
  if (!decode_group(in, in_size, cap, desc, local_off, tile_pre, G, tiles_p0, tiles_p1, coef, err, stq, D, nw,
                    direct))
    return;  // the frame's stream header is bad (k_scan_chain recorded it)
  const uint32_t gbase = D.gbase, g = D.g;
  const bool live = D.live;
  // ---- natural-order words to the quad layout (1 KiB contiguous per store)
  // Only the nonzero rows are stored; bit c of the block's row mask says
  // whether row c holds a nonzero coefficient, and K6 reads just those.
  // decode_general wrote all 64 coefficients itself: mask 0xFF.
  if (live) {
    uint32_t m = 0xFFu;
    if (!direct) {
      m = 0;
#pragma unroll
      for (int c = 0; c < 8; c++) {
        const bool nz = (nw[4 * c] | nw[4 * c + 1] | nw[4 * c + 2] | nw[4 * c + 3]) != 0u;
        m |= nz ? 1u << c : 0u;
        if (nz) coef[coef_quad(gbase + g, c)] = make_uint4(nw[4 * c], nw[4 * c + 1], nw[4 * c + 2], nw[4 * c + 3]);
      }
    }
    rmask[gbase + g] = (uint8_t)m;
  }
}

// Fused decoder (K5 + K6; MYYUV_DECODER=fused): the wave decodes its 64-block
// group as K5 does, then runs K6's transform on it in 8-block units straight
// from its registers: the unit's 8 decoding lanes write their blocks' int16
// images into the wave's transpose tile (laid over the chunk stage, dead by
// then), and the wave's lanes take (block, row) roles (idct_row8,
// xform_common.hpp).  The coefficients never reach HBM.
__global__ __launch_bounds__(64, MYYUV_K5_WAVES) void k_decode_idct(const uint8_t* __restrict__ in,
                                                   const uint32_t* __restrict__ in_size,
                                                   uint32_t cap,
                                                   const StreamDesc* __restrict__ desc,
                                                   const uint32_t* __restrict__ local_off,
                                                   const uint32_t* __restrict__ tile_pre,
                                                   FrameGeom G, uint32_t tiles_p0,
                                                   uint32_t tiles_p1, const QTables* __restrict__ qt,
                                                   uint4* __restrict__ coef,
                                                   uint8_t* __restrict__ frame,
                                                   unsigned long long* __restrict__ err) {
  static_assert(sizeof(uint4) * kStageQuads >= sizeof(float) * xf::kXfTile16, "the tile over the stage");
  __shared__ uint4 stq[kStageQuads + 1 + kGposQuads];
  __shared__ float sq[64];
  __shared__ uint16_t s_blk[64];
  const uint32_t lane = threadIdx.x;
  if (lane == 0) stq[kStageQuads] = make_uint4(0u, 0u, 0u, 0u);  // (ordered by decode_group's barrier)
  {
    // the plane's Q table by LDS-DMA (no register, no wait here; landed by
    // decode_group's final vmcnt wait, before idct_rows)
    const uint32_t t = blockIdx.x;
    const int p = t >= tiles_p0 ? (t >= tiles_p0 + tiles_p1 ? 2 : 1) : 0;
    __builtin_amdgcn_global_load_lds((const void*)&qt->q[p][lane], (__attribute__((address_space(3))) void*)sq, 4,
                                     0, 0);
  }
#ifdef MYYUV_STAMPS
  DStamps dst;
  DStamps* ds = &dst;
  dst.prev = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int k = 0; k < 8; k++) dst.acc[k] = k == 7 ? 1u : 0u;
#else
  DStamps* ds = nullptr;
#endif
  DecodeGroup D;
  uint32_t nw[32];
#pragma unroll
  for (int w = 0; w < 32; w++) nw[w] = 0;
  bool direct;
  if (!decode_group(in, in_size, cap, desc, local_off, tile_pre, G, tiles_p0, tiles_p1, coef, err, stq, D, nw,
                    direct, ds))
    return;  // the frame's stream header is bad (k_scan_chain recorded it)
  DSTAMP(4);
  if (D.live && direct) {  // decode_general wrote the block to coef (a table the reference never writes)
#pragma unroll
    for (int c = 0; c < 8; c++) {
      const uint4 v = coef[coef_quad(D.gbase + D.g, c)];
      nw[4 * c] = v.x;
      nw[4 * c + 1] = v.y;
      nw[4 * c + 2] = v.z;
      nw[4 * c + 3] = v.w;
    }
  }
  // ---- K6 on the group.  Blocks whose only nonzero coefficient is the DC
  // (53 % of the bench frame's blocks) decode to one constant pixel value:
  // with Z[0][0] = z the only nonzero coefficient, stage 1 leaves U[i][0] =
  // fl(D[0][i] * z), stage 2 R[i][v] = fl(U[i][0] * D[0][v]) (the other
  // products are +-0 and every sum starts at +0), and row 0 of the literal
  // basis is one value c, so R = fl(fl(c * z) * c) for all 64 pixels — the
  // same two roundings as the full transform, which the lane evaluates for its
  // own block and stores as 8 rows.  The other blocks are compacted into
  // 8-block units for the transform (up to eight; their rows are written
  // wherever the blocks lie).
  const int p = D.p;
  xf::Unit U;
  U.p = p;
  U.cum = G.cum[p];
  U.nb = G.cum[p + 1] - G.cum[p];
  U.poff = p == 0 ? G.poff[0] : (p == 1 ? G.poff[1] : G.poff[2]);
  U.pw = p == 0 ? G.pw[0] : (p == 1 ? G.pw[1] : G.pw[2]);
  U.bw = p == 0 ? G.bw[0] : (p == 1 ? G.bw[1] : G.bw[2]);
  U.bmag = p == 0 ? G.bmag[0] : (p == 1 ? G.bmag[1] : G.bmag[2]);
  U.local0 = 0;
  uint8_t* fr = frame + (size_t)D.f * G.fbytes;
  uint32_t acc = nw[0] & 0xFFFF0000u;
#pragma unroll
  for (int w = 1; w < 32; w++) acc |= nw[w];
  const bool isdc = D.live && acc == 0u;
  if (isdc) {
    constexpr float c0 = xf::c_dct[0];
    static_assert(xf::c_dct[0] == xf::c_dct[1] && xf::c_dct[0] == xf::c_dct[7], "row 0 of the basis is one value");
    const float z = (float)(int16_t)nw[0] * sq[0];  // dequantise (DCT.cpp:331)
    const float u = 0.0f + c0 * z;                  // stage 1: the k = 0 term
    float S = 0.0f + u * c0;                        // stage 2: the k = 0 term
    S = __builtin_amdgcn_fmed3f(S, -128.0f, 127.0f);  // (as idct_rows, DCT.cpp:358-362)
    uint32_t px = xf::bits(S + xf::kMagicPx);
    if (__builtin_amdgcn_fractf(S) == 0.5f)
      px = (uint32_t)((int)__builtin_truncf(S + __builtin_copysignf(xf::kHalfDown, S)) + 128);
    const uint32_t v4 = (px & 0xFFu) * 0x01010101u;
    const uint2 row = make_uint2(v4, v4);
#pragma unroll
    for (uint32_t r = 0; r < 8; r++) {
      const uint32_t off = xf::block_row_offset(U, D.g - U.cum, r);
      *reinterpret_cast<uint2*>(fr + off) = row;
    }
  }
  // (compacted in block order: ordering the units by sparsity kind — row 0
  // only, column 0 only, the rest — measured no faster, profiles/r3zl_*)
  const uint64_t rest = __ballot(D.live && !isdc);
  const uint32_t nrest = (uint32_t)__popcll(rest);
  const uint32_t rrank = __builtin_amdgcn_mbcnt_hi((uint32_t)(rest >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)rest, 0u));
  if (D.live && !isdc) s_blk[rrank] = (uint16_t)lane;  // compacted position -> the block's lane in the group
  float* tile = reinterpret_cast<float*>(stq);
  // 16-block units while more than 8 blocks are left (lane (b, q): rows 2q,
  // 2q+1 of block b, idct_rows), the last 1-8 blocks as one 8-block unit
  // (lane (b, r): row r, idct_row8, half the products per step).  Slots past
  // the last block are zero, so they do not keep steps alive; slot `lane` is
  // zeroed by lane `lane` whether or not that lane also writes a compacted
  // block: the two slots differ (rrank < nrest <= base + lane).
#pragma unroll 1
  for (uint32_t base = 0; base < nrest;) {
    const bool wide = nrest - base > 8u;
    const uint32_t span = wide ? 16u : 8u, stride = wide ? (uint32_t)xf::kTile : (uint32_t)xf::kTile8;
    const uint32_t s = rrank - base;
    if (D.live && !isdc && rrank >= base && s < span) {
      uint4* img = reinterpret_cast<uint4*>(tile + s * stride + (wide ? xf::img_word(s) : 0u));
#pragma unroll
      for (int c = 0; c < 8; c++) img[c] = make_uint4(nw[4 * c], nw[4 * c + 1], nw[4 * c + 2], nw[4 * c + 3]);
    }
    if (lane < span && base + lane >= nrest) {
      uint4* img = reinterpret_cast<uint4*>(tile + lane * stride + (wide ? xf::img_word(lane) : 0u));
#pragma unroll
      for (int c = 0; c < 8; c++) img[c] = make_uint4(0u, 0u, 0u, 0u);
    }
    xf::wave_sync();
    if (wide) {
      const uint32_t q = lane & 3u, b = lane >> 2;
      uint2 w0, w1;
      xf::idct_rows(tile + b * xf::kTile, q, b, sq, w0, w1);
      if (base + b < nrest) {
        const uint32_t gl = D.g0 + s_blk[base + b];  // the block of compacted position base + b
        const uint32_t off = xf::block_row_offset(U, gl - U.cum, 2u * q);
        *reinterpret_cast<uint2*>(fr + off) = w0;
        *reinterpret_cast<uint2*>(fr + off + U.pw) = w1;
      }
    } else {
      const uint32_t r = lane & 7u, b = lane >> 3;
      float qc[8];  // the lane's column of the plane's Q table, Q[k][r]
#pragma unroll
      for (int k = 0; k < 8; k++) qc[k] = sq[8 * k + r];
      const uint2 w = xf::idct_row8(tile + b * xf::kTile8, r, qc);
      if (base + b < nrest) {
        const uint32_t gl = D.g0 + s_blk[base + b];
        *reinterpret_cast<uint2*>(fr + xf::block_row_offset(U, gl - U.cum, r)) = w;
      }
    }
    xf::wave_sync();  // the next unit rewrites the tile
    base += span;
  }
  DSTAMP(5);
#ifdef MYYUV_STAMPS
  const uint32_t wid = blockIdx.y * gridDim.x + blockIdx.x;
#pragma unroll
  for (int k = 0; k < 8; k++)
    if (lane == (uint32_t)k && wid < 65536) g_dec_wstamps[wid * 8 + k] = dst.acc[k];
#endif
}

}  // namespace myyuv_gpu
