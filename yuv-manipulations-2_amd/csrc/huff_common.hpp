// huff_common.hpp — pieces of K2 (Huffman::fromData + Huffman::dump,
// myyuv_DCT/Huffman.cpp:172-241, :279-326) shared by the kernels in
// k_huff_encode.hip and compiled for the host as well (MYYUV_HD), so the
// register-resident encoder's logic can be checked against the oracle on the
// CPU (tools/r8_host.cpp, tests/test_r8_host.py).  The device build is the
// product; the host build is test infrastructure.
#pragma once
#include "codec_common.hpp"

#define MYYUV_HD __host__ __device__ __forceinline__

// diagnostic hook (k_huff_encode.hip's stamp build): per-phase wave cycles
#ifndef R8_STAMP
#define R8_STAMP(k) \
  do {              \
  } while (0)
#define R8_STAMP_DECL
#endif

namespace myyuv_gpu {

MYYUV_HD uint32_t hd_umulhi(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)a * b) >> 32);
}
MYYUV_HD uint32_t hd_brev(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __brev(x);
#else
  uint32_t r = 0;
  for (int i = 0; i < 32; i++) r |= ((x >> i) & 1u) << (31 - i);
  return r;
#endif
}
MYYUV_HD uint32_t hd_clz(uint32_t x) { return (uint32_t)__builtin_clz(x); }  // x != 0
MYYUV_HD uint32_t hd_ctz(uint32_t x) { return (uint32_t)__builtin_ctz(x); }  // x != 0
// v_perm_b32: byte i of the result = byte sel.byte[i] (0..7) of {hi, lo}
MYYUV_HD uint32_t hd_perm(uint32_t hi, uint32_t lo, uint32_t sel) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_perm(hi, lo, sel);
#else
  const uint64_t v = ((uint64_t)hi << 32) | lo;
  uint32_t r = 0;
  for (int i = 0; i < 4; i++) r |= (uint32_t)((v >> (8 * ((sel >> (8 * i)) & 7u))) & 0xFFu) << (8 * i);
  return r;
#endif
}

// Bucket-count phases of the prime rehash policy for <= 65 elements
// (_Prime_rehash_policy::_M_next_bkt / _M_need_rehash): 13 buckets from the
// first insert, 29 at the 14th, 59 at the 30th, 127 at the 60th element.
struct Phase {
  uint32_t nb, r64, magic;  // buckets, 2^64 mod nb, ceil(2^32 / nb)
};
MYYUV_HD constexpr uint32_t pow2_64_mod(uint32_t m) {
  uint64_t r = 1;
  for (int i = 0; i < 64; i++) r = (r * 2) % m;
  return (uint32_t)r;
}
MYYUV_HD Phase phase_of(int ph) {
  Phase p;
  p.nb = ph == 0 ? 13u : ph == 1 ? 29u : ph == 2 ? 59u : 127u;
  p.r64 = ph == 0   ? pow2_64_mod(13)
          : ph == 1 ? pow2_64_mod(29)
          : ph == 2 ? pow2_64_mod(59)
                    : pow2_64_mod(127);
  p.magic = ph == 0 ? 330382100u : ph == 1 ? 148102321u : ph == 2 ? 72796056u : 33818641u;
  return p;
}
// hash(int16 v) % nb with hash = (size_t)(int64)v: v >= 0 -> v % nb,
// v < 0 -> (2^64 + v) % nb = (r64 + v) % nb.  t < 2^17: the magic multiply
// is exact.
MYYUV_HD uint32_t bucket_of(int v, const Phase& P) {
  const uint32_t t = (uint32_t)(v + (v < 0 ? (int)(P.r64 + 1024u * P.nb) : 0));
  const uint32_t q = hd_umulhi(t, P.magic);
  return t - q * P.nb;
}

// LSB-first bit writer into a block's contiguous 160-B overflow slot
// (k_huff_encode_wide / _wave: blocks with more than 8 distinct symbols).
struct BitWriter {
  uint32_t* out;  // slot word 0 of this block
  uint64_t acc = 0;
  int nacc = 0;
  int widx = 0;
  MYYUV_HD void put(uint32_t v, int n) {
    acc |= (uint64_t)v << nacc;
    nacc += n;
    if (nacc >= 32) {
      out[widx] = (uint32_t)acc;
      widx++;
      acc >>= 32;
      nacc -= 32;
    }
  }
  MYYUV_HD void align_byte() { nacc = (nacc + 7) & ~7; }
  MYYUV_HD void flush() {
    if (nacc > 0) out[widx] = (uint32_t)acc;
  }
};

// LSB-first bit writer for K2's dense tile run: a workgroup's chunks are
// packed back to back in block order (byte offsets from an in-tile scan), and
// every dword is stored by exactly one lane — the block that owns the dword's
// first byte.  A chunk therefore skips its first dword when it starts
// mid-dword (the previous block stores it) and completes its last dword with
// the first bytes of the next chunk in the run.  Those can only be the next
// chunk's 3-byte header (u16 nbits, u8 table_bytes: a chunk is >= 7 bytes),
// which every block knows before anything is emitted.  No atomics, no
// read-modify-write, no shared words.
struct DenseWriter {
  uint32_t* base;  // the tile run, dword aligned
  uint32_t widx;   // dword being filled
  uint64_t acc;
  int nacc;
  bool skip;       // the dword being filled belongs to the previous chunk
  MYYUV_HD void init(uint32_t* run, uint32_t off) {
    base = run;
    widx = off >> 2;
    nacc = (int)(off & 3u) * 8;
    acc = 0;
    skip = (off & 3u) != 0;
  }
  MYYUV_HD void put(uint32_t v, int n) {
    acc |= (uint64_t)v << nacc;
    nacc += n;
    if (nacc >= 32) {
      if (!skip) base[widx] = (uint32_t)acc;
      skip = false;
      widx++;
      acc >>= 32;
      nacc -= 32;
    }
  }
  MYYUV_HD void align_byte() { nacc = (nacc + 7) & ~7; }
  // after the last byte: next = the next chunk's header | 1 << 31 (0: none)
  MYYUV_HD void finish(uint32_t next) {
    align_byte();
    if (nacc > 0) {
      if (next >> 31) acc |= (uint64_t)(next & 0xFFFFFFu) << nacc;
      base[widx] = (uint32_t)acc;  // (a chunk spans > 4 bytes: never the skipped dword)
    }
  }
};

// Per-position KC slot of the position's symbol, recorded while the distinct
// symbols are found so the emitter indexes the code table directly instead of
// probing the hash table again: kBits bits per position, positions static.
template <int CAP>
struct SlotIds {
  static constexpr int kBits = CAP <= 8 ? 3 : (CAP <= 16 ? 4 : 6);
  static constexpr int kPer = 32 / kBits;
  static constexpr int kRegs = (64 + kPer - 1) / kPer;
  uint32_t r[kRegs];
  MYYUV_HD void clear() {
#pragma unroll
    for (int i = 0; i < kRegs; i++) r[i] = 0;
  }
  MYYUV_HD void set(int pos, uint32_t slot) {
    r[pos / kPer] |= slot << (kBits * (pos % kPer));
  }
  MYYUV_HD uint32_t get(int pos) const {
    return (r[pos / kPer] >> (kBits * (pos % kPer))) & ((1u << kBits) - 1u);
  }
};

// The lane's block's coefficients (natural order, word w = coefficients 2w,
// 2w+1), loaded once into registers: every loop over positions below is
// unrolled, so sym(i) — the i-th coefficient in zig-zag order — is a static
// register index and half.
constexpr uint8_t c_zz[64] = MYYUV_ZIGZAG;

struct CoefRegs {
  uint32_t w[32];
  // rows whose bit in the block's row mask m (K1) is clear are zero: read
  // from the zero buffer zq instead (the load is still issued)
  __device__ __forceinline__ void load(const uint4* __restrict__ coef, const uint4* __restrict__ zq,
                                       uint32_t g, uint32_t m) {
#pragma unroll
    for (int c = 0; c < 8; c++) {
      const uint4 v = *((m >> c) & 1u ? coef + coef_quad(g, c) : zq);
      w[4 * c] = v.x;
      w[4 * c + 1] = v.y;
      w[4 * c + 2] = v.z;
      w[4 * c + 3] = v.w;
    }
  }
  MYYUV_HD int sym(int i) const {
    const int n = c_zz[i];
    return (int)(int16_t)(w[n >> 1] >> (16 * (n & 1)));
  }
  // 1 + zig-zag index of the last nonzero coefficient (0: all zero)
  MYYUV_HD int msz() const {
    int m = 0;
#pragma unroll
    for (int i = 0; i < 64; i++)
      if (sym(i) != 0) m = i + 1;
    return m;
  }
};

// ---------------------------------------------------------------------------
// Register-resident encoder for blocks with at most CAP (4 or 8) distinct
// symbols, lane per block.  The LDS version of encode_block is a
// chain of dependent LDS round trips per lane (probing, list and heap
// surgery), so the longest lane of each wave sets the kernel time; here every
// structure lives in registers and every dynamic index is a small select
// network or a shift into a packed word:
//   * keys: 12-bit tagged fields (0x800 | v & 0x7FF; 0 = empty), two per
//     dword; one position is matched against all 8 keys with three SWAR ops
//     per dword pair;
//   * counts: 8 x u8 in a 64-bit word; per-position slot ids (3 bits);
//   * unordered_map order in closed form (13 buckets: no rehash below 13
//     symbols, so the freq[0] probe is invisible): runs of a bucket in
//     decreasing first insertion, each run in decreasing insertion order;
//   * the libstdc++ heap (push_heap / pop_heap, __adjust_heap) on 8 registers,
//     specialised for at most 8 entries: a pop or push is a merge of one
//     entry into a root path of at most three entries (pop / push below);
//   * parents, depths, per-length counts, canonical first codes: packed
//     nibble / byte fields.
// Same bytes as encode_block.
// ---------------------------------------------------------------------------

// Positions per wave-uniform step of the per-position loops (the loops run to
// the wave's longest message).
constexpr int kPosGroup = 4;

namespace rr {

MYYUV_HD uint32_t fq(uint32_t e) { return e >> 8; }

// H[i] for a dynamic i in [0, CAP)
template <int CAP>
MYYUV_HD uint32_t hget(const uint32_t (&H)[CAP], uint32_t i) {
  const uint32_t a = (i & 1) ? H[1] : H[0], b = (i & 1) ? H[3] : H[2];
  const uint32_t ab = (i & 2) ? b : a;
  if constexpr (CAP == 4) {
    return ab;
  } else {
    const uint32_t c = (i & 1) ? H[5] : H[4], d = (i & 1) ? H[7] : H[6];
    const uint32_t cd = (i & 2) ? d : c;
    return (i & 4) ? cd : ab;
  }
}
// H[i] = x for a dynamic i in [lo, hi]
template <int lo, int hi, int CAP>
MYYUV_HD void hset(uint32_t (&H)[CAP], uint32_t i, uint32_t x) {
#pragma unroll
  for (int s = lo; s <= hi; s++) H[s] = i == (uint32_t)s ? x : H[s];
}

// Heap entries are freq << 8 | id with freq < 256, so fq(a) <= fq(b) is
// a <= (b | 0xFF) and fq(a) > fq(b) is a > (b | 0xFF): one compare.
MYYUV_HD bool fq_gt(uint32_t a, uint32_t b) { return a > (b | 0xFFu); }

// std::priority_queue::pop (libstdc++ __pop_heap + __adjust_heap, then
// __push_heap of the last element from the hole) for a heap that keeps m
// entries, m in [0, CAP-1]; returns the old top.  __adjust_heap walks a path
// down from the root, moving each path entry up one level; __push_heap then
// sifts the old last element v back up the same path.  The path entries are
// in heap order, so the result is v merged into the path: the r path
// entries with freq <= fq(v) stay above it, the others move down one.  With
// at most 7 entries left the path is the root, one child c1 (when m >= 2)
// and one grandchild c2 (m >= 4; CAP 8): the whole pop is two compares for
// the path, one for r per level and a select per touched position.
template <int CAP>
MYYUV_HD uint32_t pop(uint32_t (&H)[CAP], uint32_t m) {
  // (the entries are copied to scalars: a select between two elements of
  // the array would be folded into a dynamically indexed load, which moves
  // the array out of registers)
  uint32_t x[8];
#pragma unroll
  for (int k = 0; k < 8; k++) x[k] = k < CAP ? H[k < CAP ? k : 0] : 0u;
  const uint32_t top = x[0];
  const uint32_t v = hget<CAP>(H, m);
  const uint32_t vh = v | 0xFFu;
  // level 1: child 2 unless freq[2] > freq[1] (m >= 3); child 1 when m = 2
  const bool l1 = m >= 2;
  const bool c1is1 = !(m >= 3) || fq_gt(x[2], x[1]);
  const uint32_t a0 = c1is1 ? x[1] : x[2];
  const bool r1 = l1 && a0 <= vh;
  const uint32_t new0 = r1 ? a0 : v;
  uint32_t new1 = r1 ? v : a0;  // (used when l1)
  if constexpr (CAP == 8) {
    // level 2: the loop goes on while c1 < (m - 1) / 2; an even m ends on the
    // last internal node's single (left) child: (m, c1) = (4, 1) or (6, 2)
    const bool loop2 = c1is1 ? m >= 5 : m >= 7;
    const bool spec2 = c1is1 ? m == 4 : m == 6;
    const bool l2 = loop2 || spec2;
    const uint32_t lt = c1is1 ? x[3] : x[5], rt = c1is1 ? x[4] : x[6];
    const bool left = spec2 || fq_gt(rt, lt);
    const uint32_t a1 = left ? lt : rt;
    const bool r2 = l2 && r1 && a1 <= vh;
    new1 = r2 ? a1 : new1;
    const uint32_t new2 = r2 ? v : a1;
    H[3] = (l2 && c1is1 && left) ? new2 : x[3];
    H[4] = (l2 && c1is1 && !left) ? new2 : x[4];
    H[5] = (l2 && !c1is1 && left) ? new2 : x[5];
    H[6] = (l2 && !c1is1 && !left) ? new2 : x[6];
  }
  H[0] = new0;
  H[1] = (l1 && c1is1) ? new1 : x[1];
  H[2] = (l1 && !c1is1) ? new1 : x[2];
  return top;
}

// std::priority_queue::push (__push_heap) of e at the hole h = current size,
// h in [0, CAP-1]: the ancestors of h with freq > fq(e) (a bottom part of
// the ancestor chain) move down one level, e takes the freed position.
template <int CAP>
MYYUV_HD void push(uint32_t (&H)[CAP], uint32_t h, uint32_t e) {
  uint32_t x[8];
#pragma unroll
  for (int k = 0; k < 8; k++) x[k] = k < CAP ? H[k < CAP ? k : 0] : 0u;
  const uint32_t eh = e | 0xFFu;
  const uint32_t p1 = (h - 1) >> 1;   // parent, [0, 3] (h >= 1)
  const uint32_t p2 = (p1 - 1) >> 1;  // grandparent, [0, 1] (h >= 3)
  const uint32_t b1 = (p1 & 2) ? ((p1 & 1) ? x[3] : x[2]) : ((p1 & 1) ? x[1] : x[0]);
  const uint32_t b2 = p2 == 0 ? x[0] : x[1];
  const bool m1 = h >= 1 && b1 > eh;
  const bool m2 = m1 && h >= 3 && b2 > eh;
  const bool m3 = CAP > 4 && m2 && h >= 7 && x[0] > eh;  // h = 7: p1 = 3, p2 = 1, then the root
  const uint32_t nh = m1 ? b1 : e;
  const uint32_t np1 = m2 ? b2 : (m1 ? e : b1);
  const uint32_t np2 = m3 ? x[0] : (m2 ? e : b2);
  // positions written are distinct: root < p2 < p1 < h
#pragma unroll
  for (int k = 0; k < CAP; k++) {
    uint32_t y = x[k];
    if (k <= 1) y = (h >= 3 && p2 == (uint32_t)k) ? np2 : y;
    if (k <= 3) y = (h >= 1 && p1 == (uint32_t)k) ? np1 : y;
    y = h == (uint32_t)k ? nh : y;
    if (k == 0 && CAP > 4) y = m3 ? e : y;
    H[k] = y;
  }
}

// field i (dynamic, [0, CAP)) of CAP x 16-bit fields in CAP / 2 dwords
// (the dwords are copied to scalars first: a select between two elements of
// a local array gets folded into one dynamically indexed load, which sends
// the whole array to scratch)
template <int CAP>
MYYUV_HD uint32_t f16(const uint32_t (&a)[CAP / 2], uint32_t i) {
  const uint32_t a0 = a[0], a1 = a[1];
  uint32_t d = (i & 2) ? a1 : a0;
  if constexpr (CAP == 8) {
    const uint32_t a2 = a[2], a3 = a[3];
    d = (i & 4) ? ((i & 2) ? a3 : a2) : d;
  }
  return d >> ((i & 1) * 16) & 0xFFFFu;
}

// Ascending sort of CAP (4 or 8) values by a comparator network (19 / 5
// comparators, each a u32 min and max).
template <int CAP>
MYYUV_HD void sort_net(uint32_t (&a)[CAP]) {
  constexpr int n8[19][2] = {{0, 2}, {1, 3}, {4, 6}, {5, 7}, {0, 4}, {1, 5}, {2, 6}, {3, 7}, {0, 1}, {2, 3},
                             {4, 5}, {6, 7}, {2, 4}, {3, 5}, {1, 4}, {3, 6}, {1, 2}, {3, 4}, {5, 6}};
  constexpr int n4[5][2] = {{0, 1}, {2, 3}, {0, 2}, {1, 3}, {1, 2}};
  constexpr int nc = CAP == 8 ? 19 : 5;
#pragma unroll
  for (int c = 0; c < nc; c++) {
    const int i = CAP == 8 ? n8[c][0] : n4[c < 5 ? c : 0][0], j = CAP == 8 ? n8[c][1] : n4[c < 5 ? c : 0][1];
    const uint32_t x = a[i % CAP], y = a[j % CAP];
    a[i % CAP] = x < y ? x : y;
    a[j % CAP] = x < y ? y : x;
  }
}

}  // namespace rr

// What emit_chunk needs of a block whose code was built (build_r /
// build_single), held in registers across k_huff_encode's in-tile scan of the
// chunk sizes: <= 8 symbols.
struct EncState {
  uint32_t hdr;      // the chunk's first 3 bytes: u16 nbits | u8 table_bytes << 16
  uint32_t size;     // chunk bytes: 3 + table_bytes + ceil(nbits / 8)
  uint32_t n;        // distinct symbols
  uint32_t msz;      // message length (positions)
  uint64_t lcount;   // per code length L: symbols of that length (byte L - 1)
  uint32_t TK[4];    // table in canonical order: entry r = key & 0x7FF | len << 11 (16-bit fields)
  uint64_t cc;       // per slot k: its bit-reversed code in byte k
  uint32_t ll;       // per slot k: its code length in nibble k
  SlotIds<8> ids;    // per position: slot of its symbol
};

// The slot of the tagged key pair vv (the key in both 16-bit fields) among
// the NP key pairs KP (field k = slot k; empty fields are 0): SWAR zero-field
// tests, the match bits gathered one per byte (slot k < 4 at bit 8k + 7,
// slot k >= 4 at bit 8(k - 4) + 3) and located with one bit scan.
template <int NP>
MYYUV_HD bool match_slot(const uint32_t (&KP)[NP], uint32_t vv, uint32_t& slot) {
  // per pair, bits 15 / 31 flag fields 0 / 1 (the other bits are junk and
  // masked off after the gather)
  uint32_t mp[NP];
#pragma unroll
  for (int p = 0; p < NP; p++) mp[p] = ~(((KP[p] ^ vv) | 0x80008000u) - 0x00010001u);
  uint32_t oh = hd_perm(mp[1 % NP], mp[0], 0x07050301u) & 0x80808080u;
  if constexpr (NP == 4) oh |= (hd_perm(mp[3 % NP], mp[2 % NP], 0x07050301u) & 0x80808080u) >> 4;
  const uint32_t t = hd_ctz(oh | 0x80000000u);
  slot = (t >> 3) | ((t & 4u) ^ 4u);
  return oh != 0;
}

template <int CAP>
MYYUV_HD bool build_r(const CoefRegs& R, int msz, int wave_msz, EncState& S) {
  using namespace rr;
  static_assert(CAP == 4 || CAP == 8, "CAP");
  constexpr int NP = CAP / 2;
  R8_STAMP_DECL
  R8_STAMP(0);
  // ---------------- 1. distinct symbols, counts, per-position slots ----------------
  uint32_t KP[NP] = {};  // tagged keys, field k = slot k
  uint64_t cnt = 0;               // count of slot k in byte k
  uint32_t n = 0;                 // distinct symbols seen (past CAP: the block overflows)
  SlotIds<CAP> ids;
  ids.clear();
#pragma unroll
  for (int i0 = 0; i0 < 64; i0 += kPosGroup) {
    if (i0 < wave_msz) {
#pragma unroll
      for (int k = 0; k < kPosGroup; k++) {
        const int i = i0 + k;
        const int v = R.sym(i);
        const bool act = i < msz;
        const uint32_t f = 0x800u | ((uint32_t)v & 0x7FFu);
        const uint32_t vv = f | (f << 16);
        uint32_t sl;
        const bool found = match_slot<NP>(KP, vv, sl);
        const bool add = act && !found;
        const bool ins = add && n < CAP;
        sl = found ? sl : n;
        // the new key into field n: a 64-bit shift into the pair of dwords
        // holding fields (n & ~3) .. (n | 3)
        const uint64_t t64 = (uint64_t)(ins ? f : 0u) << (16 * (n & 3u));
        const bool lo4 = n < 4;
        KP[0] |= lo4 ? (uint32_t)t64 : 0u;
        KP[1 % NP] |= lo4 ? (uint32_t)(t64 >> 32) : 0u;
        if constexpr (NP == 4) {
          KP[2 % NP] |= lo4 ? 0u : (uint32_t)t64;
          KP[3 % NP] |= lo4 ? 0u : (uint32_t)(t64 >> 32);
        }
        // every processed position is counted; the zeros past the message are
        // taken off below
        cnt += 1ull << (8 * (sl & 7));
        n += add ? 1u : 0u;
        ids.set(i, sl);  // (read for i < msz only: sl <= 7 there unless the block overflows)
      }
    }
  }
  if (n > (uint32_t)CAP) return false;
  if (msz == 0) {  // all-zero block: one symbol 0, count 1 (Huffman.cpp:191-194)
    KP[0] = 0x800u;
    cnt = 1;
    n = 1;
    msz = 1;
  } else {
    // positions msz .. P - 1 (P: the positions the loop ran, a multiple of
    // kPosGroup) are zeros: counted into the zero's slot, or into slot n & 7
    // when the message has no zero (slot n is unused; n = 8 wraps to slot 0)
    const uint32_t P = (uint32_t)min((wave_msz + kPosGroup - 1) / kPosGroup * kPosGroup, 64);
    uint32_t zs;
    const bool zf = match_slot<NP>(KP, 0x08000800u, zs);
    cnt -= (uint64_t)(P - (uint32_t)msz) << (8 * ((zf ? zs : n) & 7u));
  }

  R8_STAMP(1);
  // ---------------- 2. unordered_map iteration order (13 buckets) ----------------
  int key[CAP];
  uint32_t bk[CAP];
  const Phase P0 = phase_of(0);
#pragma unroll
  for (int k = 0; k < CAP; k++) {
    key[k] = (int)((KP[k >> 1] >> (16 * (k & 1))) << 21) >> 21;
    bk[k] = bucket_of(key[k], P0);
  }
  uint32_t F[CAP];
#pragma unroll
  for (int k = 0; k < CAP; k++) {
    uint32_t f = (uint32_t)k;
#pragma unroll
    for (int j = k - 1; j >= 0; j--) f = bk[j] == bk[k] ? (uint32_t)j : f;
    F[k] = f;
  }
  uint32_t ord = 0;  // walk position r -> slot, nibble r
#pragma unroll
  for (int k = 0; k < CAP; k++) {
    uint32_t rank = 0;
#pragma unroll
    for (int j = 0; j < CAP; j++) {
      if (j == k) continue;
      const bool before = F[j] > F[k] || (F[j] == F[k] && j > k);
      rank += ((uint32_t)j < n && before) ? 1u : 0u;
    }
    if ((uint32_t)k < n) ord |= (uint32_t)k << (4 * rank);
  }

  R8_STAMP(2);
  // ---------------- 3. Huffman merges on the libstdc++ heap ----------------
  uint32_t H[CAP] = {};
#pragma unroll
  for (int r = 0; r < CAP; r++) {
    if ((uint32_t)r < n) {
      const uint32_t k = (ord >> (4 * r)) & 15u;
      const uint32_t e = (((uint32_t)(cnt >> (8 * k)) & 0xFFu) << 8) | k;
      push<CAP>(H, (uint32_t)r, e);
    }
  }
  uint32_t lpar = 0, ipar = 0;  // parent (merge index) of leaf k / internal j, nibbles
#pragma unroll
  for (int j = 0; j < CAP - 1; j++) {
    if ((uint32_t)j + 1 < n) {
      // the heap holds n - j entries
      const uint32_t l = pop<CAP>(H, n - 1 - (uint32_t)j);
      const uint32_t r = pop<CAP>(H, n - 2 - (uint32_t)j);
#pragma unroll
      for (int s = 0; s < 2; s++) {
        const uint32_t id = (s == 0 ? l : r) & 0xFFu;
        const uint32_t sh = 4 * (id & 7u);
        const uint32_t m = ~(15u << sh), v = (uint32_t)j << sh;
        if (id < 8) lpar = (lpar & m) | v;
        else ipar = (ipar & m) | v;
      }
      push<CAP>(H, n - 2 - (uint32_t)j, ((fq(l) + fq(r)) << 8) | (8u + (uint32_t)j));
    }
  }
  // depths of internal nodes (root = n - 2 at depth 0), then code lengths
  uint32_t dep = 0;
#pragma unroll
  for (int j = CAP - 3; j >= 0; j--) {
    if ((uint32_t)j + 2 < n) {
      const uint32_t par = (ipar >> (4 * j)) & 15u;
      dep |= (((dep >> (4 * par)) & 15u) + 1u) << (4 * j);
    }
  }
  uint32_t len[CAP];
  uint32_t nbits = 0;
  uint64_t lcount = 0;  // 8 x u8 per-length counts
#pragma unroll
  for (int k = 0; k < CAP; k++) {
    const uint32_t par = (lpar >> (4 * k)) & 15u;
    len[k] = n >= 2 ? ((dep >> (4 * par)) & 15u) + 1u : 1u;
    if ((uint32_t)k < n) {
      nbits += ((uint32_t)(cnt >> (8 * k)) & 0xFFu) * len[k];
      lcount += 1ull << (8 * (len[k] - 1));
    }
  }

  R8_STAMP(3);
  // ---------------- 4. canonical order (length, symbol) and codes ----------------
  // (len, key + 1024) << 4 | slot, unused slots last, sorted by a comparator
  // network (u32 min / max): rank r's item names its slot, so the codes and
  // the table are written in rank order
  uint32_t it[CAP];
#pragma unroll
  for (int k = 0; k < CAP; k++)
    it[k] = (uint32_t)k < n ? ((((len[k] << 11) | (uint32_t)(key[k] + 1024)) << 4) | (uint32_t)k)
                            : 0xFFFFFFF0u | (uint32_t)k;
  sort_net<CAP>(it);
  uint64_t fc64 = 0;  // per length: first code
  uint32_t fr32 = 0;            // per length: first canonical rank
  uint32_t table_bytes = 0;
  {
    uint32_t fc = 0, fr = 0;
#pragma unroll
    for (int l = 0; l < 8; l++) {
      const uint32_t c = (uint32_t)(lcount >> (8 * l)) & 0xFFu;
      fc64 |= (uint64_t)(fc & 0xFFu) << (8 * l);
      fr32 |= fr << (4 * l);
      table_bytes += c ? 1 + (c * 11 + 7) / 8 : 0;  // c <= CAP: one group per length
      fc = (fc + c) << 1;
      fr += c;
    }
  }
  uint64_t cc = 0;  // per slot: reversed code (byte k)
  uint32_t ll = 0;  // per slot: length (nibble k)
  uint32_t TK[4] = {0u, 0u, 0u, 0u};  // the table in canonical order: key & 0x7FF | len << 11
#pragma unroll
  for (int r = 0; r < CAP; r++) {
    const uint32_t k = it[r] & 15u, ck = it[r] >> 4;
    const bool used = (uint32_t)r < n;
    const uint32_t ln = used ? ck >> 11 : 1u, L = ln - 1;
    const uint32_t code = (uint32_t)(fc64 >> (8 * L)) + (uint32_t)r - ((fr32 >> (4 * L)) & 15u);
    const uint32_t rcode = hd_brev(code) >> (32 - ln);
    cc |= (uint64_t)(rcode & 0xFFu) << (8 * (k & 7u));  // (an unused rank names an unused slot)
    ll |= (used ? ln : 0u) << (4 * (k & 7u));
    TK[r >> 1] |= ((ck ^ 0x400u) & 0xFFFFu) << (16 * (r & 1));  // key + 1024 -> key & 0x7FF
  }
  S.hdr = nbits | (table_bytes << 16);
  S.size = 3 + table_bytes + (nbits + 7) / 8;
  S.n = n;
  S.msz = (uint32_t)msz;
  S.lcount = lcount;
#pragma unroll
  for (int j = 0; j < 4; j++) S.TK[j] = TK[j];
  S.cc = cc;
  S.ll = ll;
#pragma unroll
  for (int j = 0; j < SlotIds<8>::kRegs; j++) S.ids.r[j] = ids.r[j];
  R8_STAMP(4);
  return true;
}

// The chunk bytes of a built block (Huffman::dump, Huffman.cpp:279-326):
// header, 11-bit table groups (one per code length: <= 8 symbols), code bits
// of the message in position order.  W: DenseWriter (K2's tile run) or a
// host-side writer with the same put / align_byte.
template <class W>
MYYUV_HD void emit_chunk(const EncState& S, int wave_msz, W& bw) {
  bw.put(S.hdr, 24);
  uint32_t curlen = 0;
#pragma unroll
  for (int r = 0; r < 8; r++) {
    if ((uint32_t)r < S.n) {
      const uint32_t kl = (S.TK[r >> 1] >> (16 * (r & 1))) & 0xFFFFu;
      const uint32_t L = kl >> 11;
      if (L != curlen) {
        bw.align_byte();
        const uint32_t c = (uint32_t)(S.lcount >> (8 * (L - 1))) & 0xFFu;
        bw.put(((L - 1) << 5) | (c - 1), 8);
        curlen = L;
      }
      bw.put(kl & 0x7FFu, 11);  // pack11bit
    }
  }
  bw.align_byte();
  // the code bits, four positions (<= 32 bits) per put
#pragma unroll
  for (int i0 = 0; i0 < 64; i0 += 4) {
    if (i0 < wave_msz) {
      uint32_t bits = 0, nb = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int i = i0 + k;
        // (every lane looks its code up; past the message the length is 0)
        const uint32_t sl = S.ids.get(i);
        const uint32_t len = (uint32_t)i < S.msz ? (S.ll >> (4 * sl)) & 15u : 0u;
        bits |= ((uint32_t)(S.cc >> (8 * sl)) & ((1u << len) - 1u)) << nb;
        nb += len;
      }
      bw.put(bits, (int)nb);
    }
  }
}

// K2 block classes: class_of (codec_common.hpp) from the nonzero count and msz.
MYYUV_HD uint32_t block_class(const CoefRegs& R, int msz) {
  uint32_t nnz = 0;
#pragma unroll
  for (int w = 0; w < 32; w++) nnz += ((R.w[w] & 0xFFFFu) != 0) + ((R.w[w] >> 16) != 0);
  return class_of(nnz, (uint32_t)msz);
}

#if defined(__HIP_DEVICE_COMPILE__)
// block_class and CoefRegs::msz on the device in packed 16-bit arithmetic:
// per coefficient pair, the nonzero flags min(v, 1) (v_pk_min_u16), their
// running count (v_pk_add_u16) and the running maximum of flag * (zig-zag
// index + 1) (v_pk_max_u16): five instructions per pair where the scalar
// forms take about ten.  Same results as the host forms.
typedef unsigned short myyuv_us2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void block_class_msz(const CoefRegs& R, int& msz, uint32_t& cls) {
  myyuv_us2 cnt = {0, 0}, mx = {0, 0};
#pragma unroll
  for (int w = 0; w < 32; w++) {
    // (asm: the compiler rewrites min(x, 1) as two compares and selects)
    uint32_t fu;
    asm("v_pk_min_u16 %0, %1, %2" : "=v"(fu) : "v"(R.w[w]), "s"(0x00010001u));
    const myyuv_us2 f = __builtin_bit_cast(myyuv_us2, fu);
    cnt += f;
    // flag * index without the packed multiply (VOP3P takes no literal: its 32
    // index constants would sit in SGPRs): a per-half all-ones mask 0 - flag
    // (asm: the compiler turns it into a 32-bit multiply), then AND with the
    // literal pair
    uint32_t m16;
    asm("v_pk_sub_u16 %0, 0, %1" : "=v"(m16) : "v"(fu));
    mx = __builtin_elementwise_max(mx, __builtin_bit_cast(myyuv_us2, m16 & kZzPairs.v[w]));
  }
  const uint32_t nnz = (uint32_t)cnt.x + (uint32_t)cnt.y;
  const int m = (int)(mx.x > mx.y ? mx.x : mx.y);
  msz = m;
  cls = class_of(nnz, (uint32_t)m);
}
#else
MYYUV_HD void block_class_msz(const CoefRegs& R, int& msz, uint32_t& cls) {
  msz = R.msz();
  cls = block_class(R, msz);
}
#endif

// Blocks whose message is one symbol (msz <= 1: all zero, or the DC
// coefficient alone; Huffman.cpp:191-194 for the all-zero case): one code of
// length 1, one table group; the chunk is 7 bytes:
//   u16 nbits = 1, u8 table_bytes = 3, group header 0x00, 11-bit key, 1 code byte 0.
MYYUV_HD void build_single_dc(int dc, EncState& S) {
  S.hdr = 1u | (3u << 16);
  S.size = 7;
  S.n = 1;
  S.msz = 1;
  S.lcount = 1;
  S.TK[0] = ((uint32_t)dc & 0x7FFu) | (1u << 11);
  S.TK[1] = S.TK[2] = S.TK[3] = 0u;
  S.cc = 0;  // slot 0: code 0,
  S.ll = 1;  // length 1
  S.ids.clear();
}
MYYUV_HD void build_single(const CoefRegs& R, EncState& S) { build_single_dc(R.sym(0), S); }

}  // namespace myyuv_gpu
