// huff_r16.hpp — lane-per-block Huffman code construction for blocks with
// at most 16 distinct symbols, lane per block (the overflow tier behind K2's
// CAP-8 encoder: natural images at q50 put 99.8 % of their overflow blocks
// here, q90 94 %; SURVEY.md §7 hard part 2, App. B).  Same bytes as
// Huffman::fromData + Huffman::dump (myyuv_DCT/Huffman.cpp:172-241, :279-326):
//   1. distinct symbols in first-occurrence order with counts and per-position
//      slots (tagged 12-bit keys, 16 fields in 8 dwords, matched with SWAR);
//   2. std::unordered_map<int16_t,uint8_t>'s iteration order in closed form:
//      front-of-bucket / front-of-list insertion makes the list the bucket
//      runs in decreasing order of their first insertion, each run in
//      decreasing insertion order; 13 buckets up to the 13th key, a rehash to
//      29 buckets before the 14th (or before the freq[0] probe's insert of
//      key 0 into a 13-key map without it), which re-inserts the nodes in list
//      order: the same ordering rule over (previous walk order, later keys);
//      each ordering is two 16-element sorting networks;
//   3. the libstdc++ binary heap (push_heap, pop_heap = __adjust_heap +
//      __push_heap): in the kernel one LDS column per lane (LdsHeap16, the
//      walks as plain per-lane loops, one round trip per level); on the host
//      and as the reference form on 16 registers (RegHeap16: a pop walks the
//      smaller-child path down from the root and merges the old last element
//      back into it, a push merges the new element into its ancestor chain,
//      both as per-position selects over the path positions);
//   4. depths, lengths, canonical order (a sorting network), codes, table;
//   5. emission into the block's 160-B overflow slot.
// Compiled for the host as well (MYYUV_HD) and checked against the oracle on
// the CPU (tools/r8_host.cpp mode "16", tests/test_r8_host.py).
#pragma once
#include "huff_common.hpp"

namespace myyuv_gpu {

namespace r16 {

using rr::fq_gt;

// The slot of the tagged key pair vv among 16 fields (KP[p]: fields 2p, 2p+1):
// per dword, bits 15 / 31 flag equal fields; the 16 flags gathered one per
// byte position (slot s at bit 8 (s & 3) + 7 - (s >> 2)), located with one
// bit scan.
MYYUV_HD bool match16(const uint32_t (&KP)[8], uint32_t vv, uint32_t& slot) {
  uint32_t mp[8];
#pragma unroll
  for (int p = 0; p < 8; p++) mp[p] = ~(((KP[p] ^ vv) | 0x80008000u) - 0x00010001u);
  const uint32_t oh = (hd_perm(mp[1], mp[0], 0x07050301u) & 0x80808080u) |
                      ((hd_perm(mp[3], mp[2], 0x07050301u) & 0x80808080u) >> 1) |
                      ((hd_perm(mp[5], mp[4], 0x07050301u) & 0x80808080u) >> 2) |
                      ((hd_perm(mp[7], mp[6], 0x07050301u) & 0x80808080u) >> 3);
  const uint32_t t = hd_ctz(oh | 0x80000000u);
  slot = (t >> 3) | ((7u - (t & 7u)) << 2);
  return oh != 0;
}

// Nibble k (dynamic) of a 64-bit word.  Packed fields live in scalars, never
// in small local arrays: a select between two elements of a local array is
// folded into a dynamically indexed load, which moves the array to scratch.
MYYUV_HD uint32_t nib(uint64_t w, uint32_t k) { return (uint32_t)(w >> (4 * k)) & 15u; }
MYYUV_HD void nib_or(uint64_t& w, uint32_t k, uint32_t v) { w |= (uint64_t)v << (4 * k); }
MYYUV_HD void nib_set(uint64_t& w, uint32_t k, uint32_t v) {
  w = (w & ~(15ull << (4 * k))) | ((uint64_t)v << (4 * k));
}

// Batcher's odd-even merge sort network for 16 inputs (63 comparators),
// ascending (u32 min / max).
MYYUV_HD void sort16(uint32_t (&a)[16]) {
#pragma unroll
  for (int p = 1; p < 16; p <<= 1)
#pragma unroll
    for (int k = p; k >= 1; k >>= 1)
#pragma unroll
      for (int j = k % p; j + k < 16; j += 2 * k)
#pragma unroll
        for (int i = 0; i < k; i++) {
          if (i + j + k < 16 && (i + j) / (2 * p) == (i + j + k) / (2 * p)) {
            const uint32_t x = a[i + j], y = a[i + j + k];
            a[i + j] = x < y ? x : y;
            a[i + j + k] = x < y ? y : x;
          }
        }
}

// Walk order of the map's list under front-of-bucket / front-of-list
// insertion: items are bkt << 8 | q << 4 | slot for the nodes inserted (q:
// sequence position, distinct), 0xFFFFFFFF for unused entries.  Returns
// ord (nibble r = the slot at list position r) and rank (nibble s = slot s's
// list position).
MYYUV_HD void walk16(uint32_t (&it)[16], uint64_t& ord, uint64_t& rank) {
  sort16(it);  // by bucket, then q
  uint32_t F = 0, prevb = 0xFFFFFFFFu;
#pragma unroll
  for (int r = 0; r < 16; r++) {
    const uint32_t x = it[r];
    const uint32_t b = x >> 8, q = (x >> 4) & 15u;
    F = b != prevb ? q : F;  // the bucket's first insertion
    prevb = b;
    // list order: F descending, then q descending -> ascending on the complement
    it[r] = x == 0xFFFFFFFFu ? 0xFFFFFFFFu : ((((15u - F) << 4) | (15u - q)) << 4) | (x & 15u);
  }
  sort16(it);
  ord = rank = 0;
#pragma unroll
  for (int r = 0; r < 16; r++) {
    const uint32_t s = it[r] & 15u;
    if (it[r] != 0xFFFFFFFFu) {
      nib_or(ord, (uint32_t)r, s);
      nib_or(rank, s, (uint32_t)r);
    }
  }
}

// H[i] for a dynamic i in [0, 16): a select tree over scalars
MYYUV_HD uint32_t hget16(const uint32_t (&H)[16], uint32_t i) {
  const bool b0 = i & 1, b1 = i & 2, b2 = i & 4, b3 = i & 8;
  const uint32_t a0 = b0 ? H[1] : H[0], a1 = b0 ? H[3] : H[2], a2 = b0 ? H[5] : H[4], a3 = b0 ? H[7] : H[6];
  const uint32_t a4 = b0 ? H[9] : H[8], a5 = b0 ? H[11] : H[10], a6 = b0 ? H[13] : H[12], a7 = b0 ? H[15] : H[14];
  const uint32_t c0 = b1 ? a1 : a0, c1 = b1 ? a3 : a2, c2 = b1 ? a5 : a4, c3 = b1 ? a7 : a6;
  const uint32_t d0 = b2 ? c1 : c0, d1 = b2 ? c3 : c2;
  return b3 ? d1 : d0;
}

MYYUV_HD constexpr int depth_of(int k) { return k == 0 ? 0 : k < 3 ? 1 : k < 7 ? 2 : k < 15 ? 3 : 4; }

// std::priority_queue::push of e onto a heap of h entries (h in [0, 15]):
// __push_heap from the hole h — the ancestors of h whose freq exceeds e's
// move down one level, e takes the highest freed position.  Per position k:
// on the chain when k is h or an ancestor of h.
MYYUV_HD void push16(uint32_t (&H)[16], uint32_t h, uint32_t e) {
  uint32_t x[16];
#pragma unroll
  for (int k = 0; k < 16; k++) x[k] = H[k];
  const uint32_t h1 = h + 1;  // 1-based index: an ancestor's index is a prefix of h1's bits
  const uint32_t D = 31u - hd_clz(h1);  // depth of h
  const uint32_t eh = e | 0xFFu;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const uint32_t dk = (uint32_t)depth_of(k);
    const bool chain = D >= dk && (h1 >> (D - dk)) == (uint32_t)k + 1u;
    const bool down = chain && (uint32_t)k != h && x[k] > eh;  // moves down (freq > e's)
    if (k == 0) {
      H[k] = chain && (down || (uint32_t)k == h) ? e : x[k];
    } else {
      const int pk = (k - 1) / 2;
      const bool pdown = chain && x[pk] > eh;  // the parent's entry moves into k
      H[k] = pdown ? x[pk] : (chain && (down || (uint32_t)k == h) ? e : x[k]);
    }
  }
}

// std::priority_queue::pop of a heap of m + 1 entries (m in [1, 15]): returns
// the old top and leaves m entries.  __adjust_heap(first, 0, m, v = H[m])
// walks from the root to the smaller child (the right one unless its freq
// exceeds the left's) while child < (m - 1) / 2, then, for an even m ending
// at child (m - 2) / 2, once more to its left child; every entry on the walk
// moves up one level, and __push_heap puts v back: the walked entries are in
// heap order, so v lands below those whose freq is <= its own.
MYYUV_HD uint32_t pop16(uint32_t (&H)[16], uint32_t m) {
  uint32_t x[16];
#pragma unroll
  for (int k = 0; k < 16; k++) x[k] = H[k];
  const uint32_t top = x[0];
  const uint32_t v = hget16(x, m);
  const uint32_t vh = v | 0xFFu;
  const uint32_t lim = (m - 1) / 2;
  // the walk: path position at depth 1..3 (0: not reached), then the even-m step
  uint32_t p1 = 0, p2 = 0, p3 = 0, ps = 0, last = 0;
  bool on1 = false, on2 = false, on3 = false;
  if (0 < lim) {  // depth 1: children 1, 2
    on1 = true;
    p1 = fq_gt(x[2], x[1]) ? 1u : 2u;
    last = p1;
  }
  if (on1 && p1 < lim) {  // depth 2: children of p1
    on2 = true;
    const uint32_t l = p1 == 1 ? x[3] : x[5], r = p1 == 1 ? x[4] : x[6];
    p2 = 2 * p1 + (fq_gt(r, l) ? 1u : 2u);
    last = p2;
  }
  if (on2 && p2 < lim) {  // depth 3: children of p2 (3..6)
    on3 = true;
    const uint32_t q = p2 - 3;  // 0..3
    const uint32_t l = (q & 2) ? ((q & 1) ? x[13] : x[11]) : ((q & 1) ? x[9] : x[7]);
    const uint32_t r = (q & 2) ? ((q & 1) ? x[14] : x[12]) : ((q & 1) ? x[10] : x[8]);
    p3 = 2 * p2 + (fq_gt(r, l) ? 1u : 2u);
    last = p3;
  }
  const bool spec = (m & 1u) == 0 && last == (m - 2) / 2;  // the even-length edge: left child of `last`
  ps = spec ? 2 * last + 1 : 0u;
  // positions of the walk by depth: 0 (root), then the depth-d step (the
  // loop's or the edge's)
  const uint32_t q1 = on1 ? p1 : (spec ? ps : 0u);
  const bool o1 = on1 || spec;
  const uint32_t q2 = on2 ? p2 : (on1 && spec ? ps : 0u);
  const bool o2 = on2 || (on1 && spec);
  const uint32_t q3 = on3 ? p3 : (on2 && spec ? ps : 0u);
  const bool o3 = on3 || (on2 && spec);
  const uint32_t q4 = on3 && spec ? ps : 0u;
  const bool o4 = on3 && spec;
  // entries walked (E_d = the entry at depth d of the walk); v's level r =
  // the number of walked entries with freq <= v's
  const uint32_t E1 = o1 ? hget16(x, q1) : 0u, E2 = o2 ? hget16(x, q2) : 0u;
  const uint32_t E3 = o3 ? hget16(x, q3) : 0u, E4 = o4 ? hget16(x, q4) : 0u;
  const bool s1 = o1 && E1 <= vh, s2 = s1 && o2 && E2 <= vh, s3 = s2 && o3 && E3 <= vh, s4 = s3 && o4 && E4 <= vh;
  // new values at depths 0..4 of the walk: E_{d+1} moved up while it stays
  // above v, then v, then the rest in place
  const uint32_t n0 = s1 ? E1 : v;
  const uint32_t n1 = s2 ? E2 : (s1 ? v : E1);
  const uint32_t n2 = s3 ? E3 : (s2 ? v : E2);
  const uint32_t n3 = s4 ? E4 : (s3 ? v : E3);
  const uint32_t n4 = s4 ? v : E4;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int d = depth_of(k);
    uint32_t y = x[k];
    if (d == 0) y = n0;
    if (d == 1) y = o1 && q1 == (uint32_t)k ? n1 : y;
    if (d == 2) y = o2 && q2 == (uint32_t)k ? n2 : y;
    if (d == 3) y = o3 && q3 == (uint32_t)k ? n3 : y;
    if (d == 4) y = o4 && q4 == (uint32_t)k ? n4 : y;
    H[k] = y;
  }
  return top;
}

// The heap of build_r16 on 16 registers (push16 / pop16): the host build
// and the reference for LdsHeap16.
struct RegHeap16 {
  uint32_t H[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  MYYUV_HD void push(uint32_t h, uint32_t e) { push16(H, h, e); }
  MYYUV_HD uint32_t pop(uint32_t m) { return pop16(H, m); }
};

// The same heap as a column of LDS per lane: entry k of lane l's heap at
// word k * S + l.  Every access of a wave is conflict-free whatever each
// lane's k (bank = lane), so the walks are plain per-lane loops (libstdc++'s
// __push_heap / __adjust_heap, strict comparisons on the freq), one LDS
// round trip per level, instead of push16 / pop16's selects over all 16
// positions at every step (425 / 975 instructions per push / merge step).
template <uint32_t S>
struct LdsHeap16 {
  uint32_t* c;  // &lds[lane]
  MYYUV_HD uint32_t& at(uint32_t k) const { return c[k * S]; }
  // __push_heap(first, hole h, top 0, e): parents whose freq exceeds e's move down
  MYYUV_HD void push(uint32_t h, uint32_t e) const {
    const uint32_t eh = e | 0xFFu;
    uint32_t hole = h;
    while (hole > 0) {
      const uint32_t p = (hole - 1u) >> 1;
      const uint32_t pe = at(p);
      if (pe <= eh) break;
      at(hole) = pe;
      hole = p;
    }
    at(hole) = e;
  }
  // pop_heap of a heap of m + 1 entries: __adjust_heap(first, 0, m, last),
  // then __push_heap of the old last entry from the hole
  MYYUV_HD uint32_t pop(uint32_t m) const {
    const uint32_t top = at(0);
    if (m == 0) return top;  // (one entry: nothing moves)
    const uint32_t v = at(m);
    uint32_t hole = 0, child = 0;
    const uint32_t lim = (m - 1u) >> 1;
    while (child < lim) {
      child = 2u * (child + 1u);
      const uint32_t r = at(child), l = at(child - 1u);
      const bool left = fq_gt(r, l);
      child -= left ? 1u : 0u;
      at(hole) = left ? l : r;
      hole = child;
    }
    if ((m & 1u) == 0 && child == (m - 2u) >> 1) {
      child = 2u * (child + 1u);
      at(hole) = at(child - 1u);
      hole = child - 1u;
    }
    push(hole, v);
    return top;
  }
};

}  // namespace r16

// What emit_chunk16 needs of a block whose code was built by build_r16.
struct EncState16 {
  uint32_t hdr, size, n, msz;
  uint64_t lcount;   // per code length L: symbols of that length (byte L - 1)
  uint32_t TK[8];    // table in canonical order: entry r = key & 0x7FF | len << 11 (16-bit fields)
  uint64_t cc0, cc1; // per slot k: its bit-reversed code in byte k & 7 of cc0 (k < 8) / cc1
  uint64_t ll;       // per slot k: its code length in nibble k
  SlotIds<16> ids;   // per position: slot of its symbol
};

// Returns false when the block has more than 16 distinct symbols.  Heap:
// r16::RegHeap16 or (device) r16::LdsHeap16.
template <class Heap = r16::RegHeap16>
MYYUV_HD bool build_r16(const CoefRegs& R, int msz, int wave_msz, EncState16& S, Heap hp = Heap()) {
  using namespace r16;
  // ---------------- 1. distinct symbols, counts, per-position slots ----------------
  uint32_t KP[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // tagged keys, field k = slot k
  uint64_t cnt0 = 0, cnt1 = 0;               // count of slot k in byte k & 7 of cnt0 (k < 8) / cnt1
  uint32_t n = 0;
  SlotIds<16> ids;
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
        uint32_t sl;
        const bool found = match16(KP, f | (f << 16), sl);
        const bool add = act && !found;
        const bool ins = add && n < 16;
        sl = found ? sl : n;
        // the new key into field n: a 64-bit shift into the dword pair
        // holding fields (n & ~3) .. (n | 3)
        const uint64_t t64 = (uint64_t)(ins ? f : 0u) << (16 * (n & 3u));
        const uint32_t pr = (n >> 2) & 3u;
#pragma unroll
        for (int q = 0; q < 4; q++) {
          KP[2 * q] |= pr == (uint32_t)q ? (uint32_t)t64 : 0u;
          KP[2 * q + 1] |= pr == (uint32_t)q ? (uint32_t)(t64 >> 32) : 0u;
        }
        // every processed position is counted; the zeros past the message
        // are taken off below
        const uint64_t one = 1ull << (8 * (sl & 7u));
        cnt0 += (sl & 8u) ? 0ull : one;
        cnt1 += (sl & 8u) ? one : 0ull;
        n += add ? 1u : 0u;
        ids.set(i, sl & 15u);
      }
    }
  }
  if (n > 16u) return false;
  uint32_t zs;
  bool has_zero = match16(KP, 0x08000800u, zs);
  if (msz == 0) {  // all-zero block: one symbol 0, count 1 (Huffman.cpp:191-194)
    KP[0] = 0x800u;
    cnt0 = 1;
    cnt1 = 0;
    n = 1;
    msz = 1;
    has_zero = true;
    zs = 0;
  } else {
    // positions msz .. P - 1 (P: the positions the loop ran) are zeros:
    // counted into the zero's slot, or into slot n & 15 when the message has
    // no zero (unused; n = 16 wraps to slot 0)
    const uint32_t P = (uint32_t)min((wave_msz + kPosGroup - 1) / kPosGroup * kPosGroup, 64);
    const uint32_t s = (has_zero ? zs : n) & 15u;
    const uint64_t sub = (uint64_t)(P - (uint32_t)msz) << (8 * (s & 7u));
    cnt0 -= (s & 8u) ? 0ull : sub;
    cnt1 -= (s & 8u) ? sub : 0ull;
  }
  // ---------------- 2. unordered_map iteration order ----------------
  int key[16];
#pragma unroll
  for (int k = 0; k < 16; k++) key[k] = (int)((KP[k >> 1] >> (16 * (k & 1))) << 21) >> 21;
  uint64_t ord, rank;
  {
    const Phase P0 = phase_of(0);
    uint32_t it[16];
#pragma unroll
    for (int k = 0; k < 16; k++)
      it[k] = (uint32_t)k < n && k < 13 ? (bucket_of(key[k], P0) << 8) | ((uint32_t)k << 4) | (uint32_t)k
                                        : 0xFFFFFFFFu;
    walk16(it, ord, rank);
  }
  // a rehash to 29 buckets before the 14th insert, or before the freq[0]
  // probe inserts key 0 into a 13-key map without it (Huffman.cpp:186-197;
  // the probe's node is erased again, the rehash stays)
  if (n >= 14 || (n == 13 && !has_zero)) {
    const Phase P1 = phase_of(1);
    uint32_t it[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint32_t q = k < 13 ? nib(rank, (uint32_t)k) : (uint32_t)k;
      it[k] = (uint32_t)k < n ? (bucket_of(key[k], P1) << 8) | (q << 4) | (uint32_t)k : 0xFFFFFFFFu;
    }
    walk16(it, ord, rank);
  }
  // ---------------- 3. Huffman merges on the libstdc++ heap ----------------
#pragma unroll 1
  for (uint32_t r = 0; r < n; r++) {
    const uint32_t k = nib(ord, r);
    const uint32_t cv = (uint32_t)(((k & 8u) ? cnt1 : cnt0) >> (8 * (k & 7u))) & 0xFFu;
    hp.push(r, (cv << 8) | k);
  }
  uint64_t lpar = 0, ipar = 0;  // parent (merge index) of leaf k / internal j, nibbles
#pragma unroll 1
  for (uint32_t j = 0; j + 1 < n; j++) {
    const uint32_t l = hp.pop(n - 1 - j);
    const uint32_t r = hp.pop(n - 2 - j);
#pragma unroll
    for (int s = 0; s < 2; s++) {
      const uint32_t id = (s == 0 ? l : r) & 0xFFu;
      if (id < 16) nib_set(lpar, id, j);
      else nib_set(ipar, id - 16, j);
    }
    hp.push(n - 2 - j, ((rr::fq(l) + rr::fq(r)) << 8) | (16u + j));
  }
  // depths of internal nodes (root = n - 2 at depth 0), then code lengths
  uint64_t dep = 0;
#pragma unroll
  for (int j = 13; j >= 0; j--) {
    if ((uint32_t)j + 2 < n) nib_or(dep, (uint32_t)j, nib(dep, nib(ipar, (uint32_t)j)) + 1u);
  }
  uint32_t len[16];
  uint32_t nbits = 0;
  uint64_t lcount = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    len[k] = n >= 2 ? nib(dep, nib(lpar, (uint32_t)k)) + 1u : 1u;
    if ((uint32_t)k < n) {
      const uint32_t cv = (uint32_t)((k < 8 ? cnt0 : cnt1) >> (8 * (k & 7))) & 0xFFu;
      nbits += cv * len[k];
      lcount += 1ull << (8 * ((len[k] - 1) & 7u));
    }
  }
  // ---------------- 4. canonical order (length, symbol) and codes ----------------
  uint32_t it[16];
#pragma unroll
  for (int k = 0; k < 16; k++)
    it[k] = (uint32_t)k < n ? ((((len[k] << 11) | (uint32_t)(key[k] + 1024)) << 4) | (uint32_t)k)
                            : 0xFFFFFFF0u | (uint32_t)k;
  sort16(it);
  uint64_t fc64 = 0, fr64 = 0;  // per length: first code, first canonical rank (bytes)
  uint32_t table_bytes = 0;
  {
    uint32_t fc = 0, fr = 0;
#pragma unroll
    for (int l = 0; l < 8; l++) {
      const uint32_t c = (uint32_t)(lcount >> (8 * l)) & 0xFFu;
      fc64 |= (uint64_t)(fc & 0xFFu) << (8 * l);
      fr64 |= (uint64_t)fr << (8 * l);
      table_bytes += c ? 1 + (c * 11 + 7) / 8 : 0;  // c <= 16: one group per length
      fc = (fc + c) << 1;
      fr += c;
    }
  }
  uint64_t cc0 = 0, cc1 = 0, ll = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) S.TK[j] = 0;
#pragma unroll
  for (int r = 0; r < 16; r++) {
    const uint32_t k = it[r] & 15u, ck = it[r] >> 4;
    const bool used = (uint32_t)r < n;
    const uint32_t ln = used ? ck >> 11 : 1u, L = (ln - 1) & 7u;
    const uint32_t code = (uint32_t)(fc64 >> (8 * L)) + (uint32_t)r - ((uint32_t)(fr64 >> (8 * L)) & 0xFFu);
    const uint32_t rcode = hd_brev(code) >> (32 - ln);
    const uint64_t cbyte = used ? (uint64_t)(rcode & 0xFFu) << (8 * (k & 7u)) : 0ull;
    cc0 |= (k & 8u) ? 0ull : cbyte;
    cc1 |= (k & 8u) ? cbyte : 0ull;
    if (used) nib_or(ll, k, ln);
    S.TK[r >> 1] |= used ? ((ck ^ 0x400u) & 0xFFFFu) << (16 * (r & 1)) : 0u;  // key + 1024 -> key & 0x7FF
  }
  S.cc0 = cc0;
  S.cc1 = cc1;
  S.ll = ll;
  S.hdr = nbits | (table_bytes << 16);
  S.size = 3 + table_bytes + (nbits + 7) / 8;
  S.n = n;
  S.msz = (uint32_t)msz;
  S.lcount = lcount;
#pragma unroll
  for (int j = 0; j < SlotIds<16>::kRegs; j++) S.ids.r[j] = ids.r[j];
  return true;
}

// The chunk bytes of a block built by build_r16 (Huffman::dump): header,
// 11-bit table groups (one per code length: <= 16 symbols), code bits in
// position order.  W: BitWriter (the overflow slot) or a host writer.
template <class W>
MYYUV_HD void emit_chunk16(const EncState16& S, int wave_msz, W& bw) {
  bw.put(S.hdr, 24);
  uint32_t curlen = 0;
#pragma unroll
  for (int r = 0; r < 16; r++) {
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
#pragma unroll
  for (int i0 = 0; i0 < 64; i0 += 4) {
    if (i0 < wave_msz) {
      uint32_t bits = 0, nb = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int i = i0 + k;
        const uint32_t sl = S.ids.get(i);
        const uint32_t len = (uint32_t)i < S.msz ? r16::nib(S.ll, sl) : 0u;
        const uint32_t code = (uint32_t)(((sl & 8u) ? S.cc1 : S.cc0) >> (8 * (sl & 7u))) & ((1u << len) - 1u);
        bits |= code << nb;
        nb += len;
      }
      bw.put(bits, (int)nb);
    }
  }
}

}  // namespace myyuv_gpu
