// k_huff_encode.hip — K2: per-block Huffman code construction and chunk
// serialisation for gfx950 (Huffman::fromData + Huffman::dump,
// myyuv_DCT/Huffman.cpp:172-241, :279-326).
//
// One lane = one 8x8 block, one wave = 64 consecutive blocks.  The per-block
// program is short and serial (a few distinct symbols in natural images), so
// a lane per block amortises every instruction over 64 blocks; what limits it
// is LDS latency, hence a small per-lane LDS image (64 B for the CAP=8 pass:
// 32 waves per CU) and no pointer chasing on the per-symbol path:
//   1. distinct symbols of the message (zig-zag order, trailing zeros
//      stripped) in first-occurrence order with counts,
//      found through a small open-addressing table (slot ids) -> KC;
//   2. replay of std::unordered_map's iteration order over KC, libstdc++
//      binary-heap Huffman merges, code lengths, canonical order and codes;
//   3. serialisation (header, 11-bit table groups, code bits) into the
//      block's 160-B output slot.
// Coefficients come in K1's natural-order quad layout (codec_common.hpp): a
// lane loads its block's 8 quads (the wave reads 1 KiB contiguous per quad)
// into 32 registers; the zig-zag scan (Huffman.cpp:32-34, :176-182) is the
// compile-time permutation behind CoefRegs::sym(), and the message length
// (trailing zig-zag zeros stripped, Huffman.cpp:184-190) is found the same way.
// CAP bounds the distinct symbols: the CAP=8 pass runs on every block and
// appends the blocks with more to a worklist that the CAP=64 pass drains.
//
// Byte-exactness: the code lengths depend on libstdc++ container internals
// (SURVEY.md §7 hard part 2, App. B), replayed exactly:
//   * std::unordered_map<int16_t,uint8_t> iteration order: singly linked list
//     with per-bucket "before" pointers, bucket-front insertion, rehash walk,
//     prime policy 13 -> 29 -> 59 -> 127 buckets, hash(v) = (uint64)(int64)v.
//     KC holds the keys in first-occurrence order = operator[]'s insertion
//     order (Huffman.cpp:176-183);
//   * the freq[0] probe (Huffman.cpp:186-197) inserts key 0 after the message
//     symbols and erases it again: only the rehash it may trigger is visible;
//   * std::priority_queue (min-heap via Compare{a.freq > b.freq}): libstdc++
//     push_heap / pop_heap (__adjust_heap + __push_heap) exactly.
//
// Per-lane LDS image (lane-interleaved words: word w of lane l at w*64 + l,
// conflict-free for any per-lane index):
//   KC[CAP]  key:11 | cnt:7 | next:7 | bkt:7 (map phase); key:11 | cnt:7 |
//            len:4 | rcode:8 afterwards; during the heap phase bits 18..24
//            hold a leaf's parent.
//   T        open-addressing table, 2*CAP u8 entries = slot+1 (0 = empty).
//   SH       scratch: bucket before-pointers (u8) in the map replay, then the
//            heap (u16 freq<<8 | id; internal node k keeps depth<<8 | parent in
//            slot CAP-1-k), then the canonical order (u8).
#include "codec_common.hpp"
#ifdef MYYUV_STAMPS
namespace myyuv_gpu {
extern __device__ uint32_t g_k2_fstamps[8192 * 8];
}
#define R8_STAMP_DECL unsigned long long _r8prev = 0;
#define R8_STAMP(k)                                                                   \
  do {                                                                                \
    __builtin_amdgcn_sched_barrier(0);                                                \
    unsigned long long _t = __builtin_amdgcn_s_memtime();                             \
    __builtin_amdgcn_sched_barrier(0);                                                \
    if ((threadIdx.x & 63) == 0 && (k) > 0 && blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6) < 8192) \
      g_k2_fstamps[(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8 + (k)] = (uint32_t)(_t - _r8prev); \
    _r8prev = _t;                                                                     \
  } while (0)
#endif
#include "huff_common.hpp"
#include "huff_r16.hpp"
#include "xform_common.hpp"

namespace myyuv_gpu {

#ifdef MYYUV_STAMPS
// diagnostic build only: per-stage wave cycles — [0..7] fast pass summed
// over waves, [8..15] wide pass summed, [16..23] wide pass max over waves
__device__ unsigned long long g_k2_stamps[40];
// per-wave stage cycles of the CAP=8 pass (plain stores: contended atomics
// would distort the timing): g_k2_fstamps[wave][8]
__device__ uint32_t g_k2_fstamps[8192 * 8];
#define STAMP(k)                                                                     \
  do {                                                                               \
    __builtin_amdgcn_sched_barrier(0);                                               \
    unsigned long long _t = __builtin_amdgcn_s_memtime();                            \
    __builtin_amdgcn_sched_barrier(0);                                               \
    if (threadIdx.x == 0 && (k) > 0) {                                               \
      if (CAP == 8) {                                                                \
        if (blockIdx.x < 8192) g_k2_fstamps[blockIdx.x * 8 + (k)] = (uint32_t)(_t - _tprev); \
      } else {                                                                       \
        atomicAdd(&g_k2_stamps[(k) + 8], _t - _tprev);                               \
        atomicMax(&g_k2_stamps[(k) + 16], _t - _tprev);                              \
      }                                                                              \
    }                                                                                \
    _tprev = _t;                                                                     \
  } while (0)
// K2's window phases per wave: [6] tiles and the block words' arrival,
// [5] classification,
// [0] the rest of the prologue (count scan, sort, three barriers),
// [1] runs' fetch + load + build, [2] runs' emission and lists, [3] runs,
// [4] the last fetch + epilogue, [7] = 1 (g_k2_win[wave][8])
__device__ uint32_t g_k2_win[65536 * 8];
#define KWSTAMP(k)                                                                   \
  do {                                                                               \
    __builtin_amdgcn_sched_barrier(0);                                               \
    unsigned long long _t = __builtin_amdgcn_s_memtime();                            \
    __builtin_amdgcn_sched_barrier(0);                                               \
    _kw[(k)] += (uint32_t)(_t - _kwprev);                                            \
    _kwprev = _t;                                                                    \
  } while (0)
// wave encoder: per-block phase cycles into g_k2_wstamps[block slot][8]
// (plain stores: contended atomics would distort the timing)
__device__ uint32_t g_k2_wstamps[65536 * 8];
#define WSTAMP(k)                                                                    \
  do {                                                                               \
    __builtin_amdgcn_sched_barrier(0);                                               \
    unsigned long long _t = __builtin_amdgcn_s_memtime();                            \
    __builtin_amdgcn_sched_barrier(0);                                               \
    if (threadIdx.x == 0 && (k) > 0 && _wslot < 65536)                               \
      g_k2_wstamps[_wslot * 8 + (k)] = (uint32_t)(_t - _wprev);                      \
    _wprev = _t;                                                                     \
  } while (0)
#else
#define WSTAMP(k) \
  do {            \
  } while (0)
#define STAMP(k) \
  do {           \
  } while (0)
#endif

namespace {

constexpr uint32_t kNil = 127;     // next-pointer "null"
__constant__ uint8_t c_zz_lane[64] = MYYUV_ZIGZAG;
constexpr uint32_t kEmpty = 0x80;  // bucket has no before-pointer
constexpr uint32_t kHead = 0x7F;   // before-pointer = list head sentinel

template <int CAP>
struct Layout {
  static constexpr int kBuckets = CAP <= 12 ? 13 : 127;  // CAP <= 12 never rehashes
  static constexpr int kTEntries = 2 * CAP;
  static constexpr int kKC = 0;
  static constexpr int kT = CAP;
  static constexpr int kTWords = (kTEntries + 3) / 4;
  static constexpr int kSH = kT + kTWords;
  static constexpr int kShWords = (CAP / 2 > (kBuckets + 3) / 4) ? CAP / 2 : (kBuckets + 3) / 4;
  static constexpr int kWords = kSH + kShWords;
};

template <int CAP>
struct Img {
  uint32_t* base;
  int lane;
  __device__ __forceinline__ uint32_t& kc(int j) const { return base[(Layout<CAP>::kKC + j) * kWideLanes + lane]; }
  __device__ __forceinline__ uint32_t& wordAt(int w) const { return base[w * kWideLanes + lane]; }
  __device__ __forceinline__ uint8_t& t8(int i) const {
    return *(reinterpret_cast<uint8_t*>(base) + ((Layout<CAP>::kT + (i >> 2)) * kWideLanes + lane) * 4 + (i & 3));
  }
  __device__ __forceinline__ uint8_t& sh8(int i) const {
    return *(reinterpret_cast<uint8_t*>(base) + ((Layout<CAP>::kSH + (i >> 2)) * kWideLanes + lane) * 4 + (i & 3));
  }
  __device__ __forceinline__ uint16_t& sh16(int i) const {
    return *reinterpret_cast<uint16_t*>(reinterpret_cast<uint8_t*>(base) +
                                        ((Layout<CAP>::kSH + (i >> 1)) * kWideLanes + lane) * 4 + (i & 1) * 2);
  }
};

__device__ __forceinline__ int nkey(uint32_t w) { return (int)(w << 21) >> 21; }
__device__ __forceinline__ uint32_t ncnt(uint32_t w) { return (w >> 11) & 127u; }
__device__ __forceinline__ uint32_t nnext(uint32_t w) { return (w >> 18) & 127u; }
__device__ __forceinline__ uint32_t nbkt(uint32_t w) { return w >> 25; }
__device__ __forceinline__ uint32_t set_next(uint32_t w, uint32_t nx) {
  return (w & ~(127u << 18)) | (nx << 18);
}

// Slot lookup in the open-addressing table (any hash works here: it only
// finds a symbol's KC slot; the libstdc++ order is replayed separately).
template <int CAP>
__device__ __forceinline__ uint32_t thash(int v) {
  constexpr int bits = CAP == 8 ? 4 : (CAP == 16 ? 5 : 7);
  return ((uint32_t)(v + 1024) * 0x9E3779B1u) >> (32 - bits);
}

// _M_insert_bucket_begin(bkt, node)
template <int CAP>
__device__ __forceinline__ void insert_bucket_begin(const Img<CAP>& I, uint32_t& head, uint32_t b,
                                                    uint32_t node, uint32_t nodeword) {
  const uint32_t before = I.sh8(b);
  if (before != kEmpty) {
    if (before == kHead) {
      I.kc(node) = set_next(nodeword, head);
      head = node;
    } else {
      const uint32_t bw = I.kc(before);
      I.kc(node) = set_next(nodeword, nnext(bw));
      I.kc(before) = set_next(bw, node);
    }
  } else {
    I.kc(node) = set_next(nodeword, head);
    if (head != kNil) I.sh8(nbkt(I.kc(head))) = (uint8_t)node;
    head = node;
    I.sh8(b) = (uint8_t)kHead;
  }
}

template <int CAP>
__device__ __forceinline__ void clear_buckets(const Img<CAP>& I, uint32_t nb) {
  for (uint32_t w = 0; w < (nb + 3) / 4; w++) I.wordAt(Layout<CAP>::kSH + w) = 0x80808080u;
}

// _M_rehash_aux(nb, true_type): re-insert every node in list order.
template <int CAP>
__device__ __forceinline__ void rehash(const Img<CAP>& I, uint32_t& head, const Phase& P) {
  clear_buckets(I, P.nb);
  uint32_t p = head;
  head = kNil;
  uint32_t bbegin = 0;
  while (p != kNil) {
    const uint32_t w = I.kc(p);
    const uint32_t nx = nnext(w);
    const uint32_t b = bucket_of(nkey(w), P);
    const uint32_t before = I.sh8(b);
    uint32_t newnext;
    if (before == kEmpty) {
      newnext = head;
      head = p;
      I.sh8(b) = (uint8_t)kHead;
      if (newnext != kNil) I.sh8(bbegin) = (uint8_t)p;
      bbegin = b;
    } else if (before == kHead) {
      newnext = head;
      head = p;
    } else {
      const uint32_t bw = I.kc(before);
      newnext = nnext(bw);
      I.kc(before) = set_next(bw, p);
    }
    I.kc(p) = (w & 0x0003FFFFu) | (newnext << 18) | (b << 25);
    p = nx;
  }
}

// std::priority_queue push: push_back + __push_heap (sift up while
// parent.freq > value.freq).
template <int CAP>
__device__ __forceinline__ void heap_sift_up(const Img<CAP>& I, int hole, uint32_t e) {
  while (hole > 0) {
    const int parent = (hole - 1) >> 1;
    const uint32_t pe = I.sh16(parent);
    if ((pe >> 8) <= (e >> 8)) break;
    I.sh16(hole) = (uint16_t)pe;
    hole = parent;
  }
  I.sh16(hole) = (uint16_t)e;
}

// std::priority_queue pop: top + pop_heap (__pop_heap, __adjust_heap).
template <int CAP>
__device__ __forceinline__ uint32_t heap_pop(const Img<CAP>& I, int& len) {
  const uint32_t top = I.sh16(0);
  const int n = --len;
  if (n > 0) {
    const uint32_t value = I.sh16(n);
    int hole = 0, child = 0;
    while (child < (n - 1) / 2) {
      child = 2 * (child + 1);
      const uint32_t right = I.sh16(child), left = I.sh16(child - 1);
      uint32_t pick = right;
      if ((right >> 8) > (left >> 8)) {
        child--;
        pick = left;
      }
      I.sh16(hole) = (uint16_t)pick;
      hole = child;
    }
    if ((n & 1) == 0 && child == (n - 2) / 2) {
      child = 2 * (child + 1);
      I.sh16(hole) = I.sh16(child - 1);
      hole = child - 1;
    }
    heap_sift_up(I, hole, value);
  }
  return top;
}

// The whole per-block program.  Returns false (and writes nothing) when the
// block has more than CAP distinct symbols.
template <int CAP>
__device__ __forceinline__ bool encode_block(const Img<CAP>& I, const CoefRegs& R, int msz, int wave_msz,
                             uint32_t* __restrict__ slot, uint8_t* __restrict__ size_out) {
#ifdef MYYUV_STAMPS
  unsigned long long _tprev = 0;
#endif
  STAMP(0);
  // ---------------- 1. distinct symbols in first-occurrence order ----------------
#pragma unroll
  for (int w = 0; w < Layout<CAP>::kTWords; w++) I.wordAt(Layout<CAP>::kT + w) = 0u;
  int n = 0;
  bool has_zero = false, ovf = false;
  SlotIds<CAP> ids;
  ids.clear();
  // Positions are visited with a static index (R.sym(i) must stay a register
  // read), in groups of 8 behind one wave-uniform test of the wave's msz.
#pragma unroll
  for (int i0 = 0; i0 < 64; i0 += 8) {
    if (i0 < wave_msz) {
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int i = i0 + k;
        const int v = R.sym(i);
        if (i < msz && !ovf) {
          has_zero |= (v == 0);
          uint32_t h = thash<CAP>(v);
          uint32_t slot = 0;
          while (true) {
            const uint32_t e = I.t8(h);
            if (e == 0) {
              if (n == CAP) {
                ovf = true;
              } else {
                I.t8(h) = (uint8_t)(n + 1);
                I.kc(n) = ((uint32_t)v & 0x7FFu) | (1u << 11);
                slot = (uint32_t)n;
                n++;
              }
              break;
            }
            const uint32_t kw = I.kc(e - 1);
            if (nkey(kw) == v) {
              I.kc(e - 1) = kw + (1u << 11);
              slot = e - 1;
              break;
            }
            h = (h + 1) & (Layout<CAP>::kTEntries - 1);
          }
          ids.set(i, slot);
        }
      }
    }
  }
  if (ovf) return false;
  if (msz == 0) {  // all-zero block: one symbol 0, count 1 (Huffman.cpp:191-194)
    I.kc(0) = 1u << 11;
    I.t8(thash<CAP>(0)) = 1;
    n = 1;
    msz = 1;
    has_zero = true;
  }
  STAMP(1);

  // ---------------- 2. unordered_map order, heap, lengths, codes ----------------
  uint32_t head = kNil;
  int ph = 0;
  Phase P = phase_of(0);
  clear_buckets(I, Layout<CAP>::kBuckets == 13 ? 13 : 13);
  for (int j = 0; j < n; j++) {
    if (Layout<CAP>::kBuckets > 13 && j == (int)P.nb) {  // rehash before the (nb+1)-th insert
      ph++;
      P = phase_of(ph);
      rehash(I, head, P);
    }
    const uint32_t w = I.kc(j);
    const uint32_t b = bucket_of(nkey(w), P);
    insert_bucket_begin(I, head, b, (uint32_t)j, (w & 0x3FFFFu) | (b << 25));
  }
  if (Layout<CAP>::kBuckets > 13 && !has_zero && n == (int)P.nb) {  // the freq[0] probe's rehash
    ph++;
    P = phase_of(ph);
    rehash(I, head, P);
  }
  STAMP(2);

  int hlen = 0;
  for (uint32_t p = head; p != kNil;) {
    const uint32_t w = I.kc(p);
    heap_sift_up(I, hlen++, (ncnt(w) << 8) | p);
    p = nnext(w);
  }
  for (int k = 0; k + 1 < n; k++) {
    const uint32_t l = heap_pop(I, hlen);
    const uint32_t r = heap_pop(I, hlen);
    const uint32_t ids[2] = {l & 0xFF, r & 0xFF};
#pragma unroll
    for (int s = 0; s < 2; s++) {
      const uint32_t id = ids[s];
      if (id < 64) I.kc(id) = set_next(I.kc(id), (uint32_t)k);
      else I.sh16(CAP - 1 - (int)(id - 64)) = (uint16_t)k;
    }
    heap_sift_up(I, hlen++, (((l >> 8) + (r >> 8)) << 8) | (uint32_t)(64 + k));
  }
  if (n >= 2) {  // depths (generateCodeLength, Huffman.cpp:71-83); root = internal n-2
    const int root = n - 2;
    I.sh16(CAP - 1 - root) = 0;
    for (int k = root - 1; k >= 0; k--) {
      const uint32_t par = I.sh16(CAP - 1 - k) & 0xFF;
      const uint32_t d = (I.sh16(CAP - 1 - (int)par) >> 8) + 1;
      I.sh16(CAP - 1 - k) = (uint16_t)(par | (d << 8));
    }
  }
  uint32_t nbits = 0;
  uint64_t lcount = 0;  // 8 x u8 per-length counts
  for (int p = 0; p < n; p++) {
    const uint32_t w = I.kc(p);
    uint32_t len = 1;
    if (n >= 2) len = (I.sh16(CAP - 1 - (int)nnext(w)) >> 8) + 1;
    nbits += ncnt(w) * len;
    lcount += 1ull << (8 * (len - 1));
    I.kc(p) = (w & 0x3FFFFu) | (len << 18);
  }
  STAMP(3);
  // canonical order (length, symbol): slot p goes to SH (u8) position
  // rank(p) = #{q : key(q) < key(p)} (keys are distinct).  The ranks are
  // independent of one another, so the LDS reads pipeline, where an
  // insertion sort is one chain of dependent round trips.
  for (int p = 0; p < n; p++) {
    const uint32_t wp = I.kc(p);
    const uint32_t kp = (((wp >> 18) & 15u) << 11) | (uint32_t)(nkey(wp) + 1024);
    uint32_t r = 0;
    for (int q = 0; q < n; q++) {
      const uint32_t wq = I.kc(q);
      const uint32_t kq = (((wq >> 18) & 15u) << 11) | (uint32_t)(nkey(wq) + 1024);
      r += kq < kp ? 1u : 0u;
    }
    I.sh8((int)r) = (uint8_t)p;
  }
  STAMP(4);

  // ---------------- 3. chunk bytes (Huffman.cpp:279-326) ----------------
  uint32_t table_bytes = 0;
#pragma unroll
  for (int l = 0; l < 8; l++) {
    const uint32_t c = (uint32_t)(lcount >> (8 * l)) & 0xFF;
    if (c > 32) table_bytes += 2 + 44 + ((c - 32) * 11 + 7) / 8;
    else if (c > 0) table_bytes += 1 + (c * 11 + 7) / 8;
  }
  BitWriter bw;
  bw.out = slot;
  bw.put(nbits, 16);
  bw.put(table_bytes, 8);
  uint32_t code = 0, prevlen = 0, curlen = 0, left = 0, ingroup = 0;
  for (int r = 0; r < n; r++) {
    const uint32_t p = I.sh8(r);
    const uint32_t w = I.kc(p);
    const uint32_t len = (w >> 18) & 15u;
    if (len != curlen || ingroup == 32) {
      if (len != curlen) {
        left = (uint32_t)(lcount >> (8 * (len - 1))) & 0xFF;
        curlen = len;
      }
      bw.align_byte();
      const uint32_t gsz = left < 32 ? left : 32;
      bw.put(((len - 1) << 5) | (gsz - 1), 8);
      left -= gsz;
      ingroup = 0;
    }
    bw.put((uint32_t)nkey(w) & 0x7FFu, 11);  // pack11bit: 2048 + v for v < 0
    ingroup++;
    // canonical code (generateCanonicalTree, Huffman.cpp:86-103), stored
    // bit-reversed so the LSB-first writer emits it MSB-first
    code <<= (len - prevlen);
    prevlen = len;
    const uint32_t rcode = __brev(code) >> (32 - len);
    I.kc(p) = (w & 0x3FFFFu) | (len << 18) | (rcode << 22);
    code++;
  }
  bw.align_byte();
#pragma unroll
  for (int i0 = 0; i0 < 64; i0 += 8) {
    if (i0 < wave_msz) {
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int i = i0 + k;
        if (i < msz) {
          const uint32_t w = I.kc((int)ids.get(i));
          bw.put(w >> 22, (int)((w >> 18) & 15u));
        }
      }
    }
  }
  bw.flush();
  *size_out = (uint8_t)(3 + table_bytes + (nbits + 7) / 8);
  STAMP(5);
  return true;
}

template <int W = 64>
__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int d = 1; d < W; d <<= 1) v = max(v, __shfl_xor(v, d, W));
  return v;
}

// ---------------------------------------------------------------------------
// Wave-per-block encoder for short overflow worklists (natural images: a few
// percent of blocks have more than 8 distinct symbols).  In the lane-per-block
// pass such a wave is one long chain of dependent LDS round trips (heap
// merges, insertion sort, map replay), and a few hundred waves leave the chip
// idle.  Here one wave encodes one block: lanes are the block's positions /
// distinct symbols / heap slots, every order-independent step is lane
// parallel (distinct symbols by ballot, map order and canonical order by
// rank counting, code bits by prefix sum), and the inherently sequential
// steps (heap merges, depth chain) run as uniform control over
// lane-distributed arrays: a v_readlane / v_writelane per step instead of an
// LDS round trip.  Same byte output as encode_block (same libstdc++ replay):
//   * unordered_map iteration order in closed form: with front-of-bucket /
//     front-of-list insertion (_M_insert_bucket_begin) the list is the bucket
//     runs in decreasing order of their first insertion, each run in
//     decreasing insertion order; a rehash re-inserts the nodes in list order
//     with the same rule, so every phase is that ordering applied to the
//     sequence (previous walk order, then the later inserts).
// ---------------------------------------------------------------------------

__device__ __forceinline__ uint32_t rl(uint32_t v, int lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}
__device__ __forceinline__ uint32_t wl(uint32_t arr, uint32_t val, int lane) {
  return threadIdx.x == (uint32_t)lane ? val : arr;  // val, lane wave-uniform
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// Walk order of nodes 0..cnt-1 (lane = node) under the insertion rule, for
// sequence positions q and bucket count `ph`'s: lane's position in the list.
__device__ __forceinline__ uint32_t map_walk(int key, uint32_t q, int cnt, int ph) {
  const uint32_t lane = threadIdx.x;
  const uint32_t b = bucket_of(key, phase_of(ph));
  uint32_t F = q;  // first insertion (min q) of the lane's bucket
  for (int t = 0; t < cnt; t++) {
    const uint32_t bt = rl(b, t), qt = rl(q, t);
    if (bt == b && qt < F) F = qt;
  }
  uint32_t rank = 0;
  for (int t = 0; t < cnt; t++) {
    const uint32_t Ft = rl(F, t), qt = rl(q, t);
    rank += (Ft > F || (Ft == F && qt > q)) ? 1u : 0u;
  }
  return lane < (uint32_t)cnt ? rank : lane;
}

__device__ __forceinline__ void wheap_sift_up(uint32_t& heap, int hole, uint32_t e) {
  while (hole > 0) {
    const int parent = (hole - 1) >> 1;
    const uint32_t pe = rl(heap, parent);
    if ((pe >> 8) <= (e >> 8)) break;
    heap = wl(heap, pe, hole);
    hole = parent;
  }
  heap = wl(heap, e, hole);
}

__device__ __forceinline__ uint32_t wheap_pop(uint32_t& heap, int& len) {
  const uint32_t top = rl(heap, 0);
  const int m = --len;
  if (m > 0) {
    const uint32_t value = rl(heap, m);
    int hole = 0, child = 0;
    while (child < (m - 1) / 2) {
      child = 2 * (child + 1);
      const uint32_t right = rl(heap, child), left = rl(heap, child - 1);
      uint32_t pick = right;
      if ((right >> 8) > (left >> 8)) {
        child--;
        pick = left;
      }
      heap = wl(heap, pick, hole);
      hole = child;
    }
    if ((m & 1) == 0 && child == (m - 2) / 2) {
      child = 2 * (child + 1);
      heap = wl(heap, rl(heap, child - 1), hole);
      hole = child - 1;
    }
    wheap_sift_up(heap, hole, value);
  }
  return top;
}

// OR `nb` bits of `v` at bit offset `off` into the chunk image.
__device__ __forceinline__ void put_bits(uint32_t* img, uint32_t off, uint32_t v, uint32_t nb) {
  if (nb == 0) return;
  const uint32_t w = off >> 5, sh = off & 31u;
  atomicOr(&img[w], v << sh);
  if (sh + nb > 32) atomicOr(&img[w + 1], v >> (32 - sh));
}

__device__ void encode_block_wave(const uint4* __restrict__ coef, const uint8_t* __restrict__ rmask, uint32_t g,
                                  uint32_t* img,
                                  uint32_t* __restrict__ oslots, uint8_t* __restrict__ sizes,
                                  uint32_t* __restrict__ tile_bytes,
                                  uint32_t _wslot = 0) {
  const uint32_t lane = threadIdx.x;
#ifdef MYYUV_STAMPS
  unsigned long long _wprev = 0;
#endif
  WSTAMP(0);
  // ---- lane i: zig-zag position i (Huffman.cpp:176-182)
  const uint32_t nat = c_zz_lane[lane];
  const uint32_t word = (rmask[g] >> (nat >> 3)) & 1u  // row nat >> 3 is nonzero
                            ? reinterpret_cast<const uint32_t*>(coef)[coef_quad(g, nat >> 3) * 4u + ((nat >> 1) & 3u)]
                            : 0u;
  const int v = (int)(int16_t)(word >> (16 * (nat & 1)));
  const uint64_t nzm = __ballot(v != 0);
  int msz = nzm ? 64 - __clzll((long long)nzm) : 0;
  if (msz == 0) msz = 1;  // all-zero block: one symbol 0 (Huffman.cpp:191-194)
  const bool act = lane < (uint32_t)msz;
  const bool has_zero = __ballot(act && v == 0) != 0;
  WSTAMP(1);

  // ---- distinct symbols in first-occurrence order (operator[] insertion
  // order, Huffman.cpp:183): lane s of key/cnt = symbol s; slot = the
  // position's symbol
  uint32_t cntv = 0, slot = 0;
  int key = 0;
  int n = 0;
  for (int j = 0; j < msz; j++) {
    const int vj = (int)rl((uint32_t)v, j);
    const uint64_t eq = __ballot(act && v == vj);
    if ((eq & ((1ull << j) - 1ull)) == 0) {  // first occurrence
      key = (int)wl((uint32_t)key, (uint32_t)vj, n);
      cntv = wl(cntv, (uint32_t)__popcll(eq), n);
      if ((eq >> lane) & 1ull) slot = (uint32_t)n;
      n++;
    }
  }
  const bool sym = lane < (uint32_t)n;
  WSTAMP(2);

  // ---- std::unordered_map iteration order (rehash before the 14th, 30th,
  // 60th insert; the freq[0] probe's rehash, Huffman.cpp:186-197)
  int ph = 0;
  uint32_t q = lane;
  const int nbs[4] = {13, 29, 59, 127};
  while (n > nbs[ph]) {
    q = map_walk(key, q, nbs[ph], ph);
    ph++;
  }
  if (!has_zero && n == nbs[ph]) {
    q = map_walk(key, q, n, ph);
    ph++;
  }
  const uint32_t order = map_walk(key, q, n, ph);  // lane s: list position of symbol s
  WSTAMP(3);

  // ---- Huffman merges on a lane-distributed heap (libstdc++ push/pop_heap)
  uint32_t heap = 0, lpar = 0, ipar = 0;
  int hlen = 0;
  for (int r = 0; r < n; r++) {
    const int node = __ffsll((long long)__ballot(sym && order == (uint32_t)r)) - 1;
    wheap_sift_up(heap, hlen++, (rl(cntv, node) << 8) | (uint32_t)node);
  }
  for (int k = 0; k + 1 < n; k++) {
    const uint32_t l = wheap_pop(heap, hlen);
    const uint32_t r = wheap_pop(heap, hlen);
    const uint32_t li = l & 0xFF, ri = r & 0xFF;
    if (li < 64) lpar = wl(lpar, (uint32_t)k, (int)li);
    else ipar = wl(ipar, (uint32_t)k, (int)(li - 64));
    if (ri < 64) lpar = wl(lpar, (uint32_t)k, (int)ri);
    else ipar = wl(ipar, (uint32_t)k, (int)(ri - 64));
    wheap_sift_up(heap, hlen++, (((l >> 8) + (r >> 8)) << 8) | (uint32_t)(64 + k));
  }
  WSTAMP(4);
  // ---- code lengths (generateCodeLength, Huffman.cpp:71-83): depth chain
  uint32_t len = 1;
  if (n >= 2) {
    uint32_t dep = wl(0u, 0u, n - 2);  // root = last internal node
    for (int k = n - 3; k >= 0; k--) dep = wl(dep, rl(dep, (int)rl(ipar, k)) + 1u, k);
    len = (uint32_t)__shfl((int)dep, (int)lpar, 64) + 1u;
  }
  const uint32_t nbits = wave_sum(sym ? cntv * len : 0u);
  uint32_t cl[9];
#pragma unroll
  for (int l = 1; l <= 8; l++) cl[l] = (uint32_t)__popcll(__ballot(sym && len == (uint32_t)l));

  WSTAMP(5);
  // ---- canonical order (length, symbol) and codes (generateCanonicalTree,
  // Huffman.cpp:86-103): rank by counting; first code / first rank per length
  const uint32_t ckey = (len << 11) | (uint32_t)(key + 1024);
  uint32_t crank = 0;
  for (int t = 0; t < n; t++) crank += rl(ckey, t) < ckey ? 1u : 0u;
  uint32_t fc = 0, fr = 0, myfc = 0, myfr = 0, gbase = 3, mygb = 0;
  uint32_t table_bytes = 0;
#pragma unroll
  for (int l = 1; l <= 8; l++) {
    if (len == (uint32_t)l) {
      myfc = fc;
      myfr = fr;
      mygb = gbase;
    }
    const uint32_t c = cl[l];
    const uint32_t gb = c > 32 ? 2 + 44 + ((c - 32) * 11 + 7) / 8 : (c ? 1 + (c * 11 + 7) / 8 : 0);
    gbase += gb;
    table_bytes += gb;
    fc = (fc + c) << 1;
    fr += c;
  }
  const uint32_t code = myfc + (crank - myfr);
  const uint32_t rcode = __brev(code) >> (32 - len);

  WSTAMP(6);
  // ---- chunk image (Huffman::dump, Huffman.cpp:279-326), LSB-first
  if (lane < (uint32_t)kSlotWords) img[lane] = 0;
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) {
    atomicOr(&img[0], nbits | (table_bytes << 16));
    uint32_t b = 3;
#pragma unroll
    for (int l = 1; l <= 8; l++) {
      const uint32_t c = cl[l];
      if (c) {
        put_bits(img, 8 * b, ((uint32_t)(l - 1) << 5) | ((c > 32 ? 32 : c) - 1), 8);
        if (c > 32) put_bits(img, 8 * (b + 45), ((uint32_t)(l - 1) << 5) | (c - 33), 8);
        b += c > 32 ? 2 + 44 + ((c - 32) * 11 + 7) / 8 : 1 + (c * 11 + 7) / 8;
      }
    }
  }
  if (sym) {  // 11-bit values in canonical order (pack11bit)
    const uint32_t j = crank - myfr;
    const uint32_t off = j < 32 ? 8 * (mygb + 1) + 11 * j : 8 * (mygb + 46) + 11 * (j - 32);
    put_bits(img, off, (uint32_t)key & 0x7FFu, 11);
  }
  // code bits of the message, position order
  const uint32_t pl = act ? (uint32_t)__shfl((int)len, (int)slot, 64) : 0u;
  const uint32_t pc = (uint32_t)__shfl((int)rcode, (int)slot, 64);
  uint32_t pre = pl;  // inclusive prefix sum over lanes
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = (uint32_t)__shfl_up((int)pre, d, 64);
    if (lane >= (uint32_t)d) pre += o;
  }
  if (act) put_bits(img, 8 * (3 + table_bytes) + pre - pl, pc, pl);
  __builtin_amdgcn_wave_barrier();
  if (lane < (uint32_t)kSlotWords) oslots[(size_t)g * kSlotWords + lane] = img[lane];
  if (lane == 0) {
    const uint32_t size = 3 + table_bytes + (nbits + 7) / 8;
    sizes[g] = (uint8_t)size;
    atomicAdd(tile_bytes, size);  // the tile's overflow chunk bytes (K4's tile scan)
  }
  WSTAMP(7);
}

}  // namespace

// The list the wave / lane overflow passes take: K2's (`work`), or, when it
// is longer than `gate` (kR16Gate when k_huff_encode_r16 ran, else ~0u), what
// the CAP-16 tier left (`work2`).
struct OvfList {
  const uint32_t* ids;
  uint32_t n;
};
__device__ __forceinline__ OvfList overflow_list(const uint32_t* work, const uint32_t* work_count,
                                                 const uint32_t* work2, const uint32_t* work2_count,
                                                 uint32_t gate) {
  const uint32_t cnt = *work_count;
  if (cnt <= gate) return OvfList{work, cnt};
  return OvfList{work2, *work2_count};
}

// Overflow pass for short worklists: one wave per listed block (see
// encode_block_wave); exits at once when the list is long (the lane pass
// k_huff_encode_wide takes it).
__global__ __launch_bounds__(64) void k_huff_encode_wave(const uint4* __restrict__ coef,
                                                        const uint8_t* __restrict__ rmask, FrameGeom G,
                                                        uint32_t* __restrict__ oslots,
                                                        uint8_t* __restrict__ sizes,
                                                        uint32_t* __restrict__ tinfo,
                                                        const uint32_t* __restrict__ work,
                                                        const uint32_t* __restrict__ work_count,
                                                        const uint32_t* __restrict__ work2,
                                                        const uint32_t* __restrict__ work2_count,
                                                        uint32_t gate, uint32_t limit) {
  __shared__ uint32_t img[kSlotWords + 2];
  const OvfList L = overflow_list(work, work_count, work2, work2_count, gate);
  const uint32_t cnt = L.n;
  if (cnt > limit) return;
  for (uint32_t i = blockIdx.x; i < cnt; i += gridDim.x) {
    const uint32_t g = L.ids[i];
    encode_block_wave(coef, rmask, g, img, oslots, sizes, tinfo + (size_t)tile_of_block(G, g) * kTInfoWords, i);
  }
}

namespace {

// Coefficient sources of encode_tile: K1's quads in HBM (k_huff_encode), or
// the tile's LDS image (k_encode_tile: row c of the tile's block b at
// c * kK2Group + b), which also hands the overflow blocks' coefficients to the
// overflow passes through HBM.
struct GlobalCoef {
  const uint4* coef;
  const uint8_t* rmask;
  const uint4* zq;
  uint32_t gb;  // batch-global index of the tile's block 0
  __device__ __forceinline__ uint32_t rm(uint32_t b) const { return rmask[gb + b]; }
  __device__ __forceinline__ void load(CoefRegs& R, uint32_t b, uint32_t m) const { R.load(coef, zq, gb + b, m); }
  __device__ __forceinline__ void spill(const CoefRegs&, uint32_t, uint32_t) const {}
};

template <bool kSpill>
struct LdsCoefT {
  const uint4* img;
  const uint8_t* s_rm;
  uint4* coef;
  uint8_t* rmask;
  uint32_t gb;
  __device__ __forceinline__ uint32_t rm(uint32_t b) const { return s_rm[b]; }
  __device__ __forceinline__ void load(CoefRegs& R, uint32_t b, uint32_t m) const {
#pragma unroll
    for (int c = 0; c < 8; c++) {
      const uint4 v = (m >> c) & 1u ? img[c * kK2Group + b] : make_uint4(0, 0, 0, 0);
      R.w[4 * c] = v.x;
      R.w[4 * c + 1] = v.y;
      R.w[4 * c + 2] = v.z;
      R.w[4 * c + 3] = v.w;
    }
  }
  // a block for the overflow passes: its nonzero rows and row mask to HBM (K1's layout)
  __device__ __forceinline__ void spill(const CoefRegs& R, uint32_t b, uint32_t m) const {
    if (!kSpill) return;
    const uint32_t g = gb + b;
#pragma unroll
    for (int c = 0; c < 8; c++)
      if ((m >> c) & 1u) coef[coef_quad(g, c)] = make_uint4(R.w[4 * c], R.w[4 * c + 1], R.w[4 * c + 2], R.w[4 * c + 3]);
    rmask[g] = (uint8_t)m;
  }
};

using LdsCoef = LdsCoefT<true>;
constexpr int kTileWaves = kK2Group / kWave;

// K2's scratch in LDS (k_encode_tile lays it over its transpose tiles).
struct TileScratch {
  uint32_t g[kK2Group];  // sorted position -> the tile's block
  uint8_t msz[kK2Group], cls[kK2Group], rm[kK2Group];
  uint32_t cnt[kTileWaves][kClassDead + 1];
};

// K2 on one tile (kK2Group consecutive blocks of one plane of one frame:
// FrameGeom::tcum; workgroup = kK2Group threads).  The workgroup classifies
// its blocks (block_class: one symbol / <= 4 / <= 8 distinct for sure / the
// rest), sorts them by class through LDS and hands each wave 64 blocks of
// (nearly) one class, so a wave runs the cheapest register-resident encoder
// that fits all its blocks and its loops run to the maxima of similar blocks
// rather than of a 64-block stretch of the frame.  Sorted chunks are dealt to
// the waves so that each SIMD gets one heavy and one light chunk.  Each lane
// builds its block's code (sizes known before a bit is written), a wave scan
// gives every chunk its byte offset, and the wave's chunks go back to back
// into its dense run (DenseWriter: every dword stored once, by the block
// owning its first byte); srcoff records where each block's chunk is
// (codec_common.hpp, K2 -> K4).  Blocks with more than 8 distinct symbols are
// appended to `work` for the overflow passes.
template <class Src>
__device__ __forceinline__ void encode_tile(const Src& src, TileScratch& sc, uint32_t T, uint32_t nloc,
                                            uint32_t* __restrict__ stage, uint32_t* __restrict__ tinfo,
                                            uint8_t* __restrict__ sizes, uint32_t* __restrict__ srcoff,
                                            uint32_t* __restrict__ work, uint32_t* __restrict__ work_count) {
  constexpr int kWaves = kTileWaves;
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const uint32_t gb = src.gb;
  // the overflow passes add their chunk bytes to the tile's info word 0
  // (ordered before them by the kernel boundary)
  if (tid == 0) tinfo[(size_t)T * kTInfoWords] = 0u;
  // ---- classify
  uint32_t cls = kClassDead;
  int msz = 0;
  uint32_t rm = 0;
  if (tid < nloc) {
    rm = src.rm(tid);
    CoefRegs R;
    src.load(R, tid, rm);
    msz = R.msz();
    cls = block_class(R, msz);
  }
  // ---- counting sort by class (stable: class, then wave, then lane)
  const uint64_t below = (1ull << lane) - 1ull;
  uint32_t rank = 0;
#pragma unroll
  for (uint32_t c = 0; c <= kClassDead; c++) {
    const uint64_t b = __ballot(cls == c);
    if (cls == c) rank = (uint32_t)__popcll(b & below);
    if (lane == 0) sc.cnt[wave][c] = (uint32_t)__popcll(b);
  }
  __syncthreads();
  uint32_t pos = rank;
#pragma unroll
  for (uint32_t c = 0; c <= kClassDead; c++)
#pragma unroll
    for (uint32_t w = 0; w < (uint32_t)kWaves; w++)
      pos += (c < cls || (c == cls && w < wave)) ? sc.cnt[w][c] : 0u;
  sc.g[pos] = tid;
  sc.msz[pos] = (uint8_t)msz;
  sc.cls[pos] = (uint8_t)cls;
  sc.rm[pos] = (uint8_t)rm;
  __syncthreads();
  // ---- build: wave w takes sorted chunk w < kWaves/2 ? kWaves-1-w : w-kWaves/2
  const uint32_t chunk = wave < (uint32_t)kWaves / 2 ? kWaves - 1 - wave : wave - kWaves / 2;
  const uint32_t e = chunk * kWave + lane;
  const uint32_t ml = sc.g[e];  // the lane's block in the tile (every one of 0..255 once)
  const int mm = sc.msz[e];
  const uint32_t mc = sc.cls[e];
  const uint32_t mrm = sc.rm[e];
  const bool live = mc != kClassDead;
  const bool bld = live && mc != kClassOvf;  // (ovf blocks: straight to the worklist)
  const uint32_t mg = gb + ml;
  uint32_t wcls = kClassDead;  // the wave's heaviest class to build
#pragma unroll
  for (int c = kClassOvf - 1; c >= 0; c--)
    if (wcls == kClassDead && __ballot(mc == (uint32_t)c) != 0) wcls = (uint32_t)c;
  const int wmsz = max(wave_max(bld ? mm : 0), 1);
#ifdef MYYUV_STAMPS
  const uint32_t wid = T * kWaves + wave;
  if (lane == 0 && wid < 8192) g_k2_fstamps[wid * 8 + 0] = wcls | ((uint32_t)wmsz << 8);
  const unsigned long long _w0 = __builtin_amdgcn_s_memtime();
#endif
  EncState S;
  bool ok = false;
  if (__ballot(live) != 0) {
    CoefRegs R;
    src.load(R, live ? ml : 0u, live ? mrm : 0u);
    if (wcls == kClassSingle) {
      if (bld) {
        build_single(R, S);
        ok = true;
      }
    } else if (wcls == kClassR4) {
      if (bld) ok = build_r<4>(R, mm, wmsz, S);
    } else if (wcls != kClassDead) {
      if (bld) ok = build_r<8>(R, mm, wmsz, S);
    }
    if (live && !ok) src.spill(R, ml, mrm);
  }
  // ---- the wave's dense run: chunks back to back in the wave's order
  // (offsets by a wave scan of the sizes; no workgroup barrier), every dword
  // stored once (DenseWriter)
  const bool dense = live && ok;
  const uint32_t sz = dense ? S.size : 0u;
  uint32_t incl = sz;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = (uint32_t)__shfl_up((int)incl, d, 64);
    if (lane >= (uint32_t)d) incl += o;
  }
  const uint32_t off = incl - sz;
  const uint64_t dm = __ballot(dense);
  const uint64_t above = lane == 63 ? 0ull : dm & ~((2ull << lane) - 1ull);
  const int nl = above ? __ffsll((long long)above) - 1 : (int)lane;
  const uint32_t nhdr = (uint32_t)__shfl((int)(dense ? S.hdr : 0u), nl, 64);
  uint32_t* info = tinfo + (size_t)T * kTInfoWords;
  if (lane == 63) info[1 + wave] = incl;  // the run's bytes
  if (dense) {
    DenseWriter dw;
    dw.init(stage + (size_t)T * (kTileCap / 4) + wave * (kWaveRun / 4), off);
    emit_chunk(S, wmsz, dw);
    dw.finish(above ? (nhdr | 0x80000000u) : 0u);
    sizes[mg] = (uint8_t)S.size;
    srcoff[mg] = (T & (kWinTiles - 1u)) * kTileCap + wave * kWaveRun + off;  // from the window's first tile
  }
  // blocks with more than 8 distinct symbols: the overflow passes' worklist
  const uint64_t ovf = __ballot(live && !ok);
  if (ovf) {
    if (live && !ok) srcoff[mg] = kSrcOverflow;
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(work_count, (uint32_t)__popcll(ovf));
    base = __builtin_amdgcn_readfirstlane(base);
    if ((ovf >> lane) & 1) work[base + (uint32_t)__popcll(ovf & below)] = mg;
  }
#ifdef MYYUV_STAMPS
  if (lane == 0 && wid < 8192) g_k2_fstamps[wid * 8 + 7] = (uint32_t)(__builtin_amdgcn_s_memtime() - _w0);
#endif
}

}  // namespace

namespace {

// K2's window sort (k_huff_encode): the window's blocks are counting-sorted
// by class (dead slots last) over the window's W tiles at once (W =
// kWinTiles or kWinTilesBig, k2_win).  Sort slots are the (tile round, wave)
// pairs that classified them, so the order is stable: class, then window slot
// (tile, block).
// sort keys: the single class, then each class K2 builds (r4, r8, r8x)
// split by message length (the per-position loops run to the run's longest
// message), then the ovf class (built by the overflow passes: one key), the
// dead slots last.  Length buckets (MYYUV_K2_MSZ_SPLIT): 2 -> <= 8, <= 16,
// longer (rounds 3-5); 3 -> <= 6, <= 12, <= 20, longer (round 6: the sum of
// the runs' longest messages over the bench frame 28.2k -> 26.4k,
// tools/diag/k2_run_sim.py)
#ifndef MYYUV_K2_MSZ_SPLIT
#define MYYUV_K2_MSZ_SPLIT 3
#endif
constexpr uint32_t kMszBuckets = MYYUV_K2_MSZ_SPLIT + 1;
constexpr uint32_t kOvfKey = 1 + (kClassOvf - 1) * kMszBuckets;
constexpr uint32_t kKeys = kOvfKey + 2;
constexpr uint32_t kDeadKey = kKeys - 1;
__device__ __forceinline__ uint32_t sort_key(uint32_t cls, uint32_t msz) {
  if (cls == kClassDead) return kDeadKey;
  if (cls == kClassOvf) return kOvfKey;
  if (cls == kClassSingle) return 0;
  uint32_t b;
  if constexpr (MYYUV_K2_MSZ_SPLIT == 3)
    b = (msz > 6 ? 1u : 0u) + (msz > 12 ? 1u : 0u) + (msz > 20 ? 1u : 0u);
  else
    b = (msz > 8 ? 1u : 0u) + (msz > 16 ? 1u : 0u);
  return 1 + (cls - 1) * kMszBuckets + b;
}
template <uint32_t W>
struct WinCfg {
  static constexpr uint32_t kBlocks = W * kK2Group;
  static constexpr uint32_t kRuns = kBlocks / kWave;                   // 64-block runs per window
  static constexpr uint32_t kScanVals = kKeys * kRuns;                 // [key][round * 4 + wave] counts
  static constexpr uint32_t kScanPer = (kScanVals + kWave - 1) / kWave;
};
static_assert(kK2Group == 256, "window slots are tile << 8 | block");

// set bits of m below the calling lane (v_mbcnt: no 64-bit lane mask held)
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// The lane id through an opaque (volatile) v_mbcnt pair: never hoisted out
// of a loop nor merged with another evaluation.
__device__ __forceinline__ uint32_t fresh_lane_id() {
  uint32_t lo, id;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0" : "=v"(lo));
  asm volatile("v_mbcnt_hi_u32_b32 %0, -1, %1" : "=v"(id) : "v"(lo));
  return id;
}

// The wave's maximum and an inclusive sum by DPP, for k_huff_encode's count
// scan (wave 0 whole) and run loop only: the loop's control is wave-uniform
// (the run comes from a readfirstlane, the class branches are uniform), so
// every lane is active where these run.  Under a partial EXEC, inactive lanes would pass nothing
// on (the round-3 DPP episode): ds_bpermute forms stay
// wherever EXEC can be partial.
__device__ __forceinline__ int wave_max_full(int v) {  // (v >= 0)
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false));  // row_shr:1
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false));  // row_shr:2
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false));  // row_shr:4
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false));  // row_shr:8
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false));  // row_bcast:15
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false));  // row_bcast:31
  return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ uint32_t wave_incl_sum_full(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return x;
}

template <uint32_t W>
struct WinScratch {
  uint16_t slot[WinCfg<W>::kBlocks];  // sorted position -> window slot (tile << 8 | block)
  uint16_t dc[WinCfg<W>::kBlocks];    // window slot -> its DC coefficient's low 11 bits (from K1's block word)
  uint8_t msz[WinCfg<W>::kBlocks], cls[WinCfg<W>::kBlocks], rm[WinCfg<W>::kBlocks];
  uint32_t cnt[WinCfg<W>::kScanVals];  // per (key, sort slot): count, then exclusive position
  uint32_t gb[W];             // batch-global index of tile k's block 0
  uint32_t tot[W];            // tile k's dense chunk bytes
  uint32_t next, done, ntl;   // run counter, finished waves, the window's tiles
};

}  // namespace

// K2 over K1's coefficients in HBM: one workgroup per window of W (k2_win)
// batch tiles (grid: windows).
//   coef: natural-order quads (codec_common.hpp); sizes: [n] u8.
// 1. classify: thread i takes block i of each of the window's tiles (one
//    coefficient load per block, coalesced), its message length and class;
// 2. a counting sort of the window's blocks by class (ballot ranks per round
//    and wave, one wave scans the counts);
// 3. the sorted blocks in 64-block runs, heaviest run first, taken by the
//    waves from an LDS counter (no barrier between runs: a wave that drew
//    light runs takes more of them).  Each lane builds its block's code, a
//    wave scan places the chunks back to back in the run's stage region
//    (DenseWriter), srcoff records where, and the run's chunk bytes are added
//    to their tiles' totals in LDS; blocks with more than 8 distinct symbols
//    go to the overflow worklist;
// 4. the last wave to finish publishes the tiles' totals (tinfo word 1).
// Sorting over 4 tiles rather than one makes the runs more uniform: per
// 4032x3008 frame the waves' class mix (single / <= 4 / <= 8 / rest) drops
// from 1859 / 834 / 740 / 1010 runs to 2220 / 968 / 652 / 603
// (tools/k2_window_sim.py).
#ifndef MYYUV_K2_WAVES
#define MYYUV_K2_WAVES 5  // 5 workgroups of 4 waves per CU: <= 96 VGPRs (12 spilled; 6 measured +1.5 % before the emit tables, −1 % after: its spills grew; tools/ab_bench.sh, tools/kus_ab.sh)
#endif
template <uint32_t W>
__global__ __launch_bounds__(kK2Group, MYYUV_K2_WAVES) void k_huff_encode(const uint4* __restrict__ coef,
                                                         const uint32_t* __restrict__ binfo,
                                                         const uint4* __restrict__ zq, FrameGeom G,
                                                         uint32_t* __restrict__ stage,
                                                         uint32_t* __restrict__ tinfo,
                                                         uint8_t* __restrict__ sizes,
                                                         uint32_t* __restrict__ srcoff,
                                                         uint32_t* __restrict__ work,
                                                         uint32_t* __restrict__ work_count) {
  constexpr uint32_t kWinRuns = WinCfg<W>::kRuns, kScanVals = WinCfg<W>::kScanVals, kScanPer = WinCfg<W>::kScanPer;
  __shared__ WinScratch<W> sc;
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
#ifdef MYYUV_STAMPS
  uint32_t _kw[7] = {0u, 0u, 0u, 0u, 0u, 0u, 0u};
  unsigned long long _kwprev = __builtin_amdgcn_s_memtime();
#endif
  const uint32_t NT = G.nframes * G.tcum[3];
  const uint32_t T0 = blockIdx.x * W;
  // ---- the window's tiles (wave-uniform)
  uint32_t gbk[W], nlk[W];
#pragma unroll
  for (uint32_t k = 0; k < W; k++) {
    const uint32_t T = T0 + k;
    nlk[k] = 0;
    gbk[k] = 0;
    if (T < NT) {
      const uint32_t f = G.nframes > 1 ? T / G.tcum[3] : 0u;
      const uint32_t t = T - f * G.tcum[3];
      const int p = tile_plane(G, t);
      const uint32_t g0 = tile_first(G, p, t);
      nlk[k] = min(kK2Group, G.cum[p + 1] - g0);
      gbk[k] = f * G.cum[3] + g0;
    }
  }
  if (tid < W) {
    sc.gb[tid] = gbk[tid];
    sc.tot[tid] = 0;
    // the overflow passes add their chunk bytes to the tile's info word 0
    // (ordered before them by the kernel boundary)
    if (T0 + tid < NT) tinfo[(size_t)(T0 + tid) * kTInfoWords] = 0u;
  }
  if (tid == 0) {
    sc.next = 0;
    sc.done = 0;
    sc.ntl = T0 < NT ? min(W, NT - T0) : 0u;  // (no window starts past the end: grid ceil(NT / W))
  }
  // ---- 1. classify from K1's per-block words (row mask, msz, class, DC;
  // 4 B per block, coalesced), with per-round ballot ranks
  uint32_t ent[W];  // per round: class | msz << 3 | row mask << 10 | rank << 18
  uint32_t biv[W];
#pragma unroll
  for (uint32_t k = 0; k < W; k++) biv[k] = tid < nlk[k] ? binfo[gbk[k] + tid] : 0u;
#ifdef MYYUV_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (diagnostic: the block words' arrival)
  KWSTAMP(6);
#endif
#pragma unroll
  for (uint32_t k = 0; k < W; k++) {
    const uint32_t bi = biv[k];
    const uint32_t cls = tid < nlk[k] ? (bi >> 15) & 7u : kClassDead;
    const uint32_t m = (bi >> 8) & 127u, rm = bi & 0xFFu;
    const uint32_t key = sort_key(cls, m);
    sc.dc[(k << 8) | tid] = (uint16_t)(bi >> 18);  // the DC's low 11 bits (build_single_dc uses those)
    // the round's count per key and the lane's rank among its key's lanes
    // from one ballot per key bit: a lane's equal-key mask is the AND of each
    // bit's ballot or its complement (lane order: a stable sort), lane c < kKeys
    // writes key c's count.  No loop over the keys: kKeys ballots, each with
    // its own exec branch, took 16 % of a wave's cycles (profiles/r5au_k2_phase.txt)
    static_assert(kKeys <= 16 && kKeys <= 64, "four key bits");
    uint64_t bb[4];
#pragma unroll
    for (int j = 0; j < 4; j++) bb[j] = __ballot((key >> j) & 1u);
    auto eq_mask = [&](uint32_t v) {
      uint64_t e = ~0ull;
#pragma unroll
      for (int j = 0; j < 4; j++) e &= ((v >> j) & 1u) ? bb[j] : ~bb[j];
      return e;
    };
    const uint32_t rk = lanes_below(eq_mask(key));
    if (lane < kKeys) sc.cnt[lane * kWinRuns + k * kTileWaves + wave] = (uint32_t)__popcll(eq_mask(lane));
    ent[k] = cls | (m << 3) | (rm << 10) | (rk << 18) | (key << 24);
  }
#ifdef MYYUV_STAMPS
  KWSTAMP(5);
#endif
  __syncthreads();
  // ---- 2. exclusive scan of the counts in (key, round, wave) order (wave 0)
  if (wave == 0) {
    uint32_t v[kScanPer], sum = 0;
#pragma unroll
    for (uint32_t j = 0; j < kScanPer; j++) {
      const uint32_t idx = lane * kScanPer + j;
      v[j] = idx < kScanVals ? sc.cnt[idx] : 0u;
      sum += v[j];
    }
    const uint32_t incl = wave_incl_sum_full(sum);  // (all of wave 0 active)
    uint32_t ex = incl - sum;
#pragma unroll
    for (uint32_t j = 0; j < kScanPer; j++) {
      const uint32_t idx = lane * kScanPer + j;
      if (idx < kScanVals) sc.cnt[idx] = ex;
      ex += v[j];
    }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < W; k++) {
    const uint32_t x = ent[k];
    const uint32_t pos = sc.cnt[(x >> 24) * kWinRuns + k * kTileWaves + wave] + ((x >> 18) & 63u);
    sc.slot[pos] = (uint16_t)((k << 8) | tid);
    sc.msz[pos] = (uint8_t)((x >> 3) & 127u);
    sc.cls[pos] = (uint8_t)(x & 7u);
    sc.rm[pos] = (uint8_t)(x >> 10);
  }
  // the live blocks = the exclusive position of the first dead slot
  const uint32_t nlive = sc.cnt[kDeadKey * kWinRuns];
  __syncthreads();
  const uint32_t nruns = (nlive + kWave - 1) / kWave;
#ifdef MYYUV_STAMPS
  KWSTAMP(0);
#endif
  // ---- 3. the runs, heaviest first
  while (true) {
    uint32_t r = 0;
    if (lane == 0) r = atomicAdd(&sc.next, 1u);
    r = (uint32_t)__builtin_amdgcn_readfirstlane((int)r);
    if (r >= nruns) break;
    const uint32_t run = nruns - 1 - r;
    // the lane id, recomputed per run (opaque to the optimiser): kept out of
    // the loop, every lane-derived address (shuffles, LDS) would be hoisted
    // and held in registers across the run's encoder, which then spills
    const uint32_t ln = fresh_lane_id();
    const uint32_t e = run * kWave + ln;
    const uint32_t sl = sc.slot[e];
    const int mm = sc.msz[e];
    const uint32_t mc = sc.cls[e];
    const uint32_t mrm = sc.rm[e];
    const bool live = e < nlive;
    const bool bld = live && mc != kClassOvf;  // (ovf blocks: straight to the worklist)
    const uint32_t k = sl >> 8;
    const uint32_t mg = sc.gb[k] + (sl & 255u);
    uint32_t wcls = kClassDead;  // the run's heaviest class to build
#pragma unroll
    for (int c = kClassOvf - 1; c >= 0; c--)
      if (wcls == kClassDead && __ballot(bld && mc == (uint32_t)c) != 0) wcls = (uint32_t)c;
    const int wmsz = max(wave_max_full(bld ? mm : 0), 1);
    EncState S;
    bool ok = false;
    // (the coefficients are loaded inside each class's branch: loaded before
    // it, they are spilled to scratch across the branch, one dependent load
    // round trip per quad)
    if (wcls == kClassSingle) {
      // one symbol: the DC coefficient (word 0 of quad 0), or 0
      // (single-class runs take the DC from LDS, kept at classification, not from HBM)
      const uint32_t dc = bld ? (uint32_t)sc.dc[sl] : 0u;
      if (bld) {
        build_single_dc((int)(int16_t)dc, S);
        ok = true;
      }
    } else if (wcls == kClassR4) {
      CoefRegs R;
      R.load(coef, zq, bld ? mg : 0u, bld ? mrm : 0u);
      if (bld) ok = build_r<4>(R, mm, wmsz, S);
    } else if (wcls != kClassDead) {
      CoefRegs R;
      R.load(coef, zq, bld ? mg : 0u, bld ? mrm : 0u);
      if (bld) ok = build_r<8>(R, mm, wmsz, S);
    }
#ifdef MYYUV_STAMPS
    KWSTAMP(1);
#endif
    // the run's chunks back to back (offsets by a wave scan of the sizes),
    // every dword stored once (DenseWriter)
    const bool dense = live && ok;
    const uint32_t sz = dense ? S.size : 0u;
    const uint32_t incl = wave_incl_sum_full(sz);
    const uint32_t off = incl - sz;
    const uint64_t dm = __ballot(dense);
    const uint64_t above = ln == 63 ? 0ull : dm & ~((2ull << ln) - 1ull);
    const int nl = above ? __ffsll((long long)above) - 1 : (int)ln;
    const uint32_t nhdr = (uint32_t)__builtin_amdgcn_ds_bpermute(nl << 2, (int)(dense ? S.hdr : 0u));
    if (dense) {
      DenseWriter dw;
      dw.init(stage + ((size_t)blockIdx.x * W * (kTileCap / 4) + run * (kWaveRun / 4)), off);
      emit_chunk(S, wmsz, dw);
      dw.finish(above ? (nhdr | 0x80000000u) : 0u);
      sizes[mg] = (uint8_t)S.size;
      srcoff[mg] = run * kWaveRun + off;
      atomicAdd(&sc.tot[k], S.size);
    }
    // blocks with more than 8 distinct symbols: the overflow passes' worklist
    const uint64_t ovf = __ballot(live && !ok);
    if (ovf) {
      if (live && !ok) srcoff[mg] = kSrcOverflow;
      uint32_t base = 0;
      if (ln == 0) base = atomicAdd(work_count, (uint32_t)__popcll(ovf));
      base = __builtin_amdgcn_readfirstlane(base);
      if ((ovf >> ln) & 1) work[base + lanes_below(ovf)] = mg;
    }
#ifdef MYYUV_STAMPS
    KWSTAMP(2);
    _kw[3] += 1;
#endif
  }
  // ---- 4. the last wave out publishes the tiles' dense bytes
  uint32_t d = 0;
  if (lane == 0) d = __hip_atomic_fetch_add(&sc.done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
  d = (uint32_t)__builtin_amdgcn_readfirstlane((int)d);
  if (d == kTileWaves - 1) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    if (lane < sc.ntl) {
      uint32_t* info = tinfo + (size_t)(blockIdx.x * W + lane) * kTInfoWords;
      info[1] = __hip_atomic_load(&sc.tot[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      info[2] = 0u;
      info[3] = 0u;
      info[4] = 0u;
    }
  }
#ifdef MYYUV_STAMPS
  KWSTAMP(4);
  {
    const uint32_t wid = blockIdx.x * (kK2Group / kWave) + wave;
    if (lane < 8 && wid < 65536) g_k2_win[wid * 8 + lane] = lane < 7 ? _kw[lane < 7 ? lane : 0] : 1u;
  }
#endif
}

// Fused single-pass encoder: K1 + K2 for one tile, the
// coefficients never leaving the chip.  Phase 1: wave w transforms the tile's
// 16-block units 4w .. 4w+3 with K1's code (four lanes per block, all the
// pixel rows loaded up front) into the tile's LDS coefficient image and row
// masks.  Phase 2: encode_tile over that image; only blocks with more than 8
// distinct symbols go to HBM, for the overflow passes.  LDS: 32 KB image +
// 18 KB transpose tiles (K2's scratch is laid over them) + the Q tables:
// three workgroups per CU.
namespace {
// K1's pixel rows 2q, 2q+1 of block b of units 4w .. 4w+3 of a tile (lanes
// past the plane's end read its last block)
struct TileRows {
  uint4 px[4];
};
__device__ __forceinline__ void tile_geometry(const FrameGeom& G, uint32_t T, uint32_t& f, uint32_t& t, int& p,
                                              uint32_t& g0, uint32_t& nloc) {
  f = G.nframes > 1 ? T / G.tcum[3] : 0u;
  t = T - f * G.tcum[3];
  p = tile_plane(G, t);
  g0 = tile_first(G, p, t);
  nloc = min(kK2Group, G.cum[p + 1] - g0);
}
__device__ __forceinline__ xf::Unit plane_unit(const FrameGeom& G, int p) {
  xf::Unit U;
  U.p = p;
  U.cum = G.cum[p];
  U.nb = G.cum[p + 1] - G.cum[p];
  U.poff = p == 0 ? G.poff[0] : (p == 1 ? G.poff[1] : G.poff[2]);
  U.pw = p == 0 ? G.pw[0] : (p == 1 ? G.pw[1] : G.pw[2]);
  U.bw = p == 0 ? G.bw[0] : (p == 1 ? G.bw[1] : G.bw[2]);
  U.bmag = p == 0 ? G.bmag[0] : (p == 1 ? G.bmag[1] : G.bmag[2]);
  U.local0 = 0;
  return U;
}
__device__ __forceinline__ void load_tile_rows(const uint8_t* __restrict__ frame, const FrameGeom& G, uint32_t T,
                                               uint32_t wave, uint32_t b, uint32_t q, TileRows& r) {
  uint32_t f, t, g0, nloc;
  int p;
  tile_geometry(G, T, f, t, p, g0, nloc);
  const xf::Unit U = plane_unit(G, p);
  const uint32_t lbase = g0 - G.cum[p];
  const uint8_t* fr = frame + (size_t)f * G.fbytes;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint32_t local = lbase + (4 * wave + i) * kXfUnit + b;
    const uint32_t off = xf::block_row_offset(U, local < U.nb ? local : U.nb - 1, 2u * q);
    const uint2 r0 = *reinterpret_cast<const uint2*>(fr + off);
    const uint2 r1 = *reinterpret_cast<const uint2*>(fr + off + U.pw);
    r.px[i] = make_uint4(r0.x, r0.y, r1.x, r1.y);
  }
}
}  // namespace

// Fused single-pass encoder: K1 + K2 per tile, the
// coefficients never leaving the chip; one workgroup per tile (grid (tiles,
// frames)).  Phase 1: wave w transforms the tile's 16-block units 4w .. 4w+3
// with K1's code (four lanes per block, all the pixel rows loaded up front)
// into the tile's LDS coefficient image and row masks.  Phase 2: encode_tile
// over that image; only blocks with more than 8 distinct symbols go to HBM,
// for the overflow passes.  LDS: 32 KB image + 18 KB transpose tiles (K2's
// scratch laid over them) + the Q tables: three workgroups per CU.
// (A persistent variant prefetching the next tile's rows behind phase 2
// measured slower: 250 against 209 us per 4-frame launch.)
__global__ __launch_bounds__(kK2Group, 3) void k_encode_tile(const uint8_t* __restrict__ frame, FrameGeom G,
                                                             const QTables* __restrict__ qt,
                                                             uint4* __restrict__ coef,
                                                             uint8_t* __restrict__ rmask,
                                                             uint32_t* __restrict__ stage,
                                                             uint32_t* __restrict__ tinfo,
                                                             uint8_t* __restrict__ sizes,
                                                             uint32_t* __restrict__ srcoff,
                                                             uint32_t* __restrict__ work,
                                                             uint32_t* __restrict__ work_count) {
  using namespace xf;
  __shared__ uint4 s_img[8 * kK2Group];
  __shared__ float s_tile[kTileWaves][kXfUnit * kTile];
  __shared__ float s_q[kSqWords];  // QTables::q, r, kb
  __shared__ uint8_t s_rmk[kK2Group];
  static_assert(sizeof(TileScratch) <= sizeof(s_tile), "K2 scratch over the transpose tiles");
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const uint32_t q = lane & 3u, b = lane >> 2;
  const uint32_t T = blockIdx.y * G.tcum[3] + blockIdx.x;
  uint32_t f, t, g0, nloc;
  int p;
  tile_geometry(G, T, f, t, p, g0, nloc);
  TileRows rows;
  load_tile_rows(frame, G, T, wave, b, q, rows);
  stage_tables<kSqWords>(qt->q[0], s_q);
  float* tb = s_tile[wave] + b * kTile;
  uint8_t* img = reinterpret_cast<uint8_t*>(tb);
  // ---- phase 1
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint32_t lb = (4 * wave + i) * kXfUnit + b;
    if ((4 * wave + i) * kXfUnit >= nloc) break;  // (wave-uniform) the tile's units end
    *reinterpret_cast<uint2*>(img + 16u * q) = make_uint2(rows.px[i].x, rows.px[i].y);
    *reinterpret_cast<uint2*>(img + 16u * q + 8u) = make_uint2(rows.px[i].z, rows.px[i].w);
    wave_sync();
    fdct_core(img, tb, q, s_q, p, [&](const uint32_t (&c)[16], bool) {
      uint4 lo, hi;
      uint32_t rm;
      pack_quads(c, q, lo, hi, rm);
      if (lb < nloc) {
        s_img[(2 * q) * kK2Group + lb] = lo;
        s_img[(2 * q + 1) * kK2Group + lb] = hi;
        if (q == 0) s_rmk[lb] = (uint8_t)rm;
      }
    });
    wave_sync();  // the tile is rewritten by the next unit
  }
  __syncthreads();
  // ---- phase 2: K2 over the LDS image (its scratch over the transpose tiles)
  TileScratch& sc = *reinterpret_cast<TileScratch*>(&s_tile[0][0]);
  const LdsCoef src{s_img, s_rmk, coef, rmask, f * G.cum[3] + g0};
  encode_tile(src, sc, T, nloc, stage, tinfo, sizes, srcoff, work, work_count);
}

// Overflow pass (CAP=64), lane per block, for long worklists (noise-like
// frames where most blocks overflow): the blocks listed in `work` (count in
// *work_count; past kR16Gate what the CAP-16 tier left in `work2`), 64 per
// workgroup; the grid is sized for the worst case, idle groups exit.  Lists
// of at most `limit` blocks go to k_huff_encode_wave instead.
__global__ __launch_bounds__(kWideLanes) void k_huff_encode_wide(const uint4* __restrict__ coef,
                                                        const uint8_t* __restrict__ rmask,
                                                        const uint4* __restrict__ zq, FrameGeom G,
                                                        uint32_t* __restrict__ oslots,
                                                        uint8_t* __restrict__ sizes,
                                                        uint32_t* __restrict__ tinfo,
                                                        const uint32_t* __restrict__ work,
                                                        const uint32_t* __restrict__ work_count,
                                                        const uint32_t* __restrict__ work2,
                                                        const uint32_t* __restrict__ work2_count,
                                                        uint32_t gate, uint32_t limit) {
  constexpr int CAP = 64;
  __shared__ uint32_t lds[Layout<CAP>::kWords * kWideLanes];
  const OvfList L = overflow_list(work, work_count, work2, work2_count, gate);
  const uint32_t cnt = L.n;
  if (cnt <= limit) return;  // short lists: k_huff_encode_wave
  // grid-stride over kWideLanes-block slices of the list (the grid is what
  // the 512 B-per-lane LDS lets be resident)
  for (uint32_t base = blockIdx.x * kWideLanes; base < cnt; base += gridDim.x * kWideLanes) {
    const uint32_t i = base + threadIdx.x;
    const bool live = i < cnt;
    const uint32_t g = live ? L.ids[i] : 0;
    CoefRegs R;
    R.load(coef, zq, g, live ? rmask[g] : 0u);
    const int msz = live ? R.msz() : 0;
    const int wmsz = wave_max<kWideLanes>(msz);
    if (live) {
      const Img<CAP> I{lds, (int)threadIdx.x};
      encode_block<CAP>(I, R, msz, max(wmsz, 1), oslots + (size_t)g * kSlotWords, sizes + g);
      atomicAdd(tinfo + (size_t)tile_of_block(G, g) * kTInfoWords, (uint32_t)sizes[g]);  // (this lane's own store)
    }
  }
}

// Overflow tier 1 for long lists (more than kR16Gate blocks, i.e. more than
// one resident round of k_huff_encode_wide): register-resident, CAP 16
// (huff_r16.hpp), lane per block, 64 blocks per workgroup, grid-stride;
// blocks with more than 16 distinct symbols go on to `work2` for the wave /
// lane passes.  Natural images put nearly all overflow blocks here (q50:
// 99.8 %, q90: 94 %), so past one CAP-64 round the list costs one lane's
// register program per block instead of the LDS replay's chain of dependent
// round trips (8192^2 q90: 214 -> 145 us with the wave pass on work2,
// profiles/r3t_*).
#ifndef MYYUV_R16_LDS
#define MYYUV_R16_LDS 1  // the heap in LDS (r16::LdsHeap16) rather than registers (r16::RegHeap16)
#endif
#ifndef MYYUV_R16_WAVES
#define MYYUV_R16_WAVES 5  // waves per SIMD k_huff_encode_r16 is compiled for: 96 VGPRs, 12 spilled with the LDS heap (4 waves, 128 VGPRs, none spilled: 106 against 129 us alone per 32-frame launch but the bench -0.9 %, profiles/r6ag_*; 3 waves: -1.5 %, r3zzl_*)
#endif
__global__ __launch_bounds__(64, MYYUV_R16_WAVES) void k_huff_encode_r16(const uint4* __restrict__ coef,
                                                        const uint8_t* __restrict__ rmask,
                                                        const uint4* __restrict__ zq, FrameGeom G,
                                                        uint32_t* __restrict__ oslots,
                                                        uint8_t* __restrict__ sizes,
                                                        uint32_t* __restrict__ tinfo,
                                                        const uint32_t* __restrict__ work,
                                                        const uint32_t* __restrict__ work_count,
                                                        uint32_t* __restrict__ work2,
                                                        uint32_t* __restrict__ work2_count, uint32_t gate) {
  const uint32_t cnt = *work_count;
  if (cnt <= gate) return;  // short lists: the wave / lane passes take them whole
  const uint32_t lane = threadIdx.x;
#if MYYUV_R16_LDS
  __shared__ uint32_t heap[16 * kWave];  // the lanes' heaps, one LDS column each
  const r16::LdsHeap16<kWave> hp{heap + lane};
#else
  const r16::RegHeap16 hp;
#endif
  for (uint32_t base = blockIdx.x * kWave; base < cnt; base += gridDim.x * kWave) {
    const uint32_t i = base + lane;
    const bool live = i < cnt;
    const uint32_t g = live ? work[i] : 0u;
    CoefRegs R;
    R.load(coef, zq, g, live ? rmask[g] : 0u);
    const int msz = live ? R.msz() : 0;
    const int wmsz = max(wave_max(msz), 1);
    EncState16 S;
    const bool ok = live && build_r16(R, msz, wmsz, S, hp);
    if (ok) {
      BitWriter bw;
      bw.out = oslots + (size_t)g * kSlotWords;
      emit_chunk16(S, wmsz, bw);
      bw.align_byte();
      bw.flush();
      sizes[g] = (uint8_t)S.size;
      atomicAdd(tinfo + (size_t)tile_of_block(G, g) * kTInfoWords, S.size);  // the tile's overflow bytes
    }
    const uint64_t more = __ballot(live && !ok);
    if (more) {
      uint32_t b0 = 0;
      if (lane == 0) b0 = atomicAdd(work2_count, (uint32_t)__popcll(more));
      b0 = __builtin_amdgcn_readfirstlane(b0);
      if ((more >> lane) & 1ull) work2[b0 + (uint32_t)__popcll(more & ((1ull << lane) - 1ull))] = g;
    }
  }
}


// the two window sizes (k2_win)
#define MYYUV_K2_INST(W)                                                                                         \
  template __global__ void k_huff_encode<W>(const uint4* __restrict__, const uint32_t* __restrict__,             \
                                            const uint4* __restrict__, FrameGeom, uint32_t* __restrict__,       \
                                            uint32_t* __restrict__, uint8_t* __restrict__, uint32_t* __restrict__, \
                                            uint32_t* __restrict__, uint32_t* __restrict__);
MYYUV_K2_INST(kWinTiles)
#if MYYUV_K2_WIN_BIG != MYYUV_K2_WIN
MYYUV_K2_INST(kWinTilesBig)
#endif

}  // namespace myyuv_gpu
