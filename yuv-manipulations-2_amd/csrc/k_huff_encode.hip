// k_huff_encode.hip — K2: per-block Huffman code construction and chunk
// serialisation for gfx950 (Huffman::fromData + Huffman::dump,
// myyuv_DCT/Huffman.cpp:172-241, :279-326).
//
// One lane = one 8x8 block; one wave = 64 consecutive blocks (global order,
// planes do not matter here).  The work per block is a short serial program
// with data-dependent trip counts (1..64 distinct symbols, up to 63 merges),
// so it runs one block per lane rather than one block per wave; all per-block
// state lives in LDS, lane-interleaved (word w of lane l at w*64+l), which is
// bank-conflict-free for any per-lane index.
//
// Byte-exactness: the reference's code lengths depend on libstdc++ container
// internals (SURVEY.md §7 hard part 2, App. B), so this kernel replays them:
//   * std::unordered_map<int16_t,uint8_t> iteration order: singly linked list
//     with per-bucket "before" pointers, bucket-front insertion, rehash walk,
//     prime policy 13 -> 29 -> 59 -> 127 buckets, hash(v) = (uint64)(int64)v;
//   * std::priority_queue (min-heap on freq via Compare{a.freq > b.freq}):
//     libstdc++ push_heap / pop_heap (__adjust_heap + __push_heap) exactly.
// The insert-then-erase of key 0 (Huffman.cpp:186-197) only matters through
// the rehash it may trigger, which is replayed without materialising the node.
//
// Per-lane LDS image (128 words = 512 B per lane, 32 KiB per wave):
//   words [0,32)   ZD: 64 x u16 zig-zag coefficients; after insertion each
//                  slot's low byte = map node of that symbol (POS), the high
//                  byte later holds the canonical sort order (SORT).
//   words [32,96)  NODE[64]: key:11 | cnt:7 | next:7 | bkt:7   (map phase)
//                            key:11 | cnt:7 | len:4 | rcode:8  (after depths)
//                  during the heap phase bits 18..23 hold a leaf's parent.
//   words [96,128) BKT: 128 x u8 bucket "before" pointers (map phase);
//                  HEAP: 64 x u16 (freq<<8 | id) afterwards; internal node k
//                  keeps (depth<<8 | parent) in heap slot 63-k, which the
//                  shrinking heap never reaches again.
// Output: the chunk bytes in a 160-B slot per block, lane-interleaved per wave
// ([wave][40 words][64 lanes]), plus the u8 chunk size.
#include "codec_common.hpp"

namespace myyuv_gpu {
namespace {

constexpr int kZd = 0, kNode = 32, kBkt = 96, kWords = 128;
constexpr uint32_t kNil = 127;     // next-pointer "null"
constexpr uint32_t kEmpty = 0x80;  // bucket has no before-pointer
constexpr uint32_t kHead = 0x7F;   // before-pointer = list head sentinel

struct Lane {
  uint8_t* base;  // LDS byte base of this wave's image
  int lane;
  __device__ __forceinline__ uint32_t& word(int w) const {
    return reinterpret_cast<uint32_t*>(base)[w * kWave + lane];
  }
  __device__ __forceinline__ uint16_t& u16(int area, int i) const {
    return *reinterpret_cast<uint16_t*>(base + ((area + (i >> 1)) * kWave + lane) * 4 + (i & 1) * 2);
  }
  __device__ __forceinline__ uint8_t& u8(int area, int i) const {
    return *(base + ((area + (i >> 2)) * kWave + lane) * 4 + (i & 3));
  }
};

__device__ __forceinline__ int nkey(uint32_t w) { return (int)(w << 21) >> 21; }
__device__ __forceinline__ uint32_t ncnt(uint32_t w) { return (w >> 11) & 127u; }
__device__ __forceinline__ uint32_t nnext(uint32_t w) { return (w >> 18) & 127u; }
__device__ __forceinline__ uint32_t nbkt(uint32_t w) { return w >> 25; }
__device__ __forceinline__ uint32_t set_next(uint32_t w, uint32_t nx) {
  return (w & ~(127u << 18)) | (nx << 18);
}

// Bucket count phases of the prime rehash policy for <= 65 elements
// (_Prime_rehash_policy::_M_next_bkt / _M_need_rehash): 13 buckets from the
// first insert, 29 at the 14th, 59 at the 30th, 127 at the 60th element.
struct Phase {
  uint32_t nb, r64, magic;  // buckets, 2^64 mod nb, ceil(2^32 / nb)
};
__host__ __device__ constexpr uint32_t pow2_64_mod(uint32_t m) {
  uint64_t r = 1;
  for (int i = 0; i < 64; i++) r = (r * 2) % m;
  return (uint32_t)r;
}
__device__ __forceinline__ Phase phase_of(int ph) {
  Phase p;
  p.nb = ph == 0 ? 13u : ph == 1 ? 29u : ph == 2 ? 59u : 127u;
  p.r64 = ph == 0 ? pow2_64_mod(13) : ph == 1 ? pow2_64_mod(29) : ph == 2 ? pow2_64_mod(59) : pow2_64_mod(127);
  p.magic = ph == 0 ? 330382100u : ph == 1 ? 148102321u : ph == 2 ? 72796056u : 33818641u;
  return p;
}
// hash(int16 v) % nb with hash = (size_t)(int64)v: v >= 0 -> v % nb,
// v < 0 -> (2^64 + v) % nb = (r64 + v) % nb.  t < 2^17, so the magic
// multiply is exact.
__device__ __forceinline__ uint32_t bucket_of(int v, const Phase& P) {
  const uint32_t t = (uint32_t)(v + (v < 0 ? (int)(P.r64 + 1024u * P.nb) : 0));
  const uint32_t q = __umulhi(t, P.magic);
  return t - q * P.nb;
}

// _M_insert_bucket_begin(bkt, node)
__device__ __forceinline__ void insert_bucket_begin(const Lane& L, uint32_t& head, uint32_t b,
                                                    uint32_t before, uint32_t node,
                                                    uint32_t nodeword) {
  if (before != kEmpty) {
    if (before == kHead) {
      L.word(kNode + node) = set_next(nodeword, head);
      head = node;
    } else {
      uint32_t bw = L.word(kNode + before);
      L.word(kNode + node) = set_next(nodeword, nnext(bw));
      L.word(kNode + before) = set_next(bw, node);
    }
  } else {
    L.word(kNode + node) = set_next(nodeword, head);
    if (head != kNil) L.u8(kBkt, nbkt(L.word(kNode + head))) = (uint8_t)node;
    head = node;
    L.u8(kBkt, b) = (uint8_t)kHead;
  }
}

// _M_rehash_aux(nb, true_type): re-insert every node in list order.
__device__ void rehash(const Lane& L, uint32_t& head, const Phase& P) {
#pragma unroll
  for (int w = 0; w < 32; w++) L.word(kBkt + w) = 0x80808080u;
  uint32_t p = head;
  head = kNil;
  uint32_t bbegin = 0;
  while (p != kNil) {
    const uint32_t w = L.word(kNode + p);
    const uint32_t nx = nnext(w);
    const uint32_t b = bucket_of(nkey(w), P);
    const uint32_t before = L.u8(kBkt, b);
    uint32_t newnext;
    if (before == kEmpty) {
      newnext = head;
      head = p;
      L.u8(kBkt, b) = (uint8_t)kHead;
      if (newnext != kNil) L.u8(kBkt, bbegin) = (uint8_t)p;
      bbegin = b;
    } else if (before == kHead) {
      newnext = head;
      head = p;
    } else {
      const uint32_t bw = L.word(kNode + before);
      newnext = nnext(bw);
      L.word(kNode + before) = set_next(bw, p);
    }
    L.word(kNode + p) = (w & 0x0003FFFFu) | (newnext << 18) | (b << 25);
    p = nx;
  }
}

// std::priority_queue push: push_back + __push_heap (sift up while
// parent.freq > value.freq).
__device__ __forceinline__ void heap_sift_up(const Lane& L, int hole, uint32_t e) {
  while (hole > 0) {
    const int parent = (hole - 1) >> 1;
    const uint32_t pe = L.u16(kBkt, parent);
    if ((pe >> 8) <= (e >> 8)) break;
    L.u16(kBkt, hole) = (uint16_t)pe;
    hole = parent;
  }
  L.u16(kBkt, hole) = (uint16_t)e;
}

// std::priority_queue pop: top + pop_heap (__pop_heap, __adjust_heap).
__device__ __forceinline__ uint32_t heap_pop(const Lane& L, int& len) {
  const uint32_t top = L.u16(kBkt, 0);
  const int n = --len;
  if (n > 0) {
    const uint32_t value = L.u16(kBkt, n);
    int hole = 0, child = 0;
    while (child < (n - 1) / 2) {
      child = 2 * (child + 1);
      const uint32_t right = L.u16(kBkt, child), left = L.u16(kBkt, child - 1);
      uint32_t pick = right;
      if ((right >> 8) > (left >> 8)) {
        child--;
        pick = left;
      }
      L.u16(kBkt, hole) = (uint16_t)pick;
      hole = child;
    }
    if ((n & 1) == 0 && child == (n - 2) / 2) {
      child = 2 * (child + 1);
      L.u16(kBkt, hole) = L.u16(kBkt, child - 1);
      hole = child - 1;
    }
    heap_sift_up(L, hole, value);
  }
  return top;
}

// LSB-first bit writer into the lane's interleaved output slot.
struct BitWriter {
  uint32_t* out;  // &slot[wave][0][lane]
  uint64_t acc = 0;
  int nacc = 0;
  int widx = 0;
  __device__ __forceinline__ void put(uint32_t v, int n) {
    acc |= (uint64_t)v << nacc;
    nacc += n;
    if (nacc >= 32) {
      out[widx * kWave] = (uint32_t)acc;
      widx++;
      acc >>= 32;
      nacc -= 32;
    }
  }
  __device__ __forceinline__ void align_byte() { nacc = (nacc + 7) & ~7; }
  __device__ __forceinline__ void flush() {
    if (nacc > 0) out[widx * kWave] = (uint32_t)acc;
  }
};

}  // namespace

// coef: [nblocks][64] int16 zig-zag.  slots: [ceil(n/64)][40][64] u32.
// sizes: [nblocks] u8 chunk sizes.
__global__ __launch_bounds__(64) void k_huff_encode(const int16_t* __restrict__ coef,
                                                   uint32_t nblocks,
                                                   uint32_t* __restrict__ slots,
                                                   uint8_t* __restrict__ sizes) {
  __shared__ uint32_t img[kWords * kWave];
  const int lane = threadIdx.x;
  const uint32_t g0 = blockIdx.x * kWave;
  const Lane L{reinterpret_cast<uint8_t*>(img), lane};

  // ---- stage the wave's 64 x 128 B of coefficients (coalesced 16-B loads).
  // Source dword d of block bb holds coefficients 2d, 2d+1 = ZD word d.
  {
    const uint4* src = reinterpret_cast<const uint4*>(coef + (size_t)g0 * 64);
#pragma unroll
    for (int it = 0; it < 8; it++) {
      const int c = it * kWave + lane;  // 16-B chunk index inside the wave's 8 KiB
      const int bb = c >> 3, part = c & 7;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (g0 + bb < nblocks) v = src[c];
      img[(kZd + part * 4 + 0) * kWave + bb] = v.x;
      img[(kZd + part * 4 + 1) * kWave + bb] = v.y;
      img[(kZd + part * 4 + 2) * kWave + bb] = v.z;
      img[(kZd + part * 4 + 3) * kWave + bb] = v.w;
    }
  }
  __syncthreads();
  const uint32_t g = g0 + lane;
  if (g >= nblocks) return;

  // ---- message length: strip trailing zeros (Huffman.cpp:176-190).
  int msz = 0;
  for (int i = 63; i >= 0; i--)
    if (L.u16(kZd, i) != 0) {
      msz = i + 1;
      break;
    }

  // ---- unordered_map replay: freq[d]++ for the message symbols, in order.
#pragma unroll
  for (int w = 0; w < 32; w++) L.word(kBkt + w) = 0x80808080u;
  uint32_t head = kNil;
  uint32_t n = 0;
  int ph = 0;
  Phase P = phase_of(0);
  uint32_t next_resize = 13;
  bool has_zero = false;
  for (int i = 0; i < msz; i++) {
    const int v = (int16_t)L.u16(kZd, i);
    has_zero |= (v == 0);
    uint32_t b = bucket_of(v, P);
    uint32_t before = L.u8(kBkt, b);
    uint32_t found = kNil;
    if (before != kEmpty) {
      uint32_t p = before == kHead ? head : nnext(L.word(kNode + before));
      while (p != kNil) {
        const uint32_t w = L.word(kNode + p);
        if (nbkt(w) != b) break;
        if (nkey(w) == v) {
          found = p;
          L.word(kNode + p) = w + (1u << 11);
          break;
        }
        p = nnext(w);
      }
    }
    if (found == kNil) {
      if (n == next_resize) {  // _M_need_rehash -> _M_rehash
        ph++;
        P = phase_of(ph);
        next_resize = P.nb;
        rehash(L, head, P);
        b = bucket_of(v, P);
        before = L.u8(kBkt, b);
      }
      found = n++;
      const uint32_t nodeword = ((uint32_t)v & 0x7FFu) | (1u << 11) | (b << 25);
      insert_bucket_begin(L, head, b, before, found, nodeword);
    }
    L.u16(kZd, i) = (uint16_t)found;  // POS[i]
  }
  // freq[0] probe / erase (Huffman.cpp:186-197): only its rehash is visible.
  if (!has_zero) {
    if (msz == 0) {
      L.word(kNode + 0) = (0u) | (1u << 11) | (kNil << 18);
      head = 0;
      n = 1;
      msz = 1;
      L.u16(kZd, 0) = 0;
    } else if (n == next_resize) {
      ph++;
      P = phase_of(ph);
      next_resize = P.nb;
      rehash(L, head, P);
    }
  }

  // ---- priority_queue over the map's iteration order (Huffman.cpp:198-217).
  int hlen = 0;
  for (uint32_t p = head; p != kNil;) {
    const uint32_t w = L.word(kNode + p);
    heap_sift_up(L, hlen++, (ncnt(w) << 8) | p);
    p = nnext(w);
  }
  // merges: internal node k gets id 64+k; parents: leaves in NODE bits 18..23,
  // internal nodes in heap slot 63-k (low byte).
  for (int k = 0; k + 1 < (int)n; k++) {
    const uint32_t l = heap_pop(L, hlen);
    const uint32_t r = heap_pop(L, hlen);
    const uint32_t ids[2] = {l & 0xFF, r & 0xFF};
#pragma unroll
    for (int s = 0; s < 2; s++) {
      const uint32_t id = ids[s];
      if (id < 64) {
        L.word(kNode + id) = set_next(L.word(kNode + id), (uint32_t)k);
      } else {
        L.u16(kBkt, 63 - (int)(id - 64)) = (uint16_t)k;
      }
    }
    heap_sift_up(L, hlen++, ((((l >> 8) + (r >> 8)) << 8)) | (uint32_t)(64 + k));
  }

  // ---- depths (generateCodeLength, Huffman.cpp:71-83): root = internal n-2.
  if (n >= 2) {
    const int root = (int)n - 2;
    L.u16(kBkt, 63 - root) = 0;  // depth 0
    for (int k = root - 1; k >= 0; k--) {
      const uint32_t par = L.u16(kBkt, 63 - k) & 0xFF;
      const uint32_t d = (L.u16(kBkt, 63 - (int)par) >> 8) + 1;
      L.u16(kBkt, 63 - k) = (uint16_t)(par | (d << 8));
    }
  }
  // leaf lengths, total bits, per-length counts (8 x u8 packed).
  uint32_t nbits = 0;
  uint64_t lcount = 0;
  for (uint32_t p = 0; p < n; p++) {
    const uint32_t w = L.word(kNode + p);
    uint32_t len = 1;
    if (n >= 2) len = (L.u16(kBkt, 63 - (int)nnext(w)) >> 8) + 1;
    nbits += ncnt(w) * len;
    lcount += 1ull << (8 * (len - 1));
    L.word(kNode + p) = (w & 0x3FFFFu) | (len << 18);
  }

  // ---- canonical order: (length, symbol) ascending (generateCodeLength's
  // sorted vectors in map<len, ...>).  Insertion sort of node ids into SORT.
  for (uint32_t p = 0; p < n; p++) {
    const uint32_t wp = L.word(kNode + p);
    const uint32_t kp = (((wp >> 18) & 15u) << 11) | (uint32_t)(nkey(wp) + 1024);
    int j = (int)p;
    while (j > 0) {
      const uint32_t q = L.u8(kZd, 2 * (j - 1) + 1);
      const uint32_t wq = L.word(kNode + q);
      const uint32_t kq = (((wq >> 18) & 15u) << 11) | (uint32_t)(nkey(wq) + 1024);
      if (kq <= kp) break;
      L.u8(kZd, 2 * j + 1) = (uint8_t)q;
      j--;
    }
    L.u8(kZd, 2 * j + 1) = (uint8_t)p;
  }

  // ---- chunk: u16 nbits, u8 table_bytes, groups, code bits (Huffman.cpp:279-326).
  uint32_t table_bytes = 0;
#pragma unroll
  for (int l = 0; l < 8; l++) {
    const uint32_t c = (uint32_t)(lcount >> (8 * l)) & 0xFF;
    if (c > 32) table_bytes += 2 + 44 + ((c - 32) * 11 + 7) / 8;
    else if (c > 0) table_bytes += 1 + (c * 11 + 7) / 8;
  }
  BitWriter bw;
  bw.out = slots + (size_t)blockIdx.x * (kSlotWords * kWave) + lane;
  bw.put(nbits, 16);
  bw.put(table_bytes, 8);
  uint32_t code = 0, prevlen = 0, curlen = 0, left = 0, ingroup = 0;
  for (uint32_t r = 0; r < n; r++) {
    const uint32_t p = L.u8(kZd, 2 * r + 1);
    const uint32_t w = L.word(kNode + p);
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
    // bit-reversed so the LSB-first writer emits it MSB-first.
    code <<= (len - prevlen);
    prevlen = len;
    const uint32_t rcode = __brev(code) >> (32 - len);
    L.word(kNode + p) = (w & 0x3FFFFu) | (len << 18) | (rcode << 22);
    code++;
  }
  bw.align_byte();
  for (int i = 0; i < msz; i++) {
    const uint32_t p = L.u8(kZd, 2 * i);
    const uint32_t w = L.word(kNode + p);
    bw.put(w >> 22, (int)((w >> 18) & 15u));
  }
  bw.flush();
  sizes[g] = (uint8_t)(3 + table_bytes + (nbits + 7) / 8);
}

}  // namespace myyuv_gpu
