// k_huff_decode.hip — K5: per-block chunk parse + canonical Huffman decode on
// gfx950 (Huffman::fromDump, unpack11bit, decodeSymbol, decodeFromTreeData;
// myyuv_DCT/Huffman.cpp:243-277, :54-69, :106-154).
//
// One workgroup = one wave = up to 64 consecutive blocks of ONE plane, so the
// wave's chunks are one contiguous byte range of the plane's content[]; it is
// staged into LDS with dword loads (the LDS image keeps the stream's dword
// grid), then each lane decodes its own block:
//   1. header: u16 nbits, u8 table_bytes;
//   2. table: groups ((L-1)<<5 | (n-1)) + n x 11-bit values; two passes so a
//      length's groups land together however they are ordered (std::map
//      semantics of tree_data);
//   3. symbols: the reference decodes bit-serially (puff style): at length L,
//      code = first L bits, match if code < first + count[L].  Here the next 8
//      bits are peeked once and the same test is evaluated for L = 1..8
//      (unrolled, branch-free); the smallest matching L is exactly the length
//      the bit-serial loop would stop at, including on malformed tables
//      (uint8 arithmetic of `first` kept), and the bit budget checks give the
//      same "bad code" / "unknown symbol" outcomes.
// Output: 64 int16 per block, zero-filled after the last symbol, decoded in
// zig-zag order into LDS and written out in natural order (the inverse scan
// is a compile-time permutation of registers) in the quad layout of
// codec_common.hpp that K6 reads.
#include "codec_common.hpp"
#include "k_stream.hpp"

namespace myyuv_gpu {

namespace {

constexpr int kStageWords = (kWave * kMaxChunk) / 4 + 4;
constexpr int kOutStride = 65;  // words; conflict-free for both access directions

// inverse zig-zag: c_izz[n] = position of natural index n in the scan
struct IzzTable {
  uint8_t v[64];
  constexpr IzzTable() : v{} {
    constexpr uint8_t zz[64] = MYYUV_ZIGZAG;
    for (int z = 0; z < 64; z++) v[zz[z]] = (uint8_t)z;
  }
};
constexpr IzzTable kIzz{};
constexpr const uint8_t* c_izz = kIzz.v;

__device__ __forceinline__ void record_error(unsigned long long* err, uint64_t key, int code) {
  atomicMin(err, (unsigned long long)((key << 8) | (uint64_t)code));
}

// Byte sources for one lane's chunk: the LDS stage (normal case) or global
// memory (a wave whose chunks do not fit the stage: only malformed streams
// with oversized chunk_size bytes, up to 255 B each).
struct LdsBytes {
  const uint8_t* p;
  __device__ __forceinline__ uint32_t operator[](uint32_t i) const { return p[i]; }
};
struct GlobalBytes {
  const uint8_t* in;
  uint32_t base, limit;
  __device__ __forceinline__ uint32_t operator[](uint32_t i) const {
    return base + i < limit ? in[base + i] : 0u;
  }
};

// Returns 0 or the MYYUV_E_* code of the first failure (Huffman::fromDump).
template <class Bytes, class SymAt, class OutAt>
__device__ int decode_chunk(const Bytes c, const uint32_t s, SymAt&& sym_at, OutAt&& out_at) {
  int code = 0;
  if (s < 3) {
    code = 12;
  } else {
    const uint32_t nbits = (uint32_t)c[0] | ((uint32_t)c[1] << 8);
    const uint32_t tb = c[2];
    if (nbits > 512 || 3 + tb + (nbits + 7) / 8 > s) {
      code = 12;
    } else {
      // pass 1: per-length counts (8 x u8 packed)
      uint64_t cnt = 0;
      uint32_t total = 0;
      uint32_t i = 3;
      while (i - 3 < tb) {
        const uint32_t info = c[i];
        const uint32_t L = (info >> 5) + 1, n = (info & 31) + 1;
        const uint32_t nbytes = (n * 11 + 7) / 8;
        total += n;
        if (i + 1 + nbytes > 3 + tb || total > 64) {
          code = 12;
          break;
        }
        cnt += (uint64_t)n << (8 * (L - 1));
        i += 1 + nbytes;
      }
      if (!code) {
        // offsets of each length's symbols in the flat table
        uint64_t offs = 0;
        uint32_t acc = 0;
#pragma unroll
        for (int L = 0; L < 8; L++) {
          offs |= (uint64_t)acc << (8 * L);
          acc += (uint32_t)(cnt >> (8 * L)) & 0xFF;
        }
        // pass 2: unpack the 11-bit values (unpack11bit)
        uint64_t run = 0;
        i = 3;
        while (i - 3 < tb) {
          const uint32_t info = c[i++];
          const uint32_t L = (info >> 5) + 1, n = (info & 31) + 1;
          const uint32_t base = (uint32_t)(offs >> (8 * (L - 1))) & 0xFF;
          const uint32_t done = (uint32_t)(run >> (8 * (L - 1))) & 0xFF;
          for (uint32_t k = 0; k < n; k++) {
            const uint32_t bit = 11 * k;
            const uint32_t q = i + (bit >> 3);
            const uint32_t raw = (uint32_t)c[q] | ((uint32_t)c[q + 1] << 8) | ((uint32_t)c[q + 2] << 16);
            const uint32_t u = (raw >> (bit & 7)) & 0x7FF;
            sym_at(base + done + k) = (uint16_t)(u >= 1024 ? u - 2048 : u);
          }
          run += (uint64_t)n << (8 * (L - 1));
          i += (n * 11 + 7) / 8;
        }
        // symbols
        const uint32_t bits = 3 + tb;
        uint32_t bp = 0;
        uint32_t j = 0;
        while (bp < nbits && j < 64) {
          const uint32_t q = bp >> 3;
          const uint32_t x = (uint32_t)c[bits + q] | ((uint32_t)c[bits + q + 1] << 8);
          const uint32_t w8 = __brev((x >> (bp & 7)) & 0xFF) >> 24;  // next 8 bits, MSB-first
          uint32_t first = 0, mL = 0, mIdx = 0;
          bool neg = false;
#pragma unroll
          for (uint32_t L = 1; L <= 8; L++) {
            const uint32_t cL = (uint32_t)(cnt >> (8 * (L - 1))) & 0xFF;
            const uint32_t cd = w8 >> (8 - L);
            if (mL == 0 && cd < cL + first) {
              mL = L;
              neg = cd < first;
              mIdx = ((uint32_t)(offs >> (8 * (L - 1))) & 0xFF) + (cd - first);
            }
            first = ((first + cL) << 1) & 0xFF;
          }
          if (mL == 0) {
            code = (bp + 8 > nbits) ? 10 : 11;
            break;
          }
          if (bp + mL > nbits || neg) {
            code = 10;
            break;
          }
          out_at(j++) = sym_at(mIdx);
          bp += mL;
        }
      }
    }
  }
  return code;
}

}  // namespace

__global__ __launch_bounds__(64) void k_huff_decode(const uint8_t* __restrict__ in,
                                                   const uint32_t* __restrict__ in_size,
                                                   uint32_t cap,
                                                   const StreamDesc* __restrict__ desc,
                                                   const uint32_t* __restrict__ local_off,
                                                   const uint32_t* __restrict__ tile_pre,
                                                   FrameGeom G, uint32_t tiles_p0,
                                                   uint32_t tiles_p1,
                                                   uint4* __restrict__ coef,
                                                   unsigned long long* __restrict__ err) {
  __shared__ uint32_t stage[kStageWords];
  __shared__ uint32_t symw[32 * kWave];
  __shared__ uint32_t outw[32 * kOutStride];
  if (desc->bad) return;
  const int lane = threadIdx.x;
  const uint32_t t = blockIdx.x;
  const int p = t >= tiles_p0 ? (t >= tiles_p0 + tiles_p1 ? 2 : 1) : 0;
  const uint32_t tile_in_plane = t - (p == 0 ? 0 : (p == 1 ? tiles_p0 : tiles_p0 + tiles_p1));
  const uint32_t g0 = G.cum[p] + tile_in_plane * kWave;
  const uint32_t g1 = min(g0 + kWave, G.cum[p + 1]);
  const uint32_t g = g0 + lane;
  const bool live = g < g1;
  const uint32_t limit = min(*in_size, cap);

  const uint32_t plane_pre = local_off[G.cum[p]] + tile_pre[G.cum[p] / kScanTile];
  const uint32_t gl = live ? g : g1 - 1;
  const uint32_t rel = local_off[gl] + tile_pre[gl / kScanTile] - plane_pre;
  const uint32_t s = in[desc->sizes_pos[p] + (gl - G.cum[p])];
  const uint32_t cpos = desc->content_pos[p];
  const uint32_t csize = desc->content_size[p];

  // plane-level check (DCT.cpp:21-33 reads past content_size otherwise):
  // the chunks must fit the declared content.
  bool ok = live;
  if (live && rel + s > csize) {
    record_error(err, 2ull * G.cum[p], 9 /* MYYUV_E_PLANE_CONTENT */);
    ok = false;
  }

  // ---- stage [cpos + rel(g0), cpos + rel(g1-1) + s(g1-1)) into LDS
  const uint32_t first_rel = __shfl(rel, 0, 64);
  const uint32_t last_end = __shfl(rel + s, (int)(g1 - 1 - g0), 64);
  const uint32_t a0 = cpos + first_rel;
  const uint32_t a1 = min(cpos + min(last_end, csize), limit);
  const uint32_t aw = a0 & ~3u;
  const uint32_t nwords = a1 > aw ? (a1 - aw + 3) >> 2 : 0;
  const bool fits = nwords + 2 <= (uint32_t)kStageWords;  // keep >= 8 B of zero slack
  for (uint32_t i = lane; i < kStageWords; i += kWave) {
    uint32_t v = 0;
    if (i < nwords) {
      const uint32_t a = aw + 4 * i;
      if (a + 4 <= limit) {
        v = *reinterpret_cast<const uint32_t*>(in + a);
      } else {
        for (uint32_t k = 0; k < 4; k++)
          if (a + k < limit) v |= (uint32_t)in[a + k] << (8 * k);
      }
    }
    stage[i] = v;
  }
#pragma unroll
  for (int w = 0; w < 32; w++) outw[w * kOutStride + lane] = 0;
  __syncthreads();

  const uint8_t* sb = reinterpret_cast<const uint8_t*>(stage);
  uint8_t* symb = reinterpret_cast<uint8_t*>(symw);
  auto sym_at = [&](uint32_t i) -> uint16_t& {
    return *reinterpret_cast<uint16_t*>(symb + (((i >> 1) * kWave + lane) * 4 + (i & 1) * 2));
  };
  uint8_t* outb = reinterpret_cast<uint8_t*>(outw);
  auto out_at = [&](uint32_t j) -> uint16_t& {
    return *reinterpret_cast<uint16_t*>(outb + (((j >> 1) * kOutStride + lane) * 4 + (j & 1) * 2));
  };

  int code = 0;
  if (ok) {
    const uint32_t lb = a0 + rel - first_rel - aw;  // chunk start in the stage
    if (fits) {
      code = decode_chunk(LdsBytes{sb + lb}, s, sym_at, out_at);
    } else {
      const uint32_t abs0 = cpos + rel;
      code = decode_chunk(GlobalBytes{in, abs0, limit}, s, sym_at, out_at);
    }
    if (code) record_error(err, 2ull * g + 1, code);
  }
  __syncthreads();

  // ---- write-out: zig-zag words from LDS, natural words to the quad layout
  // (Huffman.cpp:148-153 de-zig-zag; 1 KiB contiguous per quad store)
  if (live) {
    uint32_t zw[32];
#pragma unroll
    for (int w = 0; w < 32; w++) zw[w] = outw[w * kOutStride + lane];
    uint32_t nw[32];
#pragma unroll
    for (int m = 0; m < 32; m++) {
      const int z0 = c_izz[2 * m], z1 = c_izz[2 * m + 1];
      const uint32_t lo = (zw[z0 >> 1] >> (16 * (z0 & 1))) & 0xFFFFu;
      const uint32_t hi = (zw[z1 >> 1] >> (16 * (z1 & 1))) & 0xFFFFu;
      nw[m] = lo | (hi << 16);
    }
#pragma unroll
    for (int c = 0; c < 8; c++)
      coef[coef_quad(g, c)] = make_uint4(nw[4 * c], nw[4 * c + 1], nw[4 * c + 2], nw[4 * c + 3]);
  }
}

}  // namespace myyuv_gpu
