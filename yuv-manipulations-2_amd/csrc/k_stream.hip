// k_stream.hip — the variable-length side of the codec on gfx950:
//   * k_scan_tiles / k_scan_sums: exclusive scan of the u8 chunk sizes
//     (DCTYUVPlane::getContentPos, DCT.cpp:21-33, done for all planes at once);
//   * k_compact: chunk slots -> the DCTYUV byte stream (DCTYUV::dump /
//     DCTYUVPlane::dumpTo, DCT.cpp:63-73, 160-173, and the serial compaction of
//     applyDCTPlane, :314-322);
//   * k_parse: decode-side validation of the stream headers (DCTYUV::load,
//     DCTYUVPlane::load, DCT.cpp:39-62, 130-159).
//
// Stream layout: u32 plane_size[3]; per plane p:
//   u32 nblocks, u32 content_size, u8 chunk_size[nblocks], u8 content[...].
// With blocks numbered globally (plane-major) and off[g] the exclusive scan of
// all chunk sizes, block g of plane p sits at
//   content: 12 + 8(p+1) + cum[p+1] + off[g]
//   size:    12 + 8(p+1) + off[cum[p]] + g
//   header:  12 + 8p + cum[p] + off[cum[p]]
// so one global scan places every byte of the stream.
#include "codec_common.hpp"
#include "k_stream.hpp"

namespace myyuv_gpu {

namespace {

__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  return v;
}

__device__ __forceinline__ void record_error(unsigned long long* err, uint64_t key, int code) {
  atomicMin(err, (unsigned long long)((key << 8) | (uint64_t)code));
}

__device__ __forceinline__ int plane_of(const uint32_t cum[4], uint32_t g) {
  return g >= cum[1] ? (g >= cum[2] ? 2 : 1) : 0;
}

}  // namespace

// Exclusive scan inside tiles of kScanTile elements.  Element g's size byte is
// src[pos[p] + (g - cum[p])] (pos: per-plane start of the u8 size array, read
// from `desc` when given, so the decoder can scan sizes in place).
__global__ __launch_bounds__(256) void k_scan_tiles(const uint8_t* __restrict__ src,
                                                   ScanSrc S, const StreamDesc* __restrict__ desc,
                                                   uint32_t* __restrict__ local_off,
                                                   uint32_t* __restrict__ tile_sum) {
  __shared__ uint32_t wsum[4];
  uint32_t pos[3] = {S.pos[0], S.pos[1], S.pos[2]};
  if (desc) {
    if (desc->bad) return;
    pos[0] = desc->sizes_pos[0];
    pos[1] = desc->sizes_pos[1];
    pos[2] = desc->sizes_pos[2];
  }
  const uint32_t base = blockIdx.x * kScanTile + threadIdx.x * kScanPerThread;
  uint32_t v[kScanPerThread];
  uint32_t sum = 0;
#pragma unroll
  for (int i = 0; i < kScanPerThread; i++) {
    const uint32_t g = base + i;
    uint32_t s = 0;
    if (g < S.cum[3]) {
      const int p = plane_of(S.cum, g);
      s = src[pos[p] + (g - S.cum[p])];
    }
    v[i] = s;
    sum += s;
  }
  const uint32_t incl = wave_inclusive_scan(sum);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  uint32_t carry = 0;
  for (int w = 0; w < wave; w++) carry += wsum[w];
  uint32_t run = carry + incl - sum;
#pragma unroll
  for (int i = 0; i < kScanPerThread; i++) {
    const uint32_t g = base + i;
    if (g < S.cum[3]) local_off[g] = run;
    run += v[i];
  }
  if (threadIdx.x == 255) tile_sum[blockIdx.x] = run;
}

// One workgroup: exclusive scan of the tile sums in place, total appended.
__global__ __launch_bounds__(256) void k_scan_sums(uint32_t* __restrict__ tile_sum,
                                                  uint32_t ntiles,
                                                  const StreamDesc* __restrict__ desc) {
  __shared__ uint32_t wsum[4];
  if (desc && desc->bad) return;
  uint32_t carry = 0;
  for (uint32_t base = 0; base < ntiles; base += 256) {
    const uint32_t i = base + threadIdx.x;
    const uint32_t v = i < ntiles ? tile_sum[i] : 0;
    const uint32_t incl = wave_inclusive_scan(v);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t c = carry;
    for (int w = 0; w < wave; w++) c += wsum[w];
    if (i < ntiles) tile_sum[i] = c + incl - v;
    const uint32_t total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
    carry += total;
  }
  if (threadIdx.x == 0) tile_sum[ntiles] = carry;
}

__device__ __forceinline__ uint32_t scanned(const uint32_t* local_off, const uint32_t* tile_pre,
                                            uint32_t g) {
  return local_off[g] + tile_pre[g / kScanTile];
}

// Compaction: one workgroup = up to 256 consecutive blocks of one plane.
// Chunks are OR-ed into an LDS image aligned to the stream's dword grid, then
// written with dword stores (edge words byte by byte: they are shared with the
// neighbouring workgroups' bytes).
__global__ __launch_bounds__(256) void k_compact(const uint32_t* __restrict__ slots,
                                                const uint8_t* __restrict__ sizes,
                                                const uint32_t* __restrict__ local_off,
                                                const uint32_t* __restrict__ tile_pre,
                                                FrameGeom G, uint32_t tiles_p0, uint32_t tiles_p1,
                                                uint8_t* __restrict__ out, uint32_t cap,
                                                uint32_t* __restrict__ out_size,
                                                unsigned long long* __restrict__ err) {
  __shared__ uint32_t img[(256 * kMaxChunk) / 4 + 2];
  const uint32_t t = blockIdx.x;
  const int p = t >= tiles_p0 ? (t >= tiles_p0 + tiles_p1 ? 2 : 1) : 0;
  const uint32_t tile_in_plane = t - (p == 0 ? 0 : (p == 1 ? tiles_p0 : tiles_p0 + tiles_p1));
  const uint32_t g0 = G.cum[p] + tile_in_plane * 256;
  const uint32_t g1 = min(g0 + 256, G.cum[p + 1]);
  const uint32_t plane_pre = scanned(local_off, tile_pre, G.cum[p]);
  const uint32_t total_content = tile_pre[(G.cum[3] + kScanTile - 1) / kScanTile];
  const uint64_t total = 12ull + 24ull + G.cum[3] + total_content;

  // headers: first workgroup of each plane
  if (g0 == G.cum[p] && threadIdx.x < 3) {
    const uint32_t next_pre = p < 2 ? scanned(local_off, tile_pre, G.cum[p + 1]) : total_content;
    const uint32_t nb = G.cum[p + 1] - G.cum[p];
    const uint32_t content = next_pre - plane_pre;
    if (threadIdx.x == 0 && total <= cap) {
      const uint64_t hpos = 12ull + 8ull * p + G.cum[p] + plane_pre;
      const uint32_t vals[2] = {nb, content};
      for (int k = 0; k < 8; k++) out[hpos + k] = (uint8_t)(vals[k >> 2] >> (8 * (k & 3)));
      const uint32_t psize = 8 + nb + content;
      for (int k = 0; k < 4; k++) out[4 * p + k] = (uint8_t)(psize >> (8 * k));
    }
    if (p == 0 && threadIdx.x == 1) {
      *out_size = (uint32_t)total;
      if (total > cap) record_error(err, 0, 5 /* MYYUV_E_CAPACITY */);
    }
  }
  if (total > cap) return;

  const uint32_t g = g0 + threadIdx.x;
  const bool live = g < g1;
  const uint64_t cbase = 12ull + 8ull * (p + 1) + G.cum[p + 1];  // + off[g]
  const uint32_t off0 = scanned(local_off, tile_pre, g0);
  const uint64_t start = cbase + off0;
  const uint32_t end_off = scanned(local_off, tile_pre, g1 - 1) + sizes[g1 - 1];
  const uint64_t end = cbase + end_off;
  const uint64_t astart = start & ~3ull;
  const uint32_t nwords = (uint32_t)((end - astart + 3) >> 2);
  for (uint32_t i = threadIdx.x; i < nwords; i += 256) img[i] = 0;
  __syncthreads();

  if (live) {
    const uint32_t s = sizes[g];
    out[12ull + 8ull * (p + 1) + plane_pre + g] = (uint8_t)s;  // chunk_size[k]
    const uint32_t lo = (uint32_t)(start - astart) + (scanned(local_off, tile_pre, g) - off0);
    const uint32_t* slot = slots + (size_t)(g / kWave) * (kSlotWords * kWave) + (g % kWave);
    const uint32_t nw = (s + 3) >> 2;
    const uint32_t sh = (lo & 3) * 8;
    for (uint32_t j = 0; j < nw; j++) {
      const uint32_t d = slot[j * kWave];
      const uint32_t wi = (lo >> 2) + j;
      atomicOr(&img[wi], d << sh);
      if (sh) atomicOr(&img[wi + 1], d >> (32 - sh));
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nwords; i += 256) {
    const uint64_t a = astart + 4ull * i;
    const uint32_t w = img[i];
    if (a >= start && a + 4 <= end) {
      *reinterpret_cast<uint32_t*>(out + a) = w;
    } else {
      for (int k = 0; k < 4; k++) {
        const uint64_t b = a + k;
        if (b >= start && b < end) out[b] = (uint8_t)(w >> (8 * k));
      }
    }
  }
}

// Decode-side header parse, one thread, in the reference's check order
// (DCTYUV::load :130-159, then DCTYUVPlane::load :39-62 per plane).  Stricter
// than the reference where it is undefined (see oracle_decompress).
__global__ void k_parse(const uint8_t* __restrict__ in, const uint32_t* __restrict__ in_size,
                        uint32_t cap, FrameGeom G, StreamDesc* __restrict__ desc,
                        unsigned long long* __restrict__ err) {
  if (threadIdx.x != 0) return;
  auto rd32 = [&](uint64_t a) -> uint32_t {
    return (uint32_t)in[a] | ((uint32_t)in[a + 1] << 8) | ((uint32_t)in[a + 2] << 16) |
           ((uint32_t)in[a + 3] << 24);
  };
  int code = 0;
  const uint32_t size = min(*in_size, cap);
  uint32_t ps[3] = {0, 0, 0};
  uint32_t hn[3] = {0, 0, 0}, hc[3] = {0, 0, 0};
  uint64_t poff[3] = {12, 0, 0};
  if (size <= 12) {
    code = 6;
  } else {
    for (int p = 0; p < 3; p++) ps[p] = rd32(4 * p);
    if (12ull + ps[0] + ps[1] + ps[2] > size) code = 6;
  }
  if (!code) {
    poff[1] = poff[0] + ps[0];
    poff[2] = poff[1] + ps[1];
    for (int p = 0; p < 3 && !code; p++) {
      if (ps[p] <= 8) { code = 7; break; }
      hn[p] = rd32(poff[p]);
      hc[p] = rd32(poff[p] + 4);
      if (hn[p] == 0) code = 8;
      else if (hc[p] == 0) code = 9;
      else if (8ull + hn[p] + hc[p] > ps[p]) code = 7;
    }
  }
  if (!code) {
    for (int p = 0; p < 3 && !code; p++)
      if (hn[p] < G.cum[p + 1] - G.cum[p]) code = 8;
  }
  if (code) {
    desc->bad = 1;
    record_error(err, 0, code);
    return;
  }
  desc->bad = 0;
  for (int p = 0; p < 3; p++) {
    desc->sizes_pos[p] = (uint32_t)(poff[p] + 8);
    desc->content_pos[p] = (uint32_t)(poff[p] + 8 + hn[p]);
    desc->content_size[p] = hc[p];
  }
}

}  // namespace myyuv_gpu
