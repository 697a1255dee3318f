// k_stream.hip — the variable-length side of the codec on gfx950:
//   * k_scan_chain: exclusive scan of the u8 chunk sizes in one pass
//     (DCTYUVPlane::getContentPos, DCT.cpp:21-33, done for all planes at once),
//     decode side with the stream header checks;
//   * k_compact: chunk slots -> the DCTYUV byte stream (DCTYUV::dump /
//     DCTYUVPlane::dumpTo, DCT.cpp:63-73, 160-173, and the serial compaction of
//     applyDCTPlane, :314-322);
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
#include "k_chain.hpp"
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

// Exclusive scan of the chunk sizes in one pass (frame blockIdx.y of a batch,
// its bytes at src + blockIdx.y * src_stride): workgroup t scans tile t
// (kScanTile sizes) and finds the tile's exclusive prefix by decoupled
// look-back over the lower tiles (k_chain.hpp); local_off[g] = offset inside
// the tile, tile_pre[t] = the tile's prefix, tile_pre[ntiles] = the total.
// Element g's size byte is src[pos[p] + (g - cum[p])].  With `desc` (decode)
// every workgroup first parses the stream header (k_parse's checks, DCTYUV::load
// DCT.cpp:130-159 then DCTYUVPlane::load :39-62) for the size positions, and
// workgroup 0 publishes it for K5 (or records the header error).
__global__ __launch_bounds__(256) void k_scan_chain(const uint8_t* __restrict__ src, uint32_t src_stride,
                                                   ScanSrc S, const uint32_t* __restrict__ in_size,
                                                   uint32_t cap, FrameGeom G,
                                                   StreamDesc* __restrict__ desc,
                                                   uint32_t* __restrict__ local_off,
                                                   uint32_t* __restrict__ tile_pre, uint32_t ntiles,
                                                   unsigned long long* __restrict__ status,
                                                   uint32_t epoch,
                                                   unsigned long long* __restrict__ err) {
  __shared__ uint32_t wsum[4];
  __shared__ uint32_t s_excl;
  // frame blockIdx.y of the batch: its own sizes / stream, offsets, tile
  // prefixes and look-back chain
  const uint32_t f = blockIdx.y;
  src += (size_t)f * src_stride;
  local_off += (size_t)f * G.cum[3];
  tile_pre += (size_t)f * (ntiles + 1);
  status += (size_t)f * (ntiles + 1);
  uint32_t pos[3] = {S.pos[0], S.pos[1], S.pos[2]};
  if (desc) {
    desc += f;
    StreamPos P;
    const int code = parse_stream(src, min(in_size[f], cap), G, P);
    if (code) {
      if (blockIdx.x == 0 && threadIdx.x == 0) {
        desc->bad = 1;
        record_error(err, 2ull * f * G.cum[3], code);  // frame f's first block (0: header of frame 0)
      }
      return;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      desc->bad = 0;
      for (int p = 0; p < 3; p++) {
        desc->sizes_pos[p] = P.sizes_pos[p];
        desc->content_pos[p] = P.content_pos[p];
        desc->content_size[p] = P.content_size[p];
      }
    }
    for (int p = 0; p < 3; p++) pos[p] = P.sizes_pos[p];
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
  const uint32_t agg = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  if (wave == 0) {
    const uint32_t ex = chained_prefix(status, blockIdx.x, 0, agg, epoch);
    if (lane == 0) s_excl = ex;
  }
  uint32_t carry = 0;
  for (int w = 0; w < wave; w++) carry += wsum[w];
  uint32_t run = carry + incl - sum;
#pragma unroll
  for (int i = 0; i < kScanPerThread; i++) {
    const uint32_t g = base + i;
    if (g < S.cum[3]) local_off[g] = run;
    run += v[i];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    tile_pre[blockIdx.x] = s_excl;
    if (blockIdx.x == ntiles - 1) tile_pre[ntiles] = s_excl + agg;
  }
}

__device__ __forceinline__ uint32_t scanned(const uint32_t* local_off, const uint32_t* tile_pre,
                                            uint32_t g) {
  return local_off[g] + tile_pre[g / kScanTile];
}

// Compaction: one workgroup = up to 256 consecutive blocks of one plane of
// frame blockIdx.y, one lane per block (chunk).
__global__ __launch_bounds__(256) void k_compact(const uint32_t* __restrict__ slots,
                                                const uint8_t* __restrict__ sizes,
                                                const uint32_t* __restrict__ local_off,
                                                const uint32_t* __restrict__ tile_pre,
                                                FrameGeom G, uint32_t tiles_p0, uint32_t tiles_p1,
                                                uint8_t* __restrict__ out, uint32_t cap,
                                                uint32_t* __restrict__ out_size,
                                                unsigned long long* __restrict__ err) {
  // frame blockIdx.y of the batch: slots / sizes at batch-global block
  // gbase + g, its scan, its output slot of `cap` bytes
  const uint32_t f = blockIdx.y, gbase = f * G.cum[3];
  const uint32_t ntiles = (G.cum[3] + kScanTile - 1) / kScanTile;
  sizes += gbase;
  local_off += gbase;
  tile_pre += (size_t)f * (ntiles + 1);
  out += (size_t)f * cap;
  out_size += f;
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
      if (total > cap) record_error(err, 0, 5 /* MYYUV_E_CAPACITY */);  // any frame
    }
  }
  if (total > cap) return;

  const uint32_t g = g0 + threadIdx.x;
  if (g >= g1) return;
  const uint32_t sz = sizes[g];
  out[12ull + 8ull * (p + 1) + plane_pre + g] = (uint8_t)sz;  // chunk_size[k]
  // The chunk's bytes [pos, end) go straight to the stream: the image words
  // strictly inside the range are this lane's alone (dword stores); the first
  // and last words can hold a neighbour's bytes, so only this chunk's bytes of
  // them are stored (byte stores: no read-modify-write, no atomics, no LDS).
  // Slot words are loaded 8 at a time with no predication (a slot is always
  // kSlotWords = 5 x 8 words long): one HBM round trip per batch.
  const uint64_t pos = 12ull + 8ull * (p + 1) + G.cum[p + 1] + scanned(local_off, tile_pre, g);
  const uint64_t end = pos + sz;
  const uint64_t a0 = pos & ~3ull, al = (end - 1) & ~3ull;
  const uint32_t sh = (uint32_t)(pos & 3) * 8;
  const uint32_t ga = gbase + g;
  const uint32_t* slot = slots + (size_t)(ga / kWave) * (kSlotWords * kWave) + (ga % kWave);
  const uint32_t nw = (sz + 3) >> 2;
  if (nw == 0) return;  // (a chunk is at least 7 bytes; a corrupt size of 0 writes nothing)
  auto edge = [&](uint64_t a, uint32_t v) {
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (a + k >= pos && a + k < end) out[a + k] = (uint8_t)(v >> (8 * k));
  };
  uint32_t carry = 0;  // bits of the previous slot word shifted past its stream word
  for (uint32_t j0 = 0; j0 < nw; j0 += 8) {
    uint32_t d[8];
#pragma unroll
    for (int k = 0; k < 8; k++) d[k] = slot[(j0 + k) * kWave];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t j = j0 + k;
      if (j < nw) {
        const uint32_t v = sh ? (d[k] << sh) | carry : d[k];
        carry = sh ? d[k] >> (32 - sh) : 0u;
        const uint64_t a = a0 + 4ull * j;
        if (a == a0 || a == al)
          edge(a, v);
        else
          *reinterpret_cast<uint32_t*>(out + a) = v;
      }
    }
  }
  if (a0 + 4ull * nw == al) edge(al, carry);
}

}  // namespace myyuv_gpu
