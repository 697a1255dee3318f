// k_stream.hip — the variable-length side of the codec on gfx950:
//   * k_scan_chain: exclusive scan of the u8 chunk sizes in one pass
//     (DCTYUVPlane::getContentPos, DCT.cpp:21-33, done for all planes at once),
//     decode side with the stream header checks;
//   * k_tile_scan + k_stream_out: K2's tiles -> the DCTYUV byte stream
//     (DCTYUV::dump / DCTYUVPlane::dumpTo, DCT.cpp:63-73, 160-173, and the
//     serial compaction of applyDCTPlane, :314-322): a scan of per-tile
//     totals, then the chunks of each tile;
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

// The same by DPP (rows of 16 by row_shr 1, 2, 4, 8, then row_bcast 15 / 31
// across rows): no LDS round trip.  Every lane of the wave must be active
// (under a partial EXEC, inactive lanes pass nothing on).
__device__ __forceinline__ uint32_t wave_inclusive_scan_dpp(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return x;
}

// Lane i + 1's value in lane i (DPP wave_shl:1; lane 63 gets 0), every lane
// active.
__device__ __forceinline__ uint32_t wave_next_lane(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xF, 0xF, false);
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
// the tile, written only where a decoder wave's 64-block group starts (g -
// cum[p] a multiple of 64: the decoders scan their own 64 sizes from there),
// tile_pre[t] = the tile's prefix, tile_pre[ntiles] = the total.
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
        record_error(err, 2ull * (G.fbase + f) * G.cum[3], code);  // frame f's first block (0: header of frame 0)
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
  uint32_t sum = 0, lead = 0;  // lead bit i: element i starts a decode group
#pragma unroll
  for (int i = 0; i < kScanPerThread; i++) {
    const uint32_t g = base + i;
    uint32_t s = 0;
    if (g < S.cum[3]) {
      const int p = plane_of(S.cum, g);
      s = src[pos[p] + (g - S.cum[p])];
      lead |= (((g - S.cum[p]) & (kWave - 1)) == 0 ? 1u : 0u) << i;
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
    if ((lead >> i) & 1u) local_off[base + i] = run;  // the decoders read group starts only
    run += v[i];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    tile_pre[blockIdx.x] = s_excl;
    if (blockIdx.x == ntiles - 1) tile_pre[ntiles] = s_excl + agg;
  }
}

struct alignas(4) Dw4 {  // a 16-byte store at a dword-aligned address (global_store_dwordx4)
  uint32_t x, y, z, w;
};

// k_stream_out: source words a lane loads in its first round trip (chunks of
// up to 4 kVw - 3 bytes are copied from registers with static indices)
constexpr uint32_t kVw = 16;
typedef __attribute__((address_space(1))) uint32_t gu32;  // global loads, not flat

__device__ __forceinline__ uint32_t scanned(const uint32_t* local_off, const uint32_t* tile_pre,
                                            uint32_t g) {
  return local_off[g] + tile_pre[g / kScanTile];
}

// Compress side, after K2 and the overflow passes (codec_common.hpp, K2 -> K4):
//   k_tile_scan: one workgroup per frame: the exclusive scan of the frame's
//     tile totals (the tiles' share of DCTYUVPlane::getContentPos, DCT.cpp:21-33),
//     the plane headers and plane sizes (DCTYUVPlane::dumpTo / DCTYUV::dump,
//     DCT.cpp:63-73, 160-173) and the payload size;
//   k_stream_out: one workgroup per tile: the chunk_size[] bytes and the
//     chunks in block order (applyDCTPlane's serial compaction, :314-322).
// A frame has ~1.1k tiles (4032x3008): one workgroup scans them in a few
// passes, so no look-back chain is needed anywhere.
__global__ __launch_bounds__(256) void k_tile_scan(uint32_t* __restrict__ tinfo, FrameGeom G,
                                                  uint8_t* __restrict__ out, uint32_t cap,
                                                  uint32_t* __restrict__ out_size,
                                                  unsigned long long* __restrict__ err) {
  // 256 threads (a small workgroup finds a free slot at once among the other
  // launch groups' kernels): thread i scans tiles [i * per, (i + 1) * per),
  // their totals loaded kTsBatch at a time with every load in flight together
  // (one dependent round trip per tile measured 14 us per 4032x3008 frame,
  // 22 us per 8192x8192 one), and kept in registers for the prefix pass
  constexpr uint32_t kTsBatch = 8;
  // tiles per thread kept in registers between the two passes (256 x 32 =
  // 8,192 tiles: an 8192x8192 frame has 6,144); above, the second pass
  // reloads its totals, a batch at a time
  constexpr uint32_t kTsKeep = 32;
  __shared__ uint32_t s_w[4];
  __shared__ uint32_t s_carry;
  __shared__ uint32_t s_pp[3];  // the content prefixes at the planes' first tiles
  const uint32_t f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t ntile = G.tcum[3];
  const uint32_t per = (ntile + 255) / 256;
  uint32_t* info = tinfo + (size_t)f * ntile * kTInfoWords;
  auto total = [&](uint32_t t) -> uint32_t {  // the tile's overflow + dense chunk bytes (words 0..4)
    const uint32_t* w = info + (size_t)t * kTInfoWords;
    const uint4 a = *reinterpret_cast<const uint4*>(w);
    return a.x + a.y + a.z + a.w + w[4];
  };
  // tiles k0 .. k0 + 7 of this thread: unconditional loads at clamped
  // indices, so all eight are in flight together (a guarded load is a branch
  // with its own wait)
  auto batch = [&](uint32_t k0, uint32_t (&x)[kTsBatch]) {
#pragma unroll
    for (uint32_t j = 0; j < kTsBatch; j++) {
      const uint32_t t = tid * per + k0 + j;
      const uint32_t tv = total(min(t, ntile - 1));
      x[j] = (k0 + j < per && t < ntile) ? tv : 0u;
    }
  };
  const bool kept = per <= kTsKeep;
  uint32_t v = 0, keep[kTsKeep];
  if (kept) {
#pragma unroll
    for (uint32_t k0 = 0; k0 < kTsKeep; k0 += kTsBatch) {
      uint32_t x[kTsBatch] = {};
      if (k0 < per) batch(k0, x);
#pragma unroll
      for (uint32_t j = 0; j < kTsBatch; j++) {
        v += x[j];
        keep[k0 + j] = x[j];
      }
    }
  } else {
    for (uint32_t k0 = 0; k0 < per; k0 += kTsBatch) {
      uint32_t x[kTsBatch];
      batch(k0, x);
#pragma unroll
      for (uint32_t j = 0; j < kTsBatch; j++) v += x[j];
    }
  }
  const uint32_t incl = wave_inclusive_scan_dpp(v);  // (every thread active)
  if (lane == 63) s_w[wave] = incl;
  if (tid == 0) s_pp[0] = 0u;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (uint32_t k = 0; k < 4; k++) {
    pre += k < wave ? s_w[k] : 0u;
    tot += s_w[k];
  }
  pre += incl - v;
  if (kept) {
#pragma unroll
    for (uint32_t j = 0; j < kTsKeep; j++) {
      const uint32_t t = tid * per + j;
      if (j < per && t < ntile) {
        info[(size_t)t * kTInfoWords + kTInfoPrefix] = pre;
        if (t == G.tcum[1]) s_pp[1] = pre;
        if (t == G.tcum[2]) s_pp[2] = pre;
        pre += keep[j];
      }
    }
  } else {
    for (uint32_t k0 = 0; k0 < per; k0 += kTsBatch) {
      uint32_t x[kTsBatch];
      batch(k0, x);
#pragma unroll
      for (uint32_t j = 0; j < kTsBatch; j++) {
        const uint32_t t = tid * per + k0 + j;
        if (k0 + j < per && t < ntile) {
          info[(size_t)t * kTInfoWords + kTInfoPrefix] = pre;
          if (t == G.tcum[1]) s_pp[1] = pre;
          if (t == G.tcum[2]) s_pp[2] = pre;
          pre += x[j];
        }
      }
    }
  }
  if (tid == 0) s_carry = tot;
  __syncthreads();
  // plane headers: the prefixes at the planes' first tiles (kept in LDS by
  // their threads above; __syncthreads orders them; no read back of tinfo)
  if (tid < 3) {
    const int p = (int)tid;
    const uint32_t total = s_carry;
    const uint32_t ppre = s_pp[p];
    const uint32_t pend = p < 2 ? s_pp[p + 1] : total;
    const uint32_t nb = G.cum[p + 1] - G.cum[p], content = pend - ppre;
    uint8_t* o = out + (size_t)f * cap;
    const uint64_t hpos = 12ull + 8ull * p + G.cum[p] + ppre;
    if (hpos + 8 <= cap) {
      const uint32_t vals[2] = {nb, content};
      for (int k = 0; k < 8; k++) o[hpos + k] = (uint8_t)(vals[k >> 2] >> (8 * (k & 3)));
    }
    const uint32_t psize = 8 + nb + content;
    for (int k = 0; k < 4; k++)
      if (4u * p + k < cap) o[4 * p + k] = (uint8_t)(psize >> (8 * k));
    if (p == 0) {
      const uint64_t bytes = 12ull + 24ull + G.cum[3] + total;
      out_size[f] = (uint32_t)bytes;
      if (bytes > cap) record_error(err, 0, 5 /* MYYUV_E_CAPACITY, any frame */);
    }
  }
}

// One tile: its chunks, in block order, from the K2 runs / overflow slots
// straight into the stream, one lane per block.  Every stream dword inside a
// plane's content is stored once, by the chunk owning its first byte, with
// the next chunk's first bytes — at most 3, so always the next chunk's header
// (u16 nbits, u8 table_bytes), which the next lane loads anyway — completing
// its last dword.  Only where the content meets other data (a plane's size
// array before its first chunk, the next plane's header after its last) are
// the shared dwords written with byte stores.  No LDS image, no atomics.
__global__ __launch_bounds__(256) void k_stream_out(const uint32_t* __restrict__ stage,
                                                    const uint32_t* __restrict__ tinfo,
                                                    const uint8_t* __restrict__ sizes,
                                                    const uint32_t* __restrict__ srcoff,
                                                    const uint32_t* __restrict__ oslots, FrameGeom G,
                                                    uint8_t* __restrict__ out, uint32_t cap, uint32_t W) {
  __shared__ uint32_t s_wt[4], s_hdr[4];
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  // the kernel arguments this workgroup uses, consumed at once (the compiler
  // would otherwise load them in three dependent batches, each where it is
  // first used)
  uint32_t ntile = G.tcum[3], nframes = G.nframes, tc1 = G.tcum[1], tc2 = G.tcum[2];
  uint32_t c1 = G.cum[1], c2 = G.cum[2], c3 = G.cum[3];
  asm volatile("" : "+s"(ntile), "+s"(nframes), "+s"(tc1), "+s"(tc2), "+s"(c1), "+s"(c2), "+s"(c3), "+s"(cap),
               "+s"(stage), "+s"(oslots), "+s"(W));
  // XCD-aware order: workgroups are dealt round-robin over the 8 XCDs (b and
  // b + 8 share one L2), and a K2 window's W tiles read interleaved
  // pieces of the same stage lines, so they go to one XCD: workgroup L takes
  // batch tile W * (8 * (L / (8 W)) + L % 8) + (L / 8) % W (a bijection on
  // the grid, a multiple of 8 W; W: the launch's K2 window, k2_win)
  const uint32_t L = blockIdx.x, slot = L >> 3, wl = (uint32_t)__builtin_ctz(W);
  const uint32_t T0 = (((slot >> wl) * 8u + (L & 7u)) << wl) + (slot & (W - 1u));
  // a surplus workgroup (the grid is a multiple of 8 * W) runs the
  // first round trip on the last tile and returns after it: no branch ahead
  // of the kernel-argument and first loads
  const bool surplus = T0 >= ntile * nframes;
  const uint32_t T = surplus ? ntile * nframes - 1 : T0;
  const uint32_t f = T / ntile, t = T - f * ntile;
  const int p = t >= tc1 ? (t >= tc2 ? 2 : 1) : 0;  // tile_plane
  // the plane's fields by static index (a dynamic index into the kernel
  // argument G is a scalar load: one more dependent round trip)
  auto sel3 = [p](uint32_t a0, uint32_t a1, uint32_t a2) { return p == 0 ? a0 : (p == 1 ? a1 : a2); };
  const uint32_t cum_p = sel3(0u, c1, c2), cum_p1 = sel3(c1, c2, c3);  // (cum[0] = tcum[0] = 0)
  const uint32_t tcum_p = sel3(0u, tc1, tc2);
  const uint32_t g0 = cum_p + (t - tcum_p) * kK2Group;
  const uint32_t nloc = min(kK2Group, cum_p1 - g0);
  const uint32_t gb = f * c3 + g0;
  out += (size_t)f * cap;
  const bool live = tid < nloc;
  const bool plane_end = g0 + nloc == cum_p1;
  // Round trip 1, every load unconditional (a guarded load is a branch with
  // its own wait): the tile's and the plane's content prefixes, the lane's
  // chunk size and source offset, and the source offset of the block after
  // the tile (whose header completes the tile's last dword when the plane
  // goes on; clamped to the tile's last block when it does not)
  uint32_t x = tinfo[(size_t)T * kTInfoWords + kTInfoPrefix];  // the tile's content prefix
  uint32_t ppre = tinfo[((size_t)f * ntile + tcum_p) * kTInfoWords + kTInfoPrefix];
  const uint32_t gl = gb + min(tid, nloc - 1);
  uint32_t sz0 = sizes[gl], so0 = srcoff[gl];
  uint32_t so1 = srcoff[gb + (plane_end ? nloc - 1 : nloc)];
  // (consumed here, so the compiler issues them together and waits once,
  // instead of sinking each scalar load to its first use)
  asm volatile("" : "+s"(x), "+s"(ppre), "+s"(so1), "+v"(sz0), "+v"(so0));
  if (surplus) return;
  const uint32_t sz = live ? sz0 : 0u;
  const uint32_t so = live ? so0 : 0u;
  const uint32_t* src;
  uint32_t sh;  // source byte misalignment
  if (so == kSrcOverflow) {
    src = oslots + (size_t)(gb + tid) * kSlotWords;
    sh = 0;
  } else {
    src = stage + (size_t)win_first_tile(T, W) * (kTileCap / 4) + (so >> 2);  // (window-relative)
    sh = so & 3u;
  }
  const uint32_t* s1 = plane_end ? stage
                       : so1 == kSrcOverflow ? oslots + (size_t)(gb + nloc) * kSlotWords
                                             : stage + (size_t)win_first_tile(T + 1, W) * (kTileCap / 4) + (so1 >> 2);
  const uint32_t r1 = plane_end || so1 == kSrcOverflow ? 0u : so1 & 3u;
  // Round trip 2: the chunk's first kVw source words (every chunk of the
  // bench frame: its longest is 55 bytes; predicated per word: most chunks
  // are a few words, and unconditional loads measured slower), which also
  // give its header, and the next tile's first header
  const uint32_t nsrc = (sh + sz + 3) >> 2;
  const gu32* gsrc = (const gu32*)src;
  uint32_t v[kVw];
#pragma unroll
  for (uint32_t k = 0; k < kVw; k++) v[k] = (k < nsrc) ? gsrc[k] : 0u;
  const uint32_t n0 = s1[0], n1 = s1[1];
  const uint32_t nxh = plane_end ? 0u : (r1 ? (n0 >> (8 * r1)) | (n1 << (32 - 8 * r1)) : n0);
  const uint32_t hdr = sh ? (v[0] >> (8 * sh)) | (v[1] << (32 - 8 * sh)) : v[0];
  // ---- offsets in the tile (block order), the next lane's header (the
  // whole workgroup is active here: DPP forms)
  const uint32_t incl = wave_inclusive_scan_dpp(sz);
  if (lane == 63) s_wt[wave] = incl;
  if (lane == 0) s_hdr[wave] = hdr;
  __syncthreads();
  uint32_t o = incl - sz;
#pragma unroll
  for (uint32_t w = 0; w < 4; w++) o += w < wave ? s_wt[w] : 0u;
  uint32_t nh = wave_next_lane(hdr);
  if (lane == 63) nh = wave < 3 ? s_hdr[wave + 1] : 0u;
  if (tid == nloc - 1) nh = nxh;
  const bool has_next = tid + 1 < nloc || !plane_end;  // a chunk follows in this plane
  // ---- chunk_size[] bytes (DCTYUVPlane layout: after the plane's 8-byte header)
  const uint64_t spos = 12ull + 8ull * (p + 1) + ppre + g0;
  if (live && spos + tid < cap) out[spos + tid] = (uint8_t)sz;
  if (!live || sz == 0) return;
  const uint64_t P = 12ull + 8ull * (p + 1) + cum_p1 + x + o;  // the chunk's stream position
  if (P + sz > cap) return;  // (capacity: k_tile_scan reports it)
  const uint32_t lead = (uint32_t)((4u - (uint32_t)(P & 3u)) & 3u);  // chunk bytes before the first own dword
  const bool plane_first = g0 + tid == cum_p;
  if (plane_first && lead) {  // the dword before is shared with the size array
    for (uint32_t k = 0; k < lead; k++) out[P + k] = (uint8_t)(hdr >> (8 * k));  // (hdr: chunk bytes 0..3)
  }
  if (sh + sz <= 4u * kVw) {
    // ---- the chunk in registers: a[m] = chunk bytes lead + 4m .. +3, i.e.
    // source bytes d + 4m (d = sh + lead <= 6: word i0 + m, shifted by qb) —
    // static indices only (a per-lane index into v[] is a select chain)
    const uint32_t d = sh + lead, qb = d & 3u;
    const bool i1 = d >= 4u;
    uint32_t u[kVw + 1], a[kVw];
#pragma unroll
    for (uint32_t m = 0; m < kVw; m++) u[m] = i1 ? (m + 1 < kVw ? v[m + 1] : 0u) : v[m];
    u[kVw] = 0u;
#pragma unroll
    for (uint32_t m = 0; m < kVw; m++) a[m] = __builtin_amdgcn_alignbyte(u[m + 1], u[m], qb);
    const uint32_t nb = sz > lead ? sz - lead : 0u;  // chunk bytes from the first own dword
    const uint32_t nq = nb >> 4, nt = (nb >> 2) & 3u, rem = nb & 3u;
    uint8_t* o = out + P + lead;  // (4-byte aligned)
#pragma unroll
    for (uint32_t it = 0; it < kVw / 4; it++)
      if (it < nq) *reinterpret_cast<Dw4*>(o + 16 * it) = Dw4{a[4 * it], a[4 * it + 1], a[4 * it + 2], a[4 * it + 3]};
    // the words after the last whole quad (4nq .. 4nq + nt - 1), then the
    // partial word 4nq + nt completed with the next chunk's first bytes
    uint32_t g[4];
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) g[j] = nq & 2u ? (nq & 1u ? a[12 + j] : a[8 + j]) : (nq & 1u ? a[4 + j] : a[j]);
    uint8_t* ot = o + 16 * nq;
#pragma unroll
    for (uint32_t j = 0; j < 3; j++)
      if (j < nt) *reinterpret_cast<uint32_t*>(ot + 4 * j) = g[j];
    if (rem) {
      const uint32_t w = nt & 2u ? (nt & 1u ? g[3] : g[2]) : (nt & 1u ? g[1] : g[0]);
      const uint64_t pk = P + sz - rem;  // = ot + 4 nt
      if (has_next && pk + 4 <= cap) {
        *reinterpret_cast<uint32_t*>(out + pk) = (w & ((1u << (8 * rem)) - 1u)) | (nh << (8 * rem));
      } else {  // the plane's last chunk (the next plane's header follows), or the end of `cap`
        for (uint32_t i = 0; i < rem; i++) out[pk + i] = (uint8_t)(w >> (8 * i));
      }
    }
    return;
  }
  // ---- longer chunks (overflow slots, up to 160 bytes): chunk bytes k ..
  // k+3 from source byte sh + k, 9 source words at a time
  auto word_at = [&](uint32_t k, const uint32_t* w, uint32_t j0) -> uint32_t {
    const uint32_t r = sh + k, i = (r >> 2) - j0, q = r & 3u;
    return q ? (w[i] >> (8 * q)) | (w[i + 1] << (32 - 8 * q)) : w[i];
  };
  uint32_t r[9];  // source words j0 .. j0 + 8
#pragma unroll
  for (uint32_t i = 0; i < 9; i++) r[i] = v[i];
  uint32_t j0 = 0;
  uint32_t k = lead;
  // 16 chunk bytes per store while 16 remain (the wave's loop runs to its
  // longest chunk: a quarter of the iterations of dword stores)
  for (; k + 16u <= sz; k += 16u) {
    const uint32_t need = (sh + k) >> 2;
    if (need + 4 >= j0 + 9) {  // refill
      j0 = need;
#pragma unroll
      for (uint32_t i = 0; i < 9; i++) r[i] = (j0 + i < nsrc) ? gsrc[j0 + i] : 0u;
    }
    const Dw4 o{word_at(k, r, j0), word_at(k + 4, r, j0), word_at(k + 8, r, j0), word_at(k + 12, r, j0)};
    *reinterpret_cast<Dw4*>(out + P + k) = o;  // (4-byte aligned: P + lead is)
  }
  for (; k < sz; k += 4) {
    const uint32_t need = (sh + k) >> 2;
    if (need + 1 >= j0 + 9) {  // refill (chunks over ~28 bytes)
      j0 = need;
#pragma unroll
      for (uint32_t i = 0; i < 9; i++) r[i] = (j0 + i < nsrc) ? gsrc[j0 + i] : 0u;
    }
    uint32_t w = word_at(k, r, j0);
    const uint32_t rem = sz - k;
    if (rem >= 4) {
      *reinterpret_cast<uint32_t*>(out + P + k) = w;
    } else if (has_next && P + k + 4 <= cap) {  // complete the dword with the next chunk's first bytes
      w = (w & ((1u << (8 * rem)) - 1u)) | (nh << (8 * rem));
      *reinterpret_cast<uint32_t*>(out + P + k) = w;
    } else {  // the plane's last chunk (the next plane's header follows), or the end of `cap`
      for (uint32_t i = 0; i < rem; i++) out[P + k + i] = (uint8_t)(w >> (8 * i));
    }
  }
}

}  // namespace myyuv_gpu
