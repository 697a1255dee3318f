// myyuv_hip.cpp — implementation of the C ABI in include/myyuv_hip.h.
//
// Host side of the gfx950 codec: frame geometry, quantisation tables, the
// per-context workspace, and the launch sequences
//   compress:   K1 fdct_quant -> K2 huff_encode (+ overflow pass) -> K4 stream_out
//   decompress: parse -> scan -> K5 huff_decode -> K6 dequant_idct
// Every launch goes to one stream; nothing synchronises inside the
// device-resident entry points, so frames pipeline back to back.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "codec_common.hpp"
#include "fdct_bfly.h"
#include "k_chain.hpp"
#include "k_stream.hpp"
#include "myyuv_hip.h"

#ifndef MYYUV_R16_BATCH
#define MYYUV_R16_BATCH 1  // batches take the CAP-16 overflow tier too (0: single frames only)
#endif

namespace myyuv_gpu {
__global__ void k_fdct_quant(const uint8_t*, FrameGeom, const QTables*, uint4*, uint8_t*, uint32_t*, uint4*,
                             uint32_t*, uint32_t*, uint32_t);
__global__ void k_fdct_fix(const uint8_t*, FrameGeom, const QTables*, uint4*, uint8_t*, uint32_t*, uint4*,
                           uint32_t*, uint32_t);
__global__ void k_dequant_idct(const uint4*, const uint8_t*, const uint4*, FrameGeom, const QTables*, uint8_t*,
                               uint4*);
__global__ void k_decode_idct(const uint8_t*, const uint32_t*, uint32_t, const StreamDesc*, const uint32_t*,
                              const uint32_t*, FrameGeom, uint32_t, uint32_t, const QTables*, uint4*, uint8_t*,
                              unsigned long long*);
template <uint32_t W>
__global__ void k_huff_encode(const uint4*, const uint32_t*, const uint4*, FrameGeom, uint32_t*, uint32_t*,
                              uint8_t*, uint32_t*, uint32_t*, uint32_t*);
__global__ void k_huff_encode_wave(const uint4*, const uint8_t*, FrameGeom, uint32_t*, uint8_t*, uint32_t*,
                                   const uint32_t*, const uint32_t*, const uint32_t*, const uint32_t*, uint32_t,
                                   uint32_t);
__global__ void k_huff_encode_wide(const uint4*, const uint8_t*, const uint4*, FrameGeom, uint32_t*, uint8_t*,
                                   uint32_t*, const uint32_t*, const uint32_t*, const uint32_t*, const uint32_t*,
                                   uint32_t, uint32_t);
__global__ void k_huff_encode_r16(const uint4*, const uint8_t*, const uint4*, FrameGeom, uint32_t*, uint8_t*,
                                  uint32_t*, const uint32_t*, const uint32_t*, uint32_t*, uint32_t*, uint32_t);
__global__ void k_encode_tile(const uint8_t*, FrameGeom, const QTables*, uint4*, uint8_t*, uint32_t*, uint32_t*,
                              uint8_t*, uint32_t*, uint32_t*, uint32_t*);
__global__ void k_tile_scan(uint32_t*, FrameGeom, uint8_t*, uint32_t, uint32_t*, unsigned long long*);
__global__ void k_scan_chain(const uint8_t*, uint32_t, ScanSrc, const uint32_t*, uint32_t, FrameGeom,
                             StreamDesc*, uint32_t*, uint32_t*, uint32_t, unsigned long long*,
                             uint32_t, unsigned long long*);
__global__ void k_stream_out(const uint32_t*, const uint32_t*, const uint8_t*, const uint32_t*,
                             const uint32_t*, FrameGeom, uint8_t*, uint32_t, uint32_t);
__global__ void k_huff_decode(const uint8_t*, const uint32_t*, uint32_t, const StreamDesc*,
                              const uint32_t*, const uint32_t*, FrameGeom, uint32_t, uint32_t,
                              uint4*, uint8_t*, unsigned long long*);
template <int BPP>
__global__ void k_bmp_to_iyuv(const uint8_t*, uint32_t, uint32_t, uint32_t, uint8_t*);
#ifdef MYYUV_STAMPS
extern __device__ unsigned long long g_k2_stamps[40];
extern __device__ uint32_t g_k2_wstamps[65536 * 8];
extern __device__ uint32_t g_k2_fstamps[8192 * 8];
extern __device__ uint32_t g_dec_wstamps[65536 * 8];
extern __device__ uint32_t g_k2_win[65536 * 8];
#endif
}  // namespace myyuv_gpu

using namespace myyuv_gpu;

namespace {

constexpr float kLumQ[64] = {16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
                             14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
                             18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
                             49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
constexpr float kChromaQ[64] = {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
                                24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
                                99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
                                99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};

// DCT.cpp:286-290: Q = clamp(roundf(base * mul), 1, 255), mul in float.
void make_qtable(int q, bool chroma, float out[64]) {
  const float* base = chroma ? kChromaQ : kLumQ;
  const float fq = (float)q;
  const float mul = (fq >= 50.5f) ? (100.0f - fq) / 50.0f : 50.0f / fq;
  for (int i = 0; i < 64; i++) out[i] = std::min(std::max(std::roundf(base[i] * mul), 1.0f), 255.0f);
}

// Reciprocals and K1's fast-path row bounds from the Q tables.
void finish_qtables(QTables& t, int planes) {
  for (int p = 0; p < planes; p++) {
    for (int n = 0; n < 64; n++) t.r[p][n] = 1.0f / t.q[p][n];
    myyuv_bfly::bfly_row_bounds(t.r[p], t.kb[p]);
  }
}

struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
  int grow(size_t want) {
    if (want <= n) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    if (hipMalloc(&p, want) != hipSuccess) return MYYUV_E_HIP;
    n = want;
    return 0;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

constexpr uint8_t kZigzag[64] = MYYUV_ZIGZAG;

uint32_t ceil_div(uint32_t a, uint32_t b) { return (a + b - 1) / b; }

// K1/K6 grid: persistent waves (four per 256-thread workgroup) striding over
// the frame's 16-block units: as many workgroups as are resident at once
// (`resident`, from the occupancy query at context creation), never more
// waves than units.
dim3 xf_grid(const FrameGeom& G, uint32_t resident) {
  const uint32_t wgs = ceil_div(G.ucum[3] * G.nframes, 4);
  return dim3(wgs < resident ? wgs : resident);
}

// ceil(2^64 / bw) for FrameGeom::bmag; 0 marks bw = 1 (block_row returns local).
uint64_t block_magic(uint32_t bw) { return bw > 1 ? ~0ull / bw + 1 : 0; }

// Dimension checks in the reference's order: per plane, width then height
// (applyDCTPlane / restoreDCTPlane, DCT.cpp:280-285, :338-343).
int make_geom(uint32_t w, uint32_t h, FrameGeom& G) {
  if (w == 0 || h == 0) return MYYUV_E_WIDTH;
  if ((uint64_t)w * h * 3 / 2 > 0xFFFFFFFFull) return MYYUV_E_ARG;
  const uint32_t pw[3] = {w, w / 2, w / 2}, ph[3] = {h, h / 2, h / 2};
  for (int p = 0; p < 3; p++) {
    if (pw[p] % 8) return MYYUV_E_WIDTH;
    if (ph[p] % 8) return MYYUV_E_HEIGHT;
  }
  std::memset(&G, 0, sizeof(G));
  G.cum[0] = 0;
  for (int p = 0; p < 3; p++) {
    G.pw[p] = pw[p];
    G.ph[p] = ph[p];
    G.bw[p] = pw[p] / 8;
    G.cum[p + 1] = G.cum[p] + G.bw[p] * (ph[p] / 8);
    G.bmag[p] = block_magic(G.bw[p]);
    G.ucum[p + 1] = G.ucum[p] + ceil_div(G.cum[p + 1] - G.cum[p], kXfUnit);
    G.tcum[p + 1] = G.tcum[p] + ceil_div(G.cum[p + 1] - G.cum[p], kK2Group);
  }
  G.poff[0] = 0;
  G.poff[1] = w * h;
  G.poff[2] = w * h + (w / 2) * (h / 2);
  G.nframes = 1;
  G.fbytes = w * h / 2 * 3;
  G.umag = block_magic(G.ucum[3]);
  G.fbase = 0;
  // one frame's coefficient image within the kernels' 32-bit offsets (> 1.4 G
  // pixels; the reference's getImageSize overflows from 537 M pixels)
  if (G.cum[3] > kMaxLaunchBlocks) return MYYUV_E_ARG;
  return 0;
}

// Frames per launch of geometry G (kMaxLaunchBlocks, or a smaller
// diagnostic cap: MYYUV_LAUNCH_BLOCKS, read at context creation).
uint32_t launch_frames(const FrameGeom& G, uint32_t cap_blocks = kMaxLaunchBlocks) {
  return std::max(1u, std::min(cap_blocks, kMaxLaunchBlocks) / G.cum[3]);
}

// A batch of nf frames of G's geometry (block, unit and byte counts of the
// whole batch must fit 32 bits).
int set_batch(FrameGeom& G, uint32_t nf) {
  if (nf == 0) return MYYUV_E_ARG;
  if ((uint64_t)G.cum[3] * nf > 0xFFFFFFFFull - 4096 || (uint64_t)G.fbytes * nf > 0xFFFFFFFFull)
    return MYYUV_E_ARG;
  G.nframes = nf;
  return 0;
}

}  // namespace

struct myyuv_hip_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  // One context's scratch buffers (coef, slots, sizes, scan status words ...)
  // serve one call at a time: every entry point records `done` on its stream
  // and a call on another stream first waits for it (StreamOrder), so calls
  // on different streams through one context run in call order.
  hipEvent_t done = nullptr;
  hipStream_t last_stream = nullptr;
  DevBuf frame, coef, sizes, loff, tiles, payload, err, psize, desc, work, qtd;
  DevBuf stage, oslots, tinfo, srcoff;  // K2 -> K4 (codec_common.hpp)
  DevBuf bmp;   // staged BMP pixels (host-buffer BMP -> IYUV)
  DevBuf bsizes;  // u32 payload sizes of a host-buffer batch
  DevBuf rmask; // per block: bit c = coefficient row c nonzero (K1 -> overflow passes, K5 -> K6)
  DevBuf binfo; // per block: K1 -> K2's classification (binfo_word, codec_common.hpp)
  DevBuf zq;    // 256 zero bytes: K6's source for rows the mask says are zero
  DevBuf sink;  // K1/K6 stores of lanes past a plane's end (128 x 16 B, never read)
  // K1 -> k_fdct_fix: the unproven units' lists and counts (fix_count /
  // fix_list, codec_common.hpp; fix_par alternates from launch to launch)
  DevBuf fix;
  uint32_t fix_par = 0;
  uint32_t xf_resident[2] = {kXfWaves / 4, kXfWaves / 4};  // K1, K6 workgroups resident on the device
  uint32_t fix_resident = kXfWaves / 4;                      // k_fdct_fix workgroups resident
  // k_fdct_fix's grid at qualities up to fix_qmax (MYYUV_FIX_GRID; 0, the
  // default: the resident count, as above fix_qmax).  A small fixed grid
  // measured no faster (profiles/r4h_fix_ab.txt), and busy content at low q
  // can list far more units than the bench frame's 0.07 %.
  uint32_t fix_grid = 0;
  uint32_t fix_qmax = 75;  // (MYYUV_FIX_QMAX)
  uint32_t launch_blocks = kMaxLaunchBlocks;  // blocks per launch (MYYUV_LAUNCH_BLOCKS: a test of the batch split)
  // encoder: K1 -> K2 through HBM (split), or the fused single-pass kernel
  // k_encode_tile (MYYUV_ENCODER=fused|split)
  bool fused = false;
  // decoder: the fused k_decode_idct (default), or K5 -> K6 through HBM
  // (MYYUV_DECODER=split)
  bool fused_dec = true;
  // chained scan (k_chain.hpp): per-tile status words tagged with the launch
  // epoch, counted here
  DevBuf status;
  uint32_t epoch = 0;
  // quantisation tables of the last quality triple (host copy; qtd on the
  // device, rewritten in stream order when the triple changes)
  QTables qt;
  hipStream_t qt_stream = nullptr;
  uint8_t q_cached[3] = {0, 0, 0};
  bool q_valid = false;
  // profiling
  uint32_t prof = 0;  // bit k: stamp kernel id k
  uint32_t skip = 0;  // diagnostic: bit k: do not launch kernel id k (myyuv_debug_skip_kernels)
  double ms[MYYUV_K_COUNT] = {};
  int64_t launches[MYYUV_K_COUNT] = {};
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> pending;
  std::vector<hipEvent_t> free_events;
  // host-buffer batch pipeline (HostPipe below): H2D on cin, kernels on
  // `stream`, D2H on cout; two slots of up to kPipeMaxChunk frames
  hipStream_t cin = nullptr, cout = nullptr;
  hipEvent_t pev[3][2] = {};  // [copied in, computed, copied out][slot]
  DevBuf pin[2], pout[2], psz[2], perr[2];
  uint32_t* hsz = nullptr;            // pinned: 2 x kPipeMaxChunk u32 sizes
  unsigned long long* herr = nullptr;  // pinned: 2 error words
  std::mutex mu;
};

namespace {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// Orders a call on stream `s` after the context's previous call (see
// myyuv_hip_ctx::done); the record at scope exit publishes this call's work.
struct StreamOrder {
  myyuv_hip_ctx* c;
  hipStream_t s;
  StreamOrder(myyuv_hip_ctx* ctx, hipStream_t st) : c(ctx), s(st) {
    if (c->last_stream && c->last_stream != s) (void)hipStreamWaitEvent(s, c->done, 0);
  }
  ~StreamOrder() {
    if (hipEventRecord(c->done, s) == hipSuccess) c->last_stream = s;
  }
};

hipEvent_t take_event(myyuv_hip_ctx* c) {
  if (!c->free_events.empty()) {
    hipEvent_t e = c->free_events.back();
    c->free_events.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

// Launches kernel `k` on `s`.  When profiling, the start/stop events are the
// ones hipExtLaunchKernel stamps from the kernel's own dispatch packet: the
// kernel's execution time (what rocprofv3's kernel trace reports), without
// the few microseconds of queue latency a hipEventRecord bracket adds.
template <class... KArgs, class... Args>
int launch(myyuv_hip_ctx* c, int kid, void (*k)(KArgs...), dim3 grid, dim3 block, hipStream_t s,
           Args... args) {
  if ((c->skip >> kid) & 1u) return 0;
  hipEvent_t a = nullptr, b = nullptr;
  const bool stamp = (c->prof >> kid) & 1u;
  if (stamp) {
    a = take_event(c);
    b = take_event(c);
  }
  hipExtLaunchKernelGGL(k, grid, block, 0, s, a, b, 0, static_cast<KArgs>(args)...);
  if (hipPeekAtLastError() != hipSuccess) {
    (void)hipGetLastError();
    return MYYUV_E_HIP;
  }
  if (stamp) c->pending.push_back({kid, {a, b}});
  return 0;
}

void drain_profile(myyuv_hip_ctx* c) {
  for (auto& it : c->pending) {
    float ms = 0;
    (void)hipEventSynchronize(it.second.second);
    if (hipEventElapsedTime(&ms, it.second.first, it.second.second) == hipSuccess) {
      c->ms[it.first] += ms;
      c->launches[it.first] += 1;
    }
    c->free_events.push_back(it.second.first);
    c->free_events.push_back(it.second.second);
  }
  c->pending.clear();
}

int set_qtables(myyuv_hip_ctx* c, const uint8_t q[3], hipStream_t s) {
  for (int p = 0; p < 3; p++)
    if (q[p] < 1 || q[p] > 100) return MYYUV_E_QUALITY;
  if (c->q_valid && std::memcmp(c->q_cached, q, 3) == 0 && c->qt_stream == s) return 0;
  for (int p = 0; p < 3; p++) {
    make_qtable(q[p], p != 0, c->qt.q[p]);
  }
  finish_qtables(c->qt, 3);
  if (c->qtd.grow(sizeof(QTables))) return MYYUV_E_HIP;
  // kernels queued on another stream may still read the old tables
  if (c->qt_stream && c->qt_stream != s && hipStreamSynchronize(c->qt_stream) != hipSuccess)
    return MYYUV_E_HIP;
  // pageable source: the copy is staged before the call returns
  if (hipMemcpyAsync(c->qtd.p, &c->qt, sizeof(QTables), hipMemcpyHostToDevice, s) != hipSuccess)
    return MYYUV_E_HIP;
  c->qt_stream = s;
  std::memcpy(c->q_cached, q, 3);
  c->q_valid = true;
  return 0;
}

// Workspace for a batch of G.nframes frames (blocks numbered batch-globally;
// scan tiles, stream descriptors and look-back status words per frame).
int reserve(myyuv_hip_ctx* c, const FrameGeom& G) {
  const uint32_t nf = G.nframes;
  const uint32_t nblk = G.cum[3] * nf;
  const uint32_t nwaves = ceil_div(nblk, kWave);
  const uint32_t ntiles = ceil_div(G.cum[3], kScanTile);
  int e = 0;
  e |= c->coef.grow((size_t)nwaves * kCoefQuadsPerWave * 16);  // natural-order quads
  e |= c->stage.grow((size_t)win_tiles_alloc(nf * G.tcum[3]) * kTileCap);
  e |= c->oslots.grow((size_t)nblk * kMaxChunk);
  // (plus a guard band of one big window's tiles past the launch's last tile:
  // myyuv_debug_tinfo_guard checks that no kernel writes into it)
  e |= c->tinfo.grow((size_t)(nf * G.tcum[3] + kWinTilesBig) * kTInfoWords * 4);
  e |= c->srcoff.grow((size_t)nblk * 4);
  e |= c->sizes.grow((size_t)nwaves * kWave);
  e |= c->rmask.grow((size_t)nblk);
  e |= c->binfo.grow((size_t)nblk * 4);
  if (c->zq.n == 0) {
    e |= c->zq.grow(256);
    if (!e && hipMemset(c->zq.p, 0, 256) != hipSuccess) e |= MYYUV_E_HIP;
  }
  e |= c->loff.grow((size_t)nblk * 4);
  e |= c->tiles.grow((size_t)nf * (ntiles + 1) * 4);
  e |= c->err.grow(8);
  e |= c->sink.grow((size_t)kSinkQuads * 16 * kSinkSlots);  // K1/K6: 2 x 64 quads + K1's 64 mask bytes + 64 words
  e |= c->psize.grow(4);
  e |= c->desc.grow((size_t)nf * sizeof(StreamDesc));
  // [0], [1]: overflow counts, then K2's list and (single frames) the CAP-16 tier's (launch_overflow)
  e |= c->work.grow((size_t)nblk * (nf == 1 || MYYUV_R16_BATCH ? 8 : 4) + 256);
  {
    const size_t fb = fix_words(G.ucum[3] * nf) * 4;
    if (c->fix.n < fb) {
      e |= c->fix.grow(fb);
      if (!e && (hipMemset(c->fix.p, 0, kFixHeader * 4) != hipSuccess || hipDeviceSynchronize() != hipSuccess))
        e |= MYYUV_E_HIP;
    }
  }
  const size_t st_bytes = (size_t)nf * (ntiles + 1) * 8;
  if (c->status.n < st_bytes) {
    e |= c->status.grow(st_bytes);
    // zeroed before any kernel on any stream reads it
    if (!e && (hipMemset(c->status.p, 0, st_bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess))
      e |= MYYUV_E_HIP;
  }
  return e ? MYYUV_E_HIP : 0;
}

uint32_t next_epoch(myyuv_hip_ctx* c) {
  c->epoch = (c->epoch + 1) & kEpochMask;
  if (c->epoch == 0) c->epoch = 1;  // status words start zeroed: epoch 0 is never current
  return c->epoch;
}

// K2: fast pass over all tiles (grid (tiles, frames)), then the overflow pass
// over the blocks with more than 8 distinct symbols (worklist filled on the
// device; no host sync): wave-per-block for lists of at most kWaveEncodeLimit
// blocks, lane-per-block for longer ones; both kernels are queued and each
// returns at once outside its regime.  A batch (nf > 1) takes the
// lane-per-block pass only: its list is long, and the wave pass's per-block
// SALU cost would crowd the other launch groups in flight (tools/kskip.py).
// A list longer than one resident round of the lane pass (kR16Gate; a
// single frame's: two rounds of the wave pass, kR16GateSingle) goes
// through the CAP-16 register tier first (k_huff_encode_r16), and the two
// passes then take what it leaves (more than 16 symbols: work[1] blocks from
// word 64 + nblk).  work[0] is zeroed by K1 (or the host), work[1] here.
int launch_overflow(myyuv_hip_ctx* c, const FrameGeom& G, hipStream_t s);

int launch_huff_encode(myyuv_hip_ctx* c, const FrameGeom& G, hipStream_t s) {
  const uint32_t nf = G.nframes;
  uint32_t* count = c->work.as<uint32_t>();
  uint32_t* list = count + 64;
  // (*count was zeroed by K1, just before in the stream: k_fdct_quant's k2ctl)
  // (the window size of the launch, k2_win: K4 uses the same)
  const uint32_t W = k2_win(nf * G.tcum[3]);
  const int e = launch(c, MYYUV_K_HUFF_ENC, W == kWinTilesBig ? k_huff_encode<kWinTilesBig> : k_huff_encode<kWinTiles>,
                       dim3(ceil_div(nf * G.tcum[3], W)), dim3(kK2Group), s,
               c->coef.as<const uint4>(), c->binfo.as<const uint32_t>(), c->zq.as<const uint4>(), G,
               c->stage.as<uint32_t>(), c->tinfo.as<uint32_t>(), c->sizes.as<uint8_t>(),
               c->srcoff.as<uint32_t>(), list, count);
  return e | launch_overflow(c, G, s);
}

int launch_overflow(myyuv_hip_ctx* c, const FrameGeom& G, hipStream_t s) {
  const uint32_t nf = G.nframes, nblk = G.cum[3] * nf;
  uint32_t* count = c->work.as<uint32_t>();
  uint32_t* list = count + 64;
  uint32_t* count2 = count + 1;
  uint32_t* list2 = list + nblk;
  const uint32_t limit = nf > 1 ? kBatchWaveLimit : kWaveEncodeLimit;
  int e = 0;
  const uint32_t g16 = nf == 1 ? kR16GateSingle : kR16Gate;
  const uint32_t gate = (nf == 1 || MYYUV_R16_BATCH) && nblk > g16 ? g16 : ~0u;
  // (launched whenever such a list is possible; with 8-frame launch groups,
  // whose lists stay below the gate, the empty launch cost 3.4 % of the
  // bench, profiles/r3zw_*; the bench's 24-frame groups take the tier)
  if (gate != ~0u) {
    // work[1], the tier's count (its own node: a store in K1's prologue
    // shifted K1's loop and cost it 5 %, profiles/r3zx_*)
    e |= hipMemsetAsync(count2, 0, 4, s) != hipSuccess;
    const uint32_t r16 = ceil_div(nblk, kWave) < kR16Grid ? ceil_div(nblk, kWave) : kR16Grid;
    e |= launch(c, MYYUV_K_HUFF_R16, k_huff_encode_r16, dim3(r16), dim3(kWave), s, c->coef.as<const uint4>(),
                c->rmask.as<const uint8_t>(), c->zq.as<const uint4>(), G, c->oslots.as<uint32_t>(),
                c->sizes.as<uint8_t>(), c->tinfo.as<uint32_t>(), (const uint32_t*)list, (const uint32_t*)count,
                list2, count2, gate);
  }
  if (limit > 0)
    e |= launch(c, MYYUV_K_HUFF_WAVE, k_huff_encode_wave, dim3(kWaveEncodeGrid), dim3(kWave), s,
                c->coef.as<const uint4>(), c->rmask.as<const uint8_t>(), G, c->oslots.as<uint32_t>(),
                c->sizes.as<uint8_t>(), c->tinfo.as<uint32_t>(), (const uint32_t*)list, (const uint32_t*)count,
                (const uint32_t*)list2, (const uint32_t*)count2, gate, limit);
  const uint32_t wide = ceil_div(nblk, kWideLanes) < kWideGrid ? ceil_div(nblk, kWideLanes) : kWideGrid;
  e |= launch(c, MYYUV_K_HUFF_WIDE, k_huff_encode_wide, dim3(wide), dim3(kWideLanes), s,
              c->coef.as<const uint4>(), c->rmask.as<const uint8_t>(), c->zq.as<const uint4>(), G,
              c->oslots.as<uint32_t>(), c->sizes.as<uint8_t>(), c->tinfo.as<uint32_t>(), (const uint32_t*)list,
              (const uint32_t*)count, (const uint32_t*)list2, (const uint32_t*)count2, gate, limit);
  return e;
}

// K1, then its exact path for the units it listed (k_fdct_fix).  The list
// is on the device, so the fix grid cannot follow its length: the resident
// count (the fast path fails for 0.07 % of the bench frame's units at q50,
// 18 % at q90, 48 % at q100, more on noise: tools/diag/fast_dct_sim.py);
// workgroups past the list return at once.  MYYUV_FIX_GRID=n caps it at n
// workgroups for qualities up to MYYUV_FIX_QMAX (a test of the grid-stride
// walk).  k2ctl: K2's overflow count, zeroed by K1
// (nullptr: none).
int launch_fdct(myyuv_hip_ctx* c, const FrameGeom& G, const uint8_t* in, const QTables* qt, uint32_t* k2ctl,
                hipStream_t s) {
  const uint32_t par = c->fix_par;
  c->fix_par ^= 1u;
  int e = launch(c, MYYUV_K_FDCT, k_fdct_quant, xf_grid(G, c->xf_resident[0]), dim3(256), s, in, G, qt,
                 c->coef.as<uint4>(), c->rmask.as<uint8_t>(), c->binfo.as<uint32_t>(), c->sink.as<uint4>(), k2ctl,
                 c->fix.as<uint32_t>(), par);
  uint32_t qmax = 0;
  for (int p = 0; p < 3; p++) qmax = std::max(qmax, (uint32_t)c->q_cached[p]);
  const uint32_t want =
      (c->fix_grid == 0 || !c->q_valid || qmax > c->fix_qmax) ? c->fix_resident : c->fix_grid;
  // (a multiple of kFixLists waves: wave w takes list w % kFixLists)
  const uint32_t per = kFixLists / kFixWaves;
  const uint32_t grid = std::max(per, (want * 4 / kFixWaves) / per * per);
  e |= launch(c, MYYUV_K_FDCT_FIX, k_fdct_fix, dim3(grid), dim3(64 * kFixWaves), s, in, G, qt, c->coef.as<uint4>(),
              c->rmask.as<uint8_t>(), c->binfo.as<uint32_t>(), c->sink.as<uint4>(), c->fix.as<uint32_t>(), par);
  // the fix kernel zeroes the next launch's counts; without it (a diagnostic
  // skip, or a failed launch) the host does
  if (e || ((c->skip >> MYYUV_K_FDCT_FIX) & 1u))
    e |= hipMemsetAsync(fix_count(c->fix.as<uint32_t>(), par ^ 1u, 0), 0, kFixLists * 32 * 4, s) != hipSuccess;
  return e;
}

// One batch of G.nframes frames (frame f at d_in + f * fbytes), payload f at
// d_out + f * cap, its size at d_size[f].
int launch_compress(myyuv_hip_ctx* c, const FrameGeom& G, const void* d_in, void* d_out,
                    uint32_t cap, uint32_t* d_size, hipStream_t s, unsigned long long* err = nullptr) {
  const uint32_t nf = G.nframes;
  const QTables* qt = c->qtd.as<const QTables>();
  if (!err) err = c->err.as<unsigned long long>();
  int e = 0;
  if (c->fused) {
    // fused single-pass encoder (K1 + K2 per tile), then the overflow passes
    uint32_t* count = c->work.as<uint32_t>();
    e |= hipMemsetAsync(count, 0, 4, s) != hipSuccess;
    e |= launch(c, MYYUV_K_ENCODE_TILE, k_encode_tile, dim3(G.tcum[3], nf), dim3(kK2Group), s,
                static_cast<const uint8_t*>(d_in), G, qt, c->coef.as<uint4>(), c->rmask.as<uint8_t>(),
                c->stage.as<uint32_t>(), c->tinfo.as<uint32_t>(), c->sizes.as<uint8_t>(), c->srcoff.as<uint32_t>(),
                count + 64, count);
    e |= launch_overflow(c, G, s);
  } else {
    e |= launch_fdct(c, G, static_cast<const uint8_t*>(d_in), qt, c->work.as<uint32_t>(), s);
    if ((c->skip >> MYYUV_K_FDCT) & 1u)  // diagnostic skip: keep K1's reset of the overflow count
      e |= hipMemsetAsync(c->work.p, 0, 4, s) != hipSuccess;
    e |= launch_huff_encode(c, G, s);
  }
  e |= launch(c, MYYUV_K_SCAN, k_tile_scan, dim3(nf), dim3(256), s, c->tinfo.as<uint32_t>(), G,
              static_cast<uint8_t*>(d_out), cap, d_size, err);
  // K4 reads the stage in K2's windows (k2_win; the fused encoder's: kWinTiles)
  const uint32_t W = c->fused ? kWinTiles : k2_win(nf * G.tcum[3]);
  e |= launch(c, MYYUV_K_COMPACT, k_stream_out, dim3(ceil_div(G.tcum[3] * nf, 8 * W) * 8 * W), dim3(256), s,
              c->stage.as<const uint32_t>(), c->tinfo.as<const uint32_t>(), c->sizes.as<const uint8_t>(),
              c->srcoff.as<const uint32_t>(), c->oslots.as<const uint32_t>(), G, static_cast<uint8_t*>(d_out),
              cap, W);
  return e ? MYYUV_E_HIP : 0;
}

// The mirror: payload f at d_in + f * cap (size d_size[f]) -> frame f at
// d_out + f * fbytes.
int launch_decompress(myyuv_hip_ctx* c, const FrameGeom& G, const void* d_in,
                      const uint32_t* d_size, uint32_t cap, void* d_out, hipStream_t s,
                      unsigned long long* err = nullptr) {
  const uint32_t nf = G.nframes;
  const uint32_t nblk = G.cum[3];
  const uint32_t ntiles = ceil_div(nblk, kScanTile);
  const QTables* qt = c->qtd.as<const QTables>();
  if (!err) err = c->err.as<unsigned long long>();
  StreamDesc* desc = c->desc.as<StreamDesc>();
  const uint8_t* in = static_cast<const uint8_t*>(d_in);
  int e = 0;
  ScanSrc S;
  for (int i = 0; i < 4; i++) S.cum[i] = G.cum[i];
  for (int p = 0; p < 3; p++) S.pos[p] = 0;
  e |= launch(c, MYYUV_K_SCAN, k_scan_chain, dim3(ntiles, nf), dim3(256), s, in, cap, S, d_size, cap,
              G, desc, c->loff.as<uint32_t>(), c->tiles.as<uint32_t>(), ntiles,
              c->status.as<unsigned long long>(), next_epoch(c), err);
  const uint32_t t0 = ceil_div(G.cum[1] - G.cum[0], kWave),
                 t1 = ceil_div(G.cum[2] - G.cum[1], kWave),
                 t2 = ceil_div(G.cum[3] - G.cum[2], kWave);
  if (c->fused_dec) {  // K5 + K6 in one pass, the coefficients kept on chip
    e |= launch(c, MYYUV_K_HUFF_DEC, k_decode_idct, dim3(t0 + t1 + t2, nf), dim3(kWave), s, in, d_size, cap,
                (const StreamDesc*)desc, c->loff.as<const uint32_t>(), c->tiles.as<const uint32_t>(), G, t0, t1,
                qt, c->coef.as<uint4>(), static_cast<uint8_t*>(d_out), err);
    return e ? MYYUV_E_HIP : 0;
  }
  e |= launch(c, MYYUV_K_HUFF_DEC, k_huff_decode, dim3(t0 + t1 + t2, nf), dim3(kWave), s, in, d_size,
              cap, (const StreamDesc*)desc, c->loff.as<const uint32_t>(),
              c->tiles.as<const uint32_t>(), G, t0, t1, c->coef.as<uint4>(), c->rmask.as<uint8_t>(), err);
  e |= launch(c, MYYUV_K_IDCT, k_dequant_idct, xf_grid(G, c->xf_resident[1]), dim3(256), s,
              c->coef.as<const uint4>(), c->rmask.as<const uint8_t>(), c->zq.as<const uint4>(), G, qt,
              static_cast<uint8_t*>(d_out), c->sink.as<uint4>());
  return e ? MYYUV_E_HIP : 0;
}

// Host <-> device copies of the host-buffer entry points: direct async copies
// from / into the caller's pageable buffers.  On this stack they run at the
// PCIe link rate whatever the buffer's alignment or age (tools/ubench/
// pcie_copy.cpp, profiles/r3b_pcie_copy.txt: 18 MB in 0.33-0.43 ms, a fresh
// or 1-byte-misaligned buffer included), faster than staging through pinned
// chunks with a CPU copy (0.47-0.59 ms H2D, 1.1-2.7 ms D2H).
int h2d(myyuv_hip_ctx*, void* dst, const void* src, size_t n, hipStream_t s) {
  return hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, s) == hipSuccess ? 0 : MYYUV_E_HIP;
}

// (synchronous: returns when dst holds the bytes)
int d2h(myyuv_hip_ctx*, void* dst, const void* src, size_t n, hipStream_t s) {
  return hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, s) == hipSuccess && hipStreamSynchronize(s) == hipSuccess
             ? 0
             : MYYUV_E_HIP;
}

int reset_err(myyuv_hip_ctx* c, hipStream_t s) {
  return hipMemsetAsync(c->err.p, 0xFF, 8, s) == hipSuccess ? 0 : MYYUV_E_HIP;
}

int read_err(myyuv_hip_ctx* c, hipStream_t s, int64_t* bad_block) {
  unsigned long long v = ~0ull;
  if (hipMemcpyAsync(&v, c->err.p, 8, hipMemcpyDeviceToHost, s) != hipSuccess) return MYYUV_E_HIP;
  if (hipStreamSynchronize(s) != hipSuccess) return MYYUV_E_HIP;
  if (bad_block) *bad_block = -1;
  if (v == ~0ull) return 0;
  const int code = (int)(v & 0xFF);
  const uint64_t key = v >> 8;
  if (bad_block) *bad_block = key == 0 ? -1 : (int64_t)(key >> 1);
  return code;
}

// Host mirror of the stream header checks (parse_stream, k_chain.hpp; same order), for host buffers.
int host_parse_headers(const uint8_t* in, uint32_t size) {
  auto rd32 = [&](uint64_t a) {
    uint32_t v;
    std::memcpy(&v, in + a, 4);
    return v;
  };
  if (size <= 12) return MYYUV_E_DCTYUV_SIZE;
  const uint32_t ps[3] = {rd32(0), rd32(4), rd32(8)};
  if (12ull + ps[0] + ps[1] + ps[2] > size) return MYYUV_E_DCTYUV_SIZE;
  uint64_t off = 12;
  for (int p = 0; p < 3; p++) {
    if (ps[p] <= 8) return MYYUV_E_PLANE_SIZE;
    const uint32_t hn = rd32(off), hc = rd32(off + 4);
    if (hn == 0) return MYYUV_E_PLANE_NBLK;
    if (hc == 0) return MYYUV_E_PLANE_CONTENT;
    if (8ull + hn + hc > ps[p]) return MYYUV_E_PLANE_SIZE;
    off += ps[p];
  }
  return 0;
}

bool hip_ok() {
  static int ok = -1;
  if (ok < 0) {
    int n = 0;
    ok = (hipGetDeviceCount(&n) == hipSuccess && n > 0) ? 1 : 0;
  }
  return ok == 1;
}

}  // namespace

extern "C" {

const char* myyuv_hip_strerror(int code) {
  switch (code) {
    case MYYUV_OK: return "Success";
    case MYYUV_E_ARG: return "Invalid argument";
    case MYYUV_E_QUALITY: return "Level of quality must be between 1 and 100";
    case MYYUV_E_WIDTH: return "Error. width % 8 must be 0";
    case MYYUV_E_HEIGHT: return "Error. height % 8 must be 0";
    case MYYUV_E_CAPACITY: return "Output buffer too small for the compressed stream";
    case MYYUV_E_DCTYUV_SIZE: return "DCTYUV load bad size";
    case MYYUV_E_PLANE_SIZE: return "DCTYUVPlane load bad size";
    case MYYUV_E_PLANE_NBLK: return "DCTYUVPlane load chunks_sizes_size bad size";
    case MYYUV_E_PLANE_CONTENT: return "DCTYUVPlane load content_size bad size";
    case MYYUV_E_BAD_CODE: return "Huffman bad code";
    case MYYUV_E_UNKNOWN_SYMBOL: return "Huffman unknown symbol";
    case MYYUV_E_BAD_CHUNK: return "Huffman bad chunk";
    case MYYUV_E_HIP: return "HIP runtime error";
    case MYYUV_E_NO_DEVICE: return "No HIP device available";
    case MYYUV_E_BMP_INVALID: return "BMP is invalid";
    case MYYUV_E_BMP_SIGN: return "Unaccounted width and height sign";
    case MYYUV_E_BMP_UNSUPPORTED: return "BMP to IYUV needs 24 or 32 bits per pixel and even height";
    default: return "Unknown error";
  }
}

uint32_t myyuv_dct_payload_bound(uint32_t w, uint32_t h) {
  const uint64_t nb = (uint64_t)(w / 8) * (h / 8) + 2ull * (uint64_t)(w / 16) * (h / 16);
  const uint64_t b = 12 + 24 + nb + nb * kMaxChunk;
  return b > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)((b + 3) & ~3ull);
}

int myyuv_hip_create(int device, myyuv_hip_handle* out) {
  if (!out) return MYYUV_E_ARG;
  *out = nullptr;
  if (!hip_ok()) return MYYUV_E_NO_DEVICE;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return MYYUV_E_NO_DEVICE;
  DeviceGuard g(device);
  auto* c = new myyuv_hip_ctx();
  c->device = device;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return MYYUV_E_HIP;
  }
  if (hipEventCreateWithFlags(&c->done, hipEventDisableTiming) != hipSuccess) {
    (void)hipStreamDestroy(c->stream);
    delete c;
    return MYYUV_E_HIP;
  }
  {
    int cus = 0, n1 = 0, n6 = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&n1, k_fdct_quant, 256, 0) == hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&n6, k_dequant_idct, 256, 0) == hipSuccess &&
        cus > 0 && n1 > 0 && n6 > 0) {
      c->xf_resident[0] = (uint32_t)(cus * n1);
      c->xf_resident[1] = (uint32_t)(cus * n6);
      int nfix = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nfix, k_fdct_fix, 64 * kFixWaves, 0) == hipSuccess &&
          nfix > 0)
        c->fix_resident = (uint32_t)(cus * nfix) * kFixWaves / 4;  // (in 4-wave workgroups)
      if (const char* v = std::getenv("MYYUV_FIX_GRID")) c->fix_grid = (uint32_t)std::atoi(v);
      if (const char* v = std::getenv("MYYUV_FIX_QMAX")) c->fix_qmax = (uint32_t)std::atoi(v);
      if (const char* v = std::getenv("MYYUV_LAUNCH_BLOCKS"))
        c->launch_blocks = std::max(1u, std::min(kMaxLaunchBlocks, (uint32_t)std::strtoul(v, nullptr, 10)));
      {
        const char* v = std::getenv("MYYUV_ENCODER");
        c->fused = v && std::strcmp(v, "fused") == 0;
        const char* d = std::getenv("MYYUV_DECODER");
        c->fused_dec = !(d && std::strcmp(d, "split") == 0);
      }
      // tuning knobs (diagnostic; default 100): K1 / K6 grids as a percentage
      // of the resident workgroups, leaving wave slots to other launch groups
      for (int k = 0; k < 2; k++) {
        const char* v = std::getenv(k == 0 ? "MYYUV_K1_GRID_PCT" : "MYYUV_K6_GRID_PCT");
        const int pct = v ? std::atoi(v) : 100;
        if (pct > 0 && pct < 100) c->xf_resident[k] = std::max(1u, c->xf_resident[k] * (uint32_t)pct / 100u);
      }
    }
  }
  if (c->err.grow(8) || c->psize.grow(4) || c->desc.grow(sizeof(StreamDesc)) ||
      hipMemset(c->err.p, 0xFF, 8) != hipSuccess) {
    (void)hipEventDestroy(c->done);
    (void)hipStreamDestroy(c->stream);
    delete c;
    return MYYUV_E_HIP;
  }
  *out = c;
  return 0;
}

void myyuv_hip_destroy(myyuv_hip_handle c) {
  if (!c) return;
  DeviceGuard g(c->device);
  (void)hipStreamSynchronize(c->stream);
  if (c->last_stream) (void)hipEventSynchronize(c->done);
  drain_profile(c);
  for (auto e : c->free_events) (void)hipEventDestroy(e);
  (void)hipEventDestroy(c->done);
  DevBuf* bufs[] = {&c->frame, &c->coef, &c->stage, &c->oslots, &c->tinfo, &c->srcoff, &c->sizes, &c->loff, &c->tiles, &c->payload,
                    &c->err,   &c->qtd,  &c->psize, &c->desc,  &c->work,  &c->status, &c->sink,
                    &c->bmp,   &c->rmask, &c->zq, &c->bsizes, &c->fix, &c->binfo,
                    &c->pin[0], &c->pin[1], &c->pout[0], &c->pout[1], &c->psz[0], &c->psz[1],
                    &c->perr[0], &c->perr[1]};
  for (auto* b : bufs) b->release();
  if (c->cin) {
    (void)hipStreamSynchronize(c->cin);
    (void)hipStreamSynchronize(c->cout);
    (void)hipStreamDestroy(c->cin);
    (void)hipStreamDestroy(c->cout);
    for (auto& row : c->pev)
      for (auto e : row) (void)hipEventDestroy(e);
    (void)hipHostFree(c->hsz);
    (void)hipHostFree(c->herr);
  }
  (void)hipStreamDestroy(c->stream);
  delete c;
}

int myyuv_hip_reserve(myyuv_hip_handle c, uint32_t w, uint32_t h) {
  if (!c) return MYYUV_E_ARG;
  FrameGeom G;
  int e = make_geom(w, h, G);
  if (e) return e;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  return reserve(c, G);
}

int myyuv_gpu_dct_compress_batch_device(myyuv_hip_handle c, const void* d_in, uint32_t nframes,
                                        uint32_t w, uint32_t h, const uint8_t q[3], void* d_out,
                                        uint32_t cap, uint32_t* d_sizes, void* stream) {
  if (!c || !d_in || !d_out || !d_sizes || !q) return MYYUV_E_ARG;
  if (((uintptr_t)d_out & 3) || ((uintptr_t)d_in & 7) || (nframes > 1 && (cap & 3)))
    return MYYUV_E_ARG;
  for (int p = 0; p < 3; p++)
    if (q[p] < 1 || q[p] > 100) return MYYUV_E_QUALITY;
  FrameGeom G;
  int e = make_geom(w, h, G);
  if (e || (e = set_batch(G, nframes))) return e;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->stream;
  StreamOrder so(c, s);
  // (as several launches when the batch's coefficient image would reach 4 GiB)
  const uint32_t per = launch_frames(G, c->launch_blocks);
  FrameGeom GL = G;
  if ((e = set_batch(GL, std::min(nframes, per))) || (e = reserve(c, GL)) || (e = set_qtables(c, q, s))) return e;
  for (uint32_t f0 = 0; f0 < nframes; f0 += per) {
    GL = G;
    GL.fbase = f0;
    if ((e = set_batch(GL, std::min(per, nframes - f0))) ||
        (e = launch_compress(c, GL, static_cast<const uint8_t*>(d_in) + (size_t)f0 * G.fbytes,
                             static_cast<uint8_t*>(d_out) + (size_t)f0 * cap, cap, d_sizes + f0, s)))
      return e;
  }
  return 0;
}

int myyuv_gpu_dct_decompress_batch_device(myyuv_hip_handle c, const void* d_in, const uint32_t* d_sizes,
                                          uint32_t cap, uint32_t nframes, uint32_t w, uint32_t h,
                                          const uint8_t q[3], void* d_out, void* stream) {
  if (!c || !d_in || !d_out || !d_sizes || !q) return MYYUV_E_ARG;
  if (((uintptr_t)d_in & 3) || ((uintptr_t)d_out & 7) || (nframes > 1 && (cap & 3)))
    return MYYUV_E_ARG;
  for (int p = 0; p < 3; p++)
    if (q[p] < 1 || q[p] > 100) return MYYUV_E_QUALITY;
  FrameGeom G;
  int e = make_geom(w, h, G);
  if (e || (e = set_batch(G, nframes))) return e;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->stream;
  StreamOrder so(c, s);
  const uint32_t per = launch_frames(G, c->launch_blocks);
  FrameGeom GL = G;
  if ((e = set_batch(GL, std::min(nframes, per))) || (e = reserve(c, GL)) || (e = set_qtables(c, q, s))) return e;
  for (uint32_t f0 = 0; f0 < nframes; f0 += per) {
    GL = G;
    GL.fbase = f0;
    if ((e = set_batch(GL, std::min(per, nframes - f0))) ||
        (e = launch_decompress(c, GL, static_cast<const uint8_t*>(d_in) + (size_t)f0 * cap, d_sizes + f0, cap,
                               static_cast<uint8_t*>(d_out) + (size_t)f0 * G.fbytes, s)))
      return e;
  }
  return 0;
}

int myyuv_gpu_dct_compress_device(myyuv_hip_handle c, const void* d_in, uint32_t w, uint32_t h,
                                  const uint8_t q[3], void* d_out, uint32_t cap,
                                  uint32_t* d_size, void* stream) {
  return myyuv_gpu_dct_compress_batch_device(c, d_in, 1, w, h, q, d_out, cap, d_size, stream);
}

int myyuv_gpu_dct_decompress_device(myyuv_hip_handle c, const void* d_in, const uint32_t* d_size,
                                    uint32_t cap, uint32_t w, uint32_t h, const uint8_t q[3],
                                    void* d_out, void* stream) {
  return myyuv_gpu_dct_decompress_batch_device(c, d_in, d_size, cap, 1, w, h, q, d_out, stream);
}

int myyuv_hip_reserve_batch(myyuv_hip_handle c, uint32_t w, uint32_t h, uint32_t nframes) {
  if (!c) return MYYUV_E_ARG;
  FrameGeom G;
  int e = make_geom(w, h, G);
  if (e || (e = set_batch(G, nframes))) return e;
  std::lock_guard<std::mutex> lk(c->mu);
  if ((e = set_batch(G, std::min(nframes, launch_frames(G, c->launch_blocks))))) return e;  // (the largest launch)
  DeviceGuard g(c->device);
  return reserve(c, G);
}

// ---- K7: BMP -> IYUV (myyuv_yuv.cpp:88-128 over myyuv_bmp.cpp:77-101) ----
namespace {

// The checks the conversion itself makes, in the reference's order:
// YUV::load's isValid (width % 4 of isValidHeader; bit_count > 0), then
// colorData's sign cases, then the bmp_to_yuv_map asserts (even size,
// 32 bpp — 24 bpp converts the same way and is accepted).
int bmp_check(int32_t width, int32_t height, uint16_t bit_count, uint32_t* W, uint32_t* H,
              uint32_t* orient) {
  const uint32_t aw = width < 0 ? 0u - (uint32_t)width : (uint32_t)width;
  const uint32_t ah = height < 0 ? 0u - (uint32_t)height : (uint32_t)height;
  if (aw % 4 != 0 || bit_count == 0) return MYYUV_E_BMP_INVALID;
  if (width > 0 && height < 0)
    *orient = 0;
  else if (width < 0 && height > 0)
    *orient = 1;
  else if (width > 0 && height > 0)
    *orient = 2;
  else
    return MYYUV_E_BMP_SIGN;
  if ((bit_count != 24 && bit_count != 32) || ah % 2 != 0) return MYYUV_E_BMP_UNSUPPORTED;
  if ((uint64_t)aw * ah * 4 > 0xFFFFFFFFull) return MYYUV_E_ARG;  // imageSize() is a u32
  *W = aw;
  *H = ah;
  return 0;
}

int launch_bmp(myyuv_hip_ctx* c, const void* src, uint32_t W, uint32_t H, uint32_t orient,
               uint16_t bits, void* dst, hipStream_t s) {
  const uint32_t tiles = (W / 4) * (H / 2);
  if (tiles == 0) return 0;
  const uint32_t grid = std::min(ceil_div(tiles, 256), 8192u);
  const uint8_t* in = static_cast<const uint8_t*>(src);
  uint8_t* out = static_cast<uint8_t*>(dst);
  return bits == 32 ? launch(c, MYYUV_K_BMP, k_bmp_to_iyuv<4>, dim3(grid), dim3(256), s, in, W, H, orient, out)
                    : launch(c, MYYUV_K_BMP, k_bmp_to_iyuv<3>, dim3(grid), dim3(256), s, in, W, H, orient, out);
}

}  // namespace

int myyuv_gpu_bmp_to_iyuv_device(myyuv_hip_handle c, const void* d_bmp, int32_t width, int32_t height,
                                 uint16_t bit_count, void* d_iyuv, void* stream) {
  if (!c || !d_bmp || !d_iyuv) return MYYUV_E_ARG;
  uint32_t W = 0, H = 0, orient = 0;
  int e = bmp_check(width, height, bit_count, &W, &H, &orient);
  if (e) return e;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->stream;
  StreamOrder so(c, s);
  return launch_bmp(c, d_bmp, W, H, orient, bit_count, d_iyuv, s);
}

int myyuv_gpu_bmp_to_iyuv(myyuv_hip_handle c, const uint8_t* bmp_data, int32_t width, int32_t height,
                          uint16_t bit_count, uint8_t* iyuv) {
  if (!c || !bmp_data || !iyuv) return MYYUV_E_ARG;
  uint32_t W = 0, H = 0, orient = 0;
  int e = bmp_check(width, height, bit_count, &W, &H, &orient);
  if (e) return e;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  hipStream_t s = c->stream;
  StreamOrder so(c, s);
  const size_t in_bytes = (size_t)W * H * (bit_count / 8), out_bytes = (size_t)W * H * 3 / 2;
  if (in_bytes == 0) return 0;
  if (c->bmp.grow(in_bytes) || c->frame.grow(out_bytes)) return MYYUV_E_HIP;
  if (h2d(c, c->bmp.p, bmp_data, in_bytes, s)) return MYYUV_E_HIP;
  if ((e = launch_bmp(c, c->bmp.p, W, H, orient, bit_count, c->frame.p, s))) return e;
  if (d2h(c, iyuv, c->frame.p, out_bytes, s)) return MYYUV_E_HIP;
  if (c->prof) drain_profile(c);
  return 0;
}

int myyuv_hip_sync_status(myyuv_hip_handle c, void* stream, int64_t* bad_block) {
  if (!c) return MYYUV_E_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->stream;
  StreamOrder so(c, s);
  int code = read_err(c, s, bad_block);
  if (reset_err(c, s) || hipStreamSynchronize(s) != hipSuccess) return MYYUV_E_HIP;
  if (c->prof) drain_profile(c);
  return code;
}

int myyuv_gpu_dct_compress(myyuv_hip_handle c, const uint8_t* iyuv, uint32_t w, uint32_t h,
                           const uint8_t q[3], uint8_t* payload, uint32_t cap,
                           uint32_t* payload_size) {
  if (!c || !iyuv || !payload || !payload_size || !q) return MYYUV_E_ARG;
  for (int p = 0; p < 3; p++)
    if (q[p] < 1 || q[p] > 100) return MYYUV_E_QUALITY;
  FrameGeom G;
  int e = make_geom(w, h, G);
  if (e) return e;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  hipStream_t s = c->stream;
  StreamOrder so(c, s);
  const size_t fbytes = (size_t)w * h * 3 / 2;
  const uint32_t bound = myyuv_dct_payload_bound(w, h);
  if ((e = reserve(c, G)) || (e = set_qtables(c, q, s))) return e;
  if (c->frame.grow(fbytes) || c->payload.grow(bound)) return MYYUV_E_HIP;
  if (reset_err(c, s)) return MYYUV_E_HIP;
  if (h2d(c, c->frame.p, iyuv, fbytes, s)) return MYYUV_E_HIP;
  if ((e = launch_compress(c, G, c->frame.p, c->payload.p, bound, c->psize.as<uint32_t>(), s)))
    return e;
  uint32_t size = 0;
  if (hipMemcpyAsync(&size, c->psize.p, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return MYYUV_E_HIP;
  int64_t bad = -1;
  if ((e = read_err(c, s, &bad))) {
    (void)reset_err(c, s);
    return e;
  }
  *payload_size = size;
  if (size > cap) return MYYUV_E_CAPACITY;
  if (d2h(c, payload, c->payload.p, size, s)) return MYYUV_E_HIP;
  if (c->prof) drain_profile(c);
  return 0;
}

int myyuv_gpu_dct_decompress(myyuv_hip_handle c, const uint8_t* payload, uint32_t size, uint32_t w,
                             uint32_t h, const uint8_t q[3], uint8_t* iyuv, int64_t* bad_block) {
  if (bad_block) *bad_block = -1;
  if (!c || !payload || !iyuv || !q) return MYYUV_E_ARG;
  int e_hdr = 0;
  for (int p = 0; p < 3; p++)
    if (q[p] < 1 || q[p] > 100) return MYYUV_E_QUALITY;
  // DCTYUV::load / DCTYUVPlane::load checks (DCT.cpp:454 -> :130-159, :39-62)
  // come before the dimension checks in the reference: validate the stream
  // header on the host (the device re-checks it in k_scan_chain).
  if ((e_hdr = host_parse_headers(payload, size))) return e_hdr;
  FrameGeom G;
  int e = make_geom(w, h, G);
  if (e) return e;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  hipStream_t s = c->stream;
  StreamOrder so(c, s);
  const uint32_t cap = (size + 3) & ~3u;
  const size_t fbytes = (size_t)w * h * 3 / 2;
  if ((e = reserve(c, G)) || (e = set_qtables(c, q, s))) return e;
  if (c->frame.grow(fbytes) || c->payload.grow(cap)) return MYYUV_E_HIP;
  if (reset_err(c, s)) return MYYUV_E_HIP;
  if (hipMemsetAsync(static_cast<uint8_t*>(c->payload.p) + (cap - 4), 0, 4, s) != hipSuccess ||
      h2d(c, c->payload.p, payload, size, s) ||
      hipMemcpyAsync(c->psize.p, &size, 4, hipMemcpyHostToDevice, s) != hipSuccess)
    return MYYUV_E_HIP;
  if ((e = launch_decompress(c, G, c->payload.p, c->psize.as<const uint32_t>(), cap, c->frame.p, s)))
    return e;
  if ((e = read_err(c, s, bad_block))) {
    (void)reset_err(c, s);
    (void)hipStreamSynchronize(s);
    return e;
  }
  if (d2h(c, iyuv, c->frame.p, fbytes, s)) return MYYUV_E_HIP;
  if (c->prof) drain_profile(c);
  return 0;
}

// ---- host-buffer batches, pipelined ------------------
//
// The batch is cut into chunks of B frames, alternating between two device
// slots.  Chunk k's host -> device copies run on cin while chunk k-1's kernels
// run on the context's stream and chunk k-2's results go back on cout, so the
// PCIe transfers of both directions and the kernels overlap; the host waits
// only for a chunk's sizes and error word (pinned, copied behind its
// kernels) before it queues that chunk's device -> host copies.  Each copy
// goes straight between the caller's (pageable) buffers and the slot.
namespace {

constexpr uint32_t kPipeMaxChunk = 8;
// MYYUV_PIPE_TRACE=1: one stderr line per pipeline step (diagnostic)
bool pipe_trace() {
  static int t = -1;
  if (t < 0) t = std::getenv("MYYUV_PIPE_TRACE") ? 1 : 0;
  return t == 1;
}
#define PIPE_TRACE(...)                   \
  do {                                    \
    if (pipe_trace()) {                   \
      std::fprintf(stderr, __VA_ARGS__);  \
      std::fflush(stderr);                \
    }                                     \
  } while (0)
constexpr size_t kPipeSlotBytes = (size_t)2 << 30;  // per slot: chunk frames x (input + output) bytes

// frames per chunk: about 8 chunks per batch (the first chunk's upload and
// the last one's download are not overlapped), at most kPipeMaxChunk and
// within the slot budget
uint32_t pipe_chunk(uint32_t nf, size_t per_frame) {
  uint32_t b = std::max(1u, std::min(kPipeMaxChunk, nf / 8));
  while (b > 1 && (size_t)b * per_frame > kPipeSlotBytes) b--;
  return b;
}

int pipe_init(myyuv_hip_ctx* c) {
  if (c->cin) return 0;
  if (hipStreamCreateWithFlags(&c->cin, hipStreamNonBlocking) != hipSuccess) return MYYUV_E_HIP;
  if (hipStreamCreateWithFlags(&c->cout, hipStreamNonBlocking) != hipSuccess) {
    (void)hipStreamDestroy(c->cin);
    c->cin = nullptr;
    return MYYUV_E_HIP;
  }
  int e = 0;
  for (auto& row : c->pev)
    for (auto& ev : row) e |= hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess;
  e |= hipHostMalloc((void**)&c->hsz, 2 * kPipeMaxChunk * 4, hipHostMallocDefault) != hipSuccess;
  e |= hipHostMalloc((void**)&c->herr, 2 * 8, hipHostMallocDefault) != hipSuccess;
  for (int k = 0; k < 2; k++) {
    e |= c->psz[k].grow(kPipeMaxChunk * 4);
    e |= c->perr[k].grow(8);
    if (!e) e |= hipMemset(c->perr[k].p, 0xFF, 8) != hipSuccess;
  }
  return e ? MYYUV_E_HIP : 0;
}

// Waits for every pipeline stream (an early return must not leave copies to
// or from the caller's buffers in flight).
struct PipeDrain {
  myyuv_hip_ctx* c;
  ~PipeDrain() {
    (void)hipStreamSynchronize(c->cin);
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->cout);
  }
};

// A chunk's error word (read_err's encoding) -> code, with the failing block
// made batch-global (chunk's first frame f0, nblk blocks per frame).
int chunk_err(unsigned long long v, uint32_t f0, uint32_t nblk, int64_t* bad_block) {
  if (v == ~0ull) return 0;
  const uint64_t key = v >> 8;
  if (bad_block) *bad_block = key == 0 ? -1 : (int64_t)(key >> 1) + (int64_t)f0 * nblk;
  return (int)(v & 0xFF);
}

int compress_frames(myyuv_hip_ctx* c, const uint8_t* const* frames, uint32_t nf, uint32_t w, uint32_t h,
                    const uint8_t q[3], myyuv_payload_alloc_fn alloc, void* user, uint32_t* sizes) {
  FrameGeom G;
  int e = make_geom(w, h, G);
  if (e) return e;
  const size_t fb = (size_t)w * h * 3 / 2;
  const uint32_t dcap = (myyuv_dct_payload_bound(w, h) + 3) & ~3u;  // device slot per frame
  const uint32_t B = std::min(pipe_chunk(nf, fb + dcap), launch_frames(G, c->launch_blocks));
  FrameGeom GB = G;
  if ((e = set_batch(GB, B))) return e;
  hipStream_t s = c->stream;
  StreamOrder so(c, s);
  if ((e = pipe_init(c)) || (e = reserve(c, GB)) || (e = set_qtables(c, q, s))) return e;
  for (int k = 0; k < 2; k++)
    if (c->pin[k].grow(fb * B) || c->pout[k].grow((size_t)dcap * B)) return MYYUV_E_HIP;
  PipeDrain drain{c};
  const uint32_t nchunks = ceil_div(nf, B);
  // chunk k's sizes and error word are on the host: its payloads go back
  auto finish = [&](uint32_t k) -> int {
    const uint32_t sl = k & 1, f0 = k * B, n = std::min(B, nf - f0);
    PIPE_TRACE("pipe c finish %u: wait kernels\n", k);
    if (hipEventSynchronize(c->pev[1][sl]) != hipSuccess) return MYYUV_E_HIP;
    PIPE_TRACE("pipe c finish %u: kernels done\n", k);
    if (int ce = chunk_err(c->herr[sl], f0, G.cum[3], nullptr)) return ce;
    for (uint32_t i = 0; i < n; i++) {
      const uint32_t size = c->hsz[sl * kPipeMaxChunk + i];
      sizes[f0 + i] = size;
      uint8_t* dst = alloc(user, f0 + i, size);
      if (!dst) return MYYUV_E_CAPACITY;
      if (hipMemcpyAsync(dst, c->pout[sl].as<uint8_t>() + (size_t)i * dcap, size, hipMemcpyDeviceToHost,
                         c->cout) != hipSuccess)
        return MYYUV_E_HIP;
    }
    PIPE_TRACE("pipe c finish %u: downloads queued\n", k);
    return hipEventRecord(c->pev[2][sl], c->cout) == hipSuccess ? 0 : MYYUV_E_HIP;
  };
  PIPE_TRACE("pipe c: %u frames, chunks of %u\n", nf, B);
  for (uint32_t k = 0; k < nchunks; k++) {
    const uint32_t sl = k & 1, f0 = k * B, n = std::min(B, nf - f0);
    FrameGeom GK = G;
    if ((e = set_batch(GK, n))) return e;
    PIPE_TRACE("pipe c chunk %u: upload\n", k);
    // upload (slot free once chunk k-2's kernels have read it)
    if (k >= 2 && hipStreamWaitEvent(c->cin, c->pev[1][sl], 0) != hipSuccess) return MYYUV_E_HIP;
    for (uint32_t i = 0; i < n; i++)
      if (hipMemcpyAsync(c->pin[sl].as<uint8_t>() + i * fb, frames[f0 + i], fb, hipMemcpyHostToDevice, c->cin) !=
          hipSuccess)
        return MYYUV_E_HIP;
    if (hipEventRecord(c->pev[0][sl], c->cin) != hipSuccess) return MYYUV_E_HIP;
    PIPE_TRACE("pipe c chunk %u: uploads queued\n", k);
    // kernels (output slot free once chunk k-2's payloads are back)
    if (hipStreamWaitEvent(s, c->pev[0][sl], 0) != hipSuccess ||
        (k >= 2 && hipStreamWaitEvent(s, c->pev[2][sl], 0) != hipSuccess))
      return MYYUV_E_HIP;
    unsigned long long* perr = c->perr[sl].as<unsigned long long>();
    if ((e = launch_compress(c, GK, c->pin[sl].p, c->pout[sl].p, dcap, c->psz[sl].as<uint32_t>(), s, perr)))
      return e;
    if (hipMemcpyAsync(c->hsz + sl * kPipeMaxChunk, c->psz[sl].p, (size_t)n * 4, hipMemcpyDeviceToHost, s) !=
            hipSuccess ||
        hipMemcpyAsync(c->herr + sl, perr, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemsetAsync(perr, 0xFF, 8, s) != hipSuccess || hipEventRecord(c->pev[1][sl], s) != hipSuccess)
      return MYYUV_E_HIP;
    if (k >= 1 && (e = finish(k - 1))) return e;
  }
  if ((e = finish(nchunks - 1))) return e;
  PIPE_TRACE("pipe c: wait downloads\n");
  if (hipStreamSynchronize(c->cout) != hipSuccess) return MYYUV_E_HIP;
  PIPE_TRACE("pipe c: done\n");
  if (c->prof) drain_profile(c);
  return 0;
}

int decompress_frames(myyuv_hip_ctx* c, const uint8_t* const* payloads, const uint32_t* psizes, uint32_t nf,
                      uint32_t w, uint32_t h, const uint8_t q[3], uint8_t* const* frames, int64_t* bad_block) {
  FrameGeom G;
  int e = make_geom(w, h, G);
  if (e) return e;
  const size_t fb = (size_t)w * h * 3 / 2;
  uint32_t icap = 4;  // device slot per stream: the longest, 4-aligned
  for (uint32_t f = 0; f < nf; f++) icap = std::max(icap, (psizes[f] + 3u) & ~3u);
  const uint32_t B = std::min(pipe_chunk(nf, fb + icap), launch_frames(G, c->launch_blocks));
  FrameGeom GB = G;
  if ((e = set_batch(GB, B))) return e;
  hipStream_t s = c->stream;
  StreamOrder so(c, s);
  if ((e = pipe_init(c)) || (e = reserve(c, GB)) || (e = set_qtables(c, q, s))) return e;
  for (int k = 0; k < 2; k++)
    if (c->pin[k].grow((size_t)icap * B) || c->pout[k].grow(fb * B)) return MYYUV_E_HIP;
  PipeDrain drain{c};
  const uint32_t nchunks = ceil_div(nf, B);
  auto finish = [&](uint32_t k) -> int {
    const uint32_t sl = k & 1, f0 = k * B, n = std::min(B, nf - f0);
    if (hipEventSynchronize(c->pev[1][sl]) != hipSuccess) return MYYUV_E_HIP;
    if (int ce = chunk_err(c->herr[sl], f0, G.cum[3], bad_block)) return ce;
    for (uint32_t i = 0; i < n; i++)
      if (hipMemcpyAsync(frames[f0 + i], c->pout[sl].as<uint8_t>() + i * fb, fb, hipMemcpyDeviceToHost, c->cout) !=
          hipSuccess)
        return MYYUV_E_HIP;
    return hipEventRecord(c->pev[2][sl], c->cout) == hipSuccess ? 0 : MYYUV_E_HIP;
  };
  for (uint32_t k = 0; k < nchunks; k++) {
    const uint32_t sl = k & 1, f0 = k * B, n = std::min(B, nf - f0);
    FrameGeom GK = G;
    if ((e = set_batch(GK, n))) return e;
    if (k >= 2 && hipStreamWaitEvent(c->cin, c->pev[1][sl], 0) != hipSuccess) return MYYUV_E_HIP;
    uint8_t* slot = c->pin[sl].as<uint8_t>();
    for (uint32_t i = 0; i < n; i++) {
      const uint32_t sz = psizes[f0 + i], cap_i = (sz + 3u) & ~3u;
      // the stream's last word zero-padded (the scan reads whole words), then the bytes
      if ((cap_i >= 4 && hipMemsetAsync(slot + (size_t)i * icap + cap_i - 4, 0, 4, c->cin) != hipSuccess) ||
          hipMemcpyAsync(slot + (size_t)i * icap, payloads[f0 + i], sz, hipMemcpyHostToDevice, c->cin) != hipSuccess)
        return MYYUV_E_HIP;
    }
    if (hipMemcpyAsync(c->psz[sl].p, psizes + f0, (size_t)n * 4, hipMemcpyHostToDevice, c->cin) != hipSuccess ||
        hipEventRecord(c->pev[0][sl], c->cin) != hipSuccess)
      return MYYUV_E_HIP;
    if (hipStreamWaitEvent(s, c->pev[0][sl], 0) != hipSuccess ||
        (k >= 2 && hipStreamWaitEvent(s, c->pev[2][sl], 0) != hipSuccess))
      return MYYUV_E_HIP;
    unsigned long long* perr = c->perr[sl].as<unsigned long long>();
    if ((e = launch_decompress(c, GK, slot, c->psz[sl].as<const uint32_t>(), icap, c->pout[sl].p, s, perr)))
      return e;
    if (hipMemcpyAsync(c->herr + sl, perr, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemsetAsync(perr, 0xFF, 8, s) != hipSuccess || hipEventRecord(c->pev[1][sl], s) != hipSuccess)
      return MYYUV_E_HIP;
    if (k >= 1 && (e = finish(k - 1))) return e;
  }
  if ((e = finish(nchunks - 1))) return e;
  if (hipStreamSynchronize(c->cout) != hipSuccess) return MYYUV_E_HIP;
  if (c->prof) drain_profile(c);
  return 0;
}

struct SlotAlloc {
  uint8_t* base;
  uint32_t cap;
};
uint8_t* slot_alloc(void* user, uint32_t frame, uint32_t size) {
  const SlotAlloc* a = static_cast<const SlotAlloc*>(user);
  return size <= a->cap ? a->base + (size_t)frame * a->cap : nullptr;
}

int check_q(const uint8_t q[3]) {
  for (int p = 0; p < 3; p++)
    if (q[p] < 1 || q[p] > 100) return MYYUV_E_QUALITY;
  return 0;
}

}  // namespace

int myyuv_gpu_dct_compress_frames(myyuv_hip_handle c, const uint8_t* const* frames, uint32_t nframes, uint32_t w,
                                  uint32_t h, const uint8_t q[3], myyuv_payload_alloc_fn alloc, void* user,
                                  uint32_t* sizes) {
  if (!c || !frames || !alloc || !sizes || !q || nframes == 0) return MYYUV_E_ARG;
  for (uint32_t f = 0; f < nframes; f++)
    if (!frames[f]) return MYYUV_E_ARG;
  if (int e = check_q(q)) return e;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  return compress_frames(c, frames, nframes, w, h, q, alloc, user, sizes);
}

int myyuv_gpu_dct_compress_batch(myyuv_hip_handle c, const uint8_t* iyuv, uint32_t nframes, uint32_t w,
                                 uint32_t h, const uint8_t q[3], uint8_t* payloads, uint32_t cap,
                                 uint32_t* sizes) {
  if (!c || !iyuv || !payloads || !sizes || !q || nframes == 0) return MYYUV_E_ARG;
  if (int e = check_q(q)) return e;
  const size_t fb = (size_t)w * h * 3 / 2;
  std::vector<const uint8_t*> fr(nframes);
  for (uint32_t f = 0; f < nframes; f++) fr[f] = iyuv + f * fb;
  SlotAlloc a{payloads, cap};
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  return compress_frames(c, fr.data(), nframes, w, h, q, slot_alloc, &a, sizes);
}

int myyuv_gpu_dct_decompress_frames(myyuv_hip_handle c, const uint8_t* const* payloads, const uint32_t* sizes,
                                    uint32_t nframes, uint32_t w, uint32_t h, const uint8_t q[3],
                                    uint8_t* const* frames, int64_t* bad_block) {
  if (bad_block) *bad_block = -1;
  if (!c || !payloads || !sizes || !frames || !q || nframes == 0) return MYYUV_E_ARG;
  for (uint32_t f = 0; f < nframes; f++)
    if (!payloads[f] || !frames[f]) return MYYUV_E_ARG;
  if (int e = check_q(q)) return e;
  // every stream's DCTYUV::load checks first (DCT.cpp:454; the single-frame
  // call's order), frame by frame
  for (uint32_t f = 0; f < nframes; f++)
    if (int e = host_parse_headers(payloads[f], sizes[f])) return e;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  return decompress_frames(c, payloads, sizes, nframes, w, h, q, frames, bad_block);
}

int myyuv_gpu_dct_decompress_batch(myyuv_hip_handle c, const uint8_t* payloads, const uint32_t* sizes, uint32_t cap,
                                   uint32_t nframes, uint32_t w, uint32_t h, const uint8_t q[3], uint8_t* iyuv,
                                   int64_t* bad_block) {
  if (bad_block) *bad_block = -1;
  if (!c || !payloads || !sizes || !iyuv || !q || nframes == 0) return MYYUV_E_ARG;
  for (uint32_t f = 0; f < nframes; f++)
    if (sizes[f] > cap) return MYYUV_E_ARG;
  const size_t fb = (size_t)w * h * 3 / 2;
  std::vector<const uint8_t*> in(nframes);
  std::vector<uint8_t*> out(nframes);
  for (uint32_t f = 0; f < nframes; f++) {
    in[f] = payloads + (size_t)f * cap;
    out[f] = iyuv + f * fb;
  }
  return myyuv_gpu_dct_decompress_frames(c, in.data(), sizes, nframes, w, h, q, out.data(), bad_block);
}

int myyuv_hip_profile(myyuv_hip_handle c, int enable) {
  return myyuv_hip_profile_kernels(c, enable ? (1u << MYYUV_K_COUNT) - 1u : 0u);
}

int myyuv_hip_profile_kernels(myyuv_hip_handle c, uint32_t mask) {
  if (!c) return MYYUV_E_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  (void)hipStreamSynchronize(c->stream);
  drain_profile(c);
  c->prof = mask & ((1u << MYYUV_K_COUNT) - 1u);
  for (int k = 0; k < MYYUV_K_COUNT; k++) {
    c->ms[k] = 0;
    c->launches[k] = 0;
  }
  return 0;
}

int myyuv_hip_kernel_stats(myyuv_hip_handle c, double ms[MYYUV_K_COUNT],
                           int64_t launches[MYYUV_K_COUNT]) {
  if (!c || !ms || !launches) return MYYUV_E_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  drain_profile(c);
  for (int k = 0; k < MYYUV_K_COUNT; k++) {
    ms[k] = c->ms[k];
    launches[k] = c->launches[k];
  }
  return 0;
}

// Diagnostic builds: per-wave stage cycles of the CAP=8 pass (n waves).
int myyuv_debug_k2_fstamps(uint32_t* out, uint32_t n) {
#ifdef MYYUV_STAMPS
  if (n > 8192) n = 8192;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_k2_fstamps), (size_t)n * 32) == hipSuccess ? 0 : MYYUV_E_HIP;
#else
  (void)out;
  (void)n;
  return MYYUV_E_ARG;
#endif
}

// Diagnostic builds (-DMYYUV_STAMPS): K2's per-wave window phases of the last
// launch, n waves x 8 words (k_huff_encode.hip g_k2_win; word 7 = 1 for a
// wave that ran), then zeroed.
int myyuv_debug_k2_win(uint32_t* out, uint32_t n) {
#ifdef MYYUV_STAMPS
  if (n > 65536) n = 65536;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_k2_win), (size_t)n * 32) != hipSuccess) return MYYUV_E_HIP;
  std::vector<uint32_t> zero((size_t)n * 8, 0u);
  return hipMemcpyToSymbol(HIP_SYMBOL(g_k2_win), zero.data(), (size_t)n * 32) == hipSuccess ? 0 : MYYUV_E_HIP;
#else
  (void)out;
  (void)n;
  return MYYUV_E_ARG;
#endif
}

// Diagnostic builds: per-block phase cycles of the wave encoder (n blocks).
int myyuv_debug_k2_wstamps(uint32_t* out, uint32_t n) {
#ifdef MYYUV_STAMPS
  if (n > 65536) n = 65536;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_k2_wstamps), (size_t)n * 32) == hipSuccess ? 0 : MYYUV_E_HIP;
#else
  (void)out;
  (void)n;
  return MYYUV_E_ARG;
#endif
}

// Diagnostic builds (-DMYYUV_STAMPS): the fused decoder's per-phase wave
// cycles of the last launch, n waves x 8 words (k_huff_decode.hip
// g_dec_wstamps; word 7 = 1 for a wave that ran), then zeroed.
int myyuv_debug_dec_stamps(uint32_t* out, uint32_t n) {
#ifdef MYYUV_STAMPS
  if (n > 65536) n = 65536;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dec_wstamps), (size_t)n * 32) != hipSuccess) return MYYUV_E_HIP;
  std::vector<uint32_t> zero((size_t)n * 8, 0u);
  return hipMemcpyToSymbol(HIP_SYMBOL(g_dec_wstamps), zero.data(), (size_t)n * 32) == hipSuccess ? 0 : MYYUV_E_HIP;
#else
  (void)out;
  (void)n;
  return MYYUV_E_ARG;
#endif
}

// Diagnostic: stop launching the kernels whose bit (1 << MYYUV_K_*) is set,
// to measure each kernel's share of a pipelined run.  The buffers keep what the
// last real launch wrote, so repeating identical frames still decodes.
int myyuv_debug_skip_kernels(myyuv_hip_handle c, uint32_t mask) {
  if (!c) return MYYUV_E_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  c->skip = mask;
  return 0;
}

// Diagnostic builds (-DMYYUV_STAMPS): summed per-stage wave cycles of K2
// since the last call; returns MYYUV_E_ARG in normal builds.
int myyuv_debug_k2_stamps(unsigned long long out[40]) {
#ifdef MYYUV_STAMPS
  unsigned long long zero[40] = {0};
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_k2_stamps), 320) != hipSuccess) return MYYUV_E_HIP;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_k2_stamps), zero, 320) != hipSuccess) return MYYUV_E_HIP;
  return 0;
#else
  (void)out;
  return MYYUV_E_ARG;
#endif
}

// Diagnostic: the coefficient image of the last compress/decompress (natural
// order, the quad layout of codec_common.hpp), n blocks, as int16[n][64].
int myyuv_debug_coef(myyuv_hip_handle c, int16_t* out, uint32_t n) {
  if (!c || !out) return MYYUV_E_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  const size_t nq = (size_t)ceil_div(n, kWave) * kCoefQuadsPerWave;
  if (nq * 16 > c->coef.n) return MYYUV_E_ARG;
  if (n > c->rmask.n) return MYYUV_E_ARG;
  std::vector<uint4> img(nq);
  std::vector<uint8_t> rm(n);
  if (hipStreamSynchronize(c->stream) != hipSuccess ||
      hipMemcpy(img.data(), c->coef.p, nq * 16, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(rm.data(), c->rmask.p, n, hipMemcpyDeviceToHost) != hipSuccess)
    return MYYUV_E_HIP;
  for (uint32_t b = 0; b < n; b++)
    for (uint32_t q = 0; q < 8; q++) {  // rows outside the row mask are zero (not stored)
      if ((rm[b] >> q) & 1u)
        std::memcpy(out + (size_t)b * 64 + q * 8, &img[coef_quad(b, q)], 16);
      else
        std::memset(out + (size_t)b * 64 + q * 8, 0, 16);
    }
  return 0;
}

// Diagnostic: the tile-info guard band.  arm != 0 fills the kWinTilesBig x
// kTInfoWords words after tile ntiles (the batch's last tile) with a canary;
// arm == 0 returns in *changed how many of them no longer hold it (a kernel
// wrote past the batch's tiles: the K2 window overrun of round 5's advice).
int myyuv_debug_tinfo_guard(myyuv_hip_handle c, uint32_t ntiles, int arm, uint32_t* changed) {
  if (!c) return MYYUV_E_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  constexpr uint32_t kGuardWords = kWinTilesBig * kTInfoWords;
  constexpr uint32_t kCanary = 0xA5C3E1F7u;
  const size_t off = (size_t)ntiles * kTInfoWords * 4;
  if (off + kGuardWords * 4 > c->tinfo.n) return MYYUV_E_ARG;
  std::vector<uint32_t> w(kGuardWords, kCanary);
  if (hipStreamSynchronize(c->stream) != hipSuccess) return MYYUV_E_HIP;
  uint8_t* p = static_cast<uint8_t*>(c->tinfo.p) + off;
  if (arm) return hipMemcpy(p, w.data(), kGuardWords * 4, hipMemcpyHostToDevice) == hipSuccess ? 0 : MYYUV_E_HIP;
  if (!changed) return MYYUV_E_ARG;
  if (hipMemcpy(w.data(), p, kGuardWords * 4, hipMemcpyDeviceToHost) != hipSuccess) return MYYUV_E_HIP;
  uint32_t n = 0;
  for (uint32_t v : w) n += v != kCanary;
  *changed = n;
  return 0;
}

// ---- block-level KAT entry points -----------------------------------------
int myyuv_gpu_fdct_blocks(myyuv_hip_handle c, const uint8_t* px, uint32_t nblocks,
                          const float qtable[64], int16_t* coef_zz) {
  if (!c || !px || !qtable || !coef_zz || nblocks == 0) return MYYUV_E_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  hipStream_t s = c->stream;
  StreamOrder so(c, s);
  // one plane of width 8 (one block per block-row); planes 1, 2 empty
  FrameGeom G;
  std::memset(&G, 0, sizeof(G));
  G.pw[0] = 8;
  G.ph[0] = 8 * nblocks;
  G.bw[0] = 1;
  G.bmag[0] = block_magic(1);
  G.cum[1] = G.cum[2] = G.cum[3] = nblocks;
  G.ucum[1] = G.ucum[2] = G.ucum[3] = ceil_div(nblocks, kXfUnit);
  G.nframes = 1;
  G.fbytes = nblocks * 64;
  G.umag = block_magic(G.ucum[3]);
  QTables t;
  std::memset(&t, 0, sizeof(t));
  std::memcpy(t.q[0], qtable, 256);
  finish_qtables(t, 1);
  if (reserve(c, G) || c->frame.grow((size_t)nblocks * 64) || c->qtd.grow(sizeof(QTables)))
    return MYYUV_E_HIP;
  c->q_valid = false;
  if (hipStreamSynchronize(s) != hipSuccess ||
      hipMemcpy(c->qtd.p, &t, sizeof(t), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(c->frame.p, px, (size_t)nblocks * 64, hipMemcpyHostToDevice) != hipSuccess)
    return MYYUV_E_HIP;
  if (launch_fdct(c, G, c->frame.as<const uint8_t>(), c->qtd.as<const QTables>(), nullptr, s))
    return MYYUV_E_HIP;
  std::vector<uint32_t> words((size_t)ceil_div(nblocks, kWave) * kCoefQuadsPerWave * 4);
  std::vector<uint8_t> rm(nblocks);
  if (hipGetLastError() != hipSuccess ||
      hipMemcpyAsync(words.data(), c->coef.p, words.size() * 4, hipMemcpyDeviceToHost, s) !=
          hipSuccess ||
      hipMemcpyAsync(rm.data(), c->rmask.p, nblocks, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return MYYUV_E_HIP;
  for (uint32_t g = 0; g < nblocks; g++) {
    int16_t nat[64];
    for (uint32_t c4 = 0; c4 < 8; c4++) {  // rows K1 left out of the image (mask bit clear) are zero
      if ((rm[g] >> c4) & 1u)
        std::memcpy(nat + 8 * c4, &words[(size_t)coef_quad(g, c4) * 4], 16);
      else
        std::memset(nat + 8 * c4, 0, 16);
    }
    for (int z = 0; z < 64; z++) coef_zz[(size_t)g * 64 + z] = nat[kZigzag[z]];
  }
  return 0;
}

int myyuv_gpu_huff_encode_blocks(myyuv_hip_handle c, const int16_t* coef_zz, uint32_t nblocks,
                                 uint8_t* chunks160, uint8_t* sizes) {
  if (!c || !coef_zz || !chunks160 || !sizes || nblocks == 0) return MYYUV_E_ARG;
  // the chunk format carries 11-bit symbols (pack11bit, Huffman.cpp:36-52);
  // K1 never produces others (DCT.cpp:276 asserts the range)
  for (size_t i = 0; i < (size_t)nblocks * 64; i++)
    if (coef_zz[i] < -1024 || coef_zz[i] > 1023) return MYYUV_E_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  hipStream_t s = c->stream;
  StreamOrder so(c, s);
  FrameGeom G;
  std::memset(&G, 0, sizeof(G));
  G.cum[1] = G.cum[2] = G.cum[3] = nblocks;  // one plane of nblocks blocks
  G.tcum[1] = G.tcum[2] = G.tcum[3] = ceil_div(nblocks, kK2Group);
  G.nframes = 1;
  if (reserve(c, G)) return MYYUV_E_HIP;
  const uint32_t nwaves = ceil_div(nblocks, kWave);
  // host-side relayout into K1's output format: natural-order quads
  // and the per-block words K1 writes for K2's classification (binfo_word;
  // every row marked present)
  std::vector<uint32_t> words((size_t)nwaves * kCoefQuadsPerWave * 4, 0u), info(nblocks);
  for (uint32_t g = 0; g < nblocks; g++) {
    int16_t nat[64];
    uint32_t nnz = 0, msz = 0;
    for (int z = 0; z < 64; z++) {
      const int16_t v = coef_zz[(size_t)g * 64 + z];
      nat[kZigzag[z]] = v;
      if (v != 0) {
        nnz++;
        msz = (uint32_t)z + 1u;
      }
    }
    for (uint32_t c4 = 0; c4 < 8; c4++)
      std::memcpy(&words[(size_t)coef_quad(g, c4) * 4], nat + 8 * c4, 16);
    info[g] = binfo_word(0xFFu, msz, class_of(nnz, msz), (uint32_t)(uint16_t)nat[0]);
  }
  if (hipMemcpy(c->coef.p, words.data(), words.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(c->binfo.p, info.data(), (size_t)nblocks * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemsetAsync(c->rmask.p, 0xFF, nblocks, s) != hipSuccess ||  // every row present
      hipMemsetAsync(c->work.p, 0, 4, s) != hipSuccess)  // K1 zeroes it in the codec path
    return MYYUV_E_HIP;
  if (launch_huff_encode(c, G, s)) return MYYUV_E_HIP;
  // K2's hand-off (codec_common.hpp): per tile the waves' dense runs, the
  // chunks of blocks with more than 8 symbols in their own slots
  const uint32_t ntile = G.tcum[3];
  std::vector<uint8_t> stage((size_t)win_tiles_alloc(ntile) * kTileCap), oslots((size_t)nblocks * kMaxChunk);
  std::vector<uint32_t> soff(nblocks);
  if (hipMemcpyAsync(stage.data(), c->stage.p, stage.size(), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipMemcpyAsync(oslots.data(), c->oslots.p, oslots.size(), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipMemcpyAsync(soff.data(), c->srcoff.p, (size_t)nblocks * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipMemcpyAsync(sizes, c->sizes.p, nblocks, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return MYYUV_E_HIP;
  for (uint32_t g = 0; g < nblocks; g++) {
    uint8_t* dst = chunks160 + (size_t)g * kMaxChunk;
    std::memset(dst, 0, kMaxChunk);
    const uint8_t* src = soff[g] == kSrcOverflow ? oslots.data() + (size_t)g * kMaxChunk
                                                 : stage.data() + (size_t)win_first_tile(g / kK2Group, k2_win(G.nframes * ntile)) * kTileCap + soff[g];
    std::memcpy(dst, src, sizes[g]);
  }
  return 0;
}

}  // extern "C"
