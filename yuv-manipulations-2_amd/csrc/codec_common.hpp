// codec_common.hpp — shared constants and frame geometry for the gfx950 DCT
// codec kernels.  Constants restate myyuv_DCT/DCT.cpp:199-230 (quantisation
// bases, float-literal DCT basis) and Huffman.cpp:32-34 (zig-zag order).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace myyuv_gpu {

constexpr int kWave = 64;
constexpr uint32_t kXfUnit = 16;  // blocks per K1/K6 wave unit (four lanes per block)
#ifndef MYYUV_XF_WAVES
#define MYYUV_XF_WAVES 8192
#endif
constexpr uint32_t kXfWaves = MYYUV_XF_WAVES;  // persistent K1/K6 grid: waves (8 per SIMD)
constexpr int kSlotWords = 40;  // 160-B chunk slot per block (max chunk 155 B)
// K1/K6 sink (stores of lanes past a plane's end and of all-zero rows):
// kSinkQuads 16-B words per slot, kSinkSlots slots, wave w using slot
// w % kSinkSlots (one slot: every wave's skipped stores meet in 3 KB)
#ifndef MYYUV_SINK_SLOTS
#define MYYUV_SINK_SLOTS 1
#endif
constexpr uint32_t kSinkQuads = 192, kSinkSlots = MYYUV_SINK_SLOTS;
// k_fdct_fix: waves per workgroup
#ifndef MYYUV_FIX_WAVES
#define MYYUV_FIX_WAVES 4
#endif
constexpr uint32_t kFixWaves = MYYUV_FIX_WAVES;
// K1 -> k_fdct_fix: the unproven BLOCKS (entry ua * 16 + b: block slot b of
// unit ua) in kFixLists lists (unit ua's blocks in list ua % kFixLists), so
// the appends spread over as many atomic counters: the counters of parity p
// (launches alternate) one per 128-B line from word 0, list c from word
// kFixHeader at c * fix_list_cap(units) (16 blocks per unit: no list can
// overflow)
constexpr uint32_t kFixLists = 32, kFixHeader = 2 * kFixLists * 32;
__host__ __device__ __forceinline__ uint32_t* fix_count(uint32_t* fix, uint32_t par, uint32_t c) {
  return fix + (par * kFixLists + c) * 32u;
}
__host__ __device__ __forceinline__ uint32_t fix_list_cap(uint32_t units) {
  return 16u * ((units + kFixLists - 1) / kFixLists);
}
__host__ __device__ __forceinline__ size_t fix_words(uint32_t units) {
  return kFixHeader + (size_t)kFixLists * fix_list_cap(units);
}
constexpr int kMaxChunk = 160;

// Float-literal DCT-II basis, row u = basis u (DCT.cpp:221-230).  Literal
// values, not cos(): they are slightly asymmetric and bit-exactness depends on
// them.
#define MYYUV_DCT_MATRIX                                                                       \
  {0.3535533845424652f,   0.3535533845424652f,  0.3535533845424652f,  0.3535533845424652f,   \
   0.3535533845424652f,   0.3535533845424652f,  0.3535533845424652f,  0.3535533845424652f,   \
   0.4903925955295563f,   0.4157347679138184f,  0.277785062789917f,   0.09754510968923569f,  \
   -0.09754515439271927f, -0.2777851521968842f, -0.4157347977161407f, -0.4903926253318787f,  \
   0.4619397222995758f,   0.1913416981697083f,  -0.1913417428731918f, -0.4619397819042206f,  \
   -0.4619397222995758f,  -0.1913415491580963f, 0.1913417875766754f,  0.4619397521018982f,   \
   0.4157347679138184f,   -0.09754515439271927f, -0.4903926253318787f, -0.2777849733829498f, \
   0.2777851819992065f,   0.4903925955295563f,  0.09754502773284912f, -0.4157348573207855f,  \
   0.3535533547401428f,   -0.3535533547401428f, -0.353553295135498f,  0.3535534739494324f,   \
   0.3535533547401428f,   -0.3535535931587219f, -0.3535532355308533f, 0.3535533845424652f,   \
   0.277785062789917f,    -0.4903926253318787f, 0.09754519909620285f, 0.4157346487045288f,   \
   -0.4157348573207855f,  -0.09754510223865509f, 0.4903926253318787f, -0.2777853906154633f,  \
   0.1913416981697083f,   -0.4619397222995758f, 0.4619397521018982f,  -0.1913419365882874f,  \
   -0.1913414746522903f,  0.4619396328926086f,  -0.4619398415088654f, 0.1913419365882874f,   \
   0.09754510968923569f,  -0.2777849733829498f, 0.4157346487045288f,  -0.4903925657272339f,  \
   0.4903926849365234f,   -0.4157347679138184f, 0.2777855396270752f,  -0.09754576534032822f}

#define MYYUV_ZIGZAG                                                                          \
  {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,    \
   41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,    \
   30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63}

// K2 block classes (k_huff_encode sorts a window's blocks by class so each
// wave runs the cheapest encoder that fits all its blocks):
//   single: msz <= 1, one symbol;  r4 / r8: at most 4 / 8 distinct symbols
//   for sure (nonzero coefficients, plus one for a zero inside the message);
//   r8x: up to kOvfNub - 1 such symbol slots, encode_block_r<8> with the
//   overflow worklist behind it;  ovf: kOvfNub or more, straight to the
//   overflow worklist (K2 builds nothing for them: of the bench frame's
//   blocks with 16 or more, 10 % fit 8 distinct symbols, and they carry the
//   longest messages: msz 23-50; the CAP-16 tier takes them whole).
// msz = 1 + zig-zag index of the last nonzero coefficient (0: all zero).
constexpr uint32_t kClassSingle = 0, kClassR4 = 1, kClassR8 = 2, kClassR8x = 3, kClassOvf = 4, kClassDead = 5;
#ifndef MYYUV_OVF_NUB
#define MYYUV_OVF_NUB 16  // (65: no block is of the ovf class)
#endif
constexpr uint32_t kOvfNub = MYYUV_OVF_NUB;
__host__ __device__ __forceinline__ uint32_t class_of(uint32_t nnz, uint32_t msz) {
  if (msz <= 1) return kClassSingle;
  const uint32_t nub = nnz + (msz > nnz ? 1u : 0u);
  return nub <= 4 ? kClassR4 : (nub <= 8 ? kClassR8 : (nub < kOvfNub ? kClassR8x : kClassOvf));
}
// Natural coefficient pair w (coefficients 2w, 2w+1): (zig-zag index + 1) of
// each, in the two 16-bit halves.
struct ZzPairs {
  uint32_t v[32];
  constexpr ZzPairs() : v{} {
    constexpr uint8_t zz[64] = MYYUV_ZIGZAG;
    uint32_t inv[64] = {};
    for (int i = 0; i < 64; i++) inv[zz[i]] = (uint32_t)i + 1u;
    for (int w = 0; w < 32; w++) v[w] = inv[2 * w] | (inv[2 * w + 1] << 16);
  }
};
constexpr ZzPairs kZzPairs{};
// K1 -> K2 per-block word (binfo): bits 0-7 the row mask, 8-14 msz, 15-17 the
// class, 18-28 the DC coefficient's low 11 bits (all K2's classification
// needs: it reads 4 B per block instead of the coefficient rows).
__host__ __device__ __forceinline__ uint32_t binfo_word(uint32_t rm, uint32_t msz, uint32_t cls, uint32_t dc) {
  return rm | (msz << 8) | (cls << 15) | ((dc & 0x7FFu) << 18);
}

// Geometry of one IYUV frame as the kernels see it.  Blocks are numbered
// globally plane-major (Y, U, V), row-major inside a plane, which is the
// reference's block order k = (y/8)*(w/8) + x/8 per plane (DCT.cpp:308, 355)
// concatenated over planes.
struct FrameGeom {
  uint32_t pw[3], ph[3];  // plane width / height in pixels
  uint32_t bw[3];         // blocks per block-row
  uint32_t cum[4];        // cumulative block counts: plane p owns [cum[p], cum[p+1])
  uint32_t poff[3];       // byte offset of plane p in the IYUV frame
  uint32_t ucum[4];       // transform units (kXfUnit blocks of one plane) per plane, cumulative
  uint64_t bmag[3];       // ceil(2^64 / bw[p]) (0 for bw = 1): block_row() divides by it
  // A batch of `nframes` frames of this geometry, frame f at byte f * fbytes
  // of the frame buffer; its blocks are numbered f * cum[3] + g (batch-global)
  // in the coefficient, slot and size buffers.
  uint32_t nframes;
  uint32_t fbytes;        // W * H * 3 / 2
  uint64_t umag;          // ceil(2^64 / ucum[3]) (0 for 1 unit): batch unit -> frame
  // K2 / K4 tiles: kK2Group consecutive blocks of one plane (the last tile of
  // a plane may be shorter), cumulative per plane; tile t of frame f is
  // batch tile f * tcum[3] + t
  uint32_t tcum[4];
  // index of frame 0 of this launch in the caller's batch (a batch whose
  // coefficient image would reach 4 GiB runs as several launches, kMaxLaunchBlocks):
  // only the error keys use it, which name batch-global blocks
  uint32_t fbase;
};
// Blocks per launch: the coefficient image (128 B per block, in 64-block
// groups) stays below 4 GiB, the range of the kernels' 32-bit buffer offsets.
constexpr uint32_t kMaxLaunchBlocks = (1u << 25) - 64u;

// floor(x / d) for a 32-bit x from m = ceil(2^64 / d) (m = 0 for d = 1): the
// product overshoots x / d by less than x / 2^64, below the 1 / d slack.
__host__ __device__ __forceinline__ uint32_t div_magic(uint32_t x, uint64_t m) {
  if (m == 0) return x;
  const uint64_t lo = (uint64_t)x * (uint32_t)m;
  const uint64_t hi = (uint64_t)x * (uint32_t)(m >> 32) + (lo >> 32);
  return (uint32_t)(hi >> 32);
}

// by = floor(local / bw) = high 64 bits of local * ceil(2^64 / bw): the
// product overshoots local / bw by less than local / 2^64, below the 1 / bw
// slack, so the floor is exact for every 32-bit local.
__host__ __device__ __forceinline__ uint32_t block_row(const FrameGeom& G, int p, uint32_t local) {
  return div_magic(local, G.bmag[p]);
}

// Per-quality tables (a device buffer; K1/K6 stage q and r into LDS).
struct QTables {
  float q[3][64];     // natural order, DCT.cpp:286-290
  float r[3][64];     // 1.0f / q, correctly rounded (K1's division-free fast path)
  float kb[3][8];     // K1's fast-path bound per row (fdct_bfly.h bfly_row_bounds)
};

// K1's near-tie window per unit of |t| (k_transform.hip): t = y * fl(1/Q)
// may differ from fl(y / Q) by |t| * 1.5 * 2^-23; 2^-21 covers it with margin
// (tools/check_numerics.c checks every Q at every tie; 2^-24 already fails).
constexpr float kNearRel = 0x1p-21f;

// Coefficient layout shared by K1, K2, K5 and K6: per block 64 int16 in
// NATURAL (row-major) order, word w = coefficients 2w, 2w+1; words grouped in
// quads (16 B) and the quads of 64 consecutive blocks interleaved, so that
//   quad c (words 4c..4c+3, i.e. row c/2's half) of block g is uint4 element
//   ((g >> 6) * 8 + c) * 64 + (g & 63).
// A lane-per-block wave reads one quad of 64 blocks as 1 KiB contiguous; K1/K6
// (four lanes per block, two rows each) write/read 256 B runs.  The zig-zag
// scan is a fixed permutation applied with static register indices where the
// coefficients are consumed (K2) or produced (K5).
constexpr uint32_t kCoefQuadsPerWave = 8 * 64;

// K2 overflow worklists up to this many blocks are encoded wave-per-block
// (k_huff_encode_wave), longer ones lane-per-block (k_huff_encode_wide).
#ifndef MYYUV_WAVE_LIMIT
#define MYYUV_WAVE_LIMIT 24576
#endif
constexpr uint32_t kWaveEncodeLimit = MYYUV_WAVE_LIMIT;
#ifndef MYYUV_BATCH_WAVE_LIMIT
#define MYYUV_BATCH_WAVE_LIMIT 0
#endif
constexpr uint32_t kBatchWaveLimit = MYYUV_BATCH_WAVE_LIMIT;  // the same limit for batches (nframes > 1)
constexpr uint32_t kWaveEncodeGrid = 8192;   // waves of k_huff_encode_wave (grid-stride)
#ifndef MYYUV_WIDE_LANES
#define MYYUV_WIDE_LANES 64
#endif
constexpr uint32_t kWideLanes = MYYUV_WIDE_LANES;  // blocks (lanes) per workgroup of k_huff_encode_wide
#ifndef MYYUV_WIDE_GRID
#define MYYUV_WIDE_GRID (1280 * 64 / MYYUV_WIDE_LANES)
#endif
constexpr uint32_t kWideGrid = MYYUV_WIDE_GRID;  // workgroups of k_huff_encode_wide: its LDS fits 5 x 64 lanes per CU
// Overflow lists longer than one resident round of k_huff_encode_wide (its
// grid x lanes) go through the CAP-16 register tier first
// (k_huff_encode_r16, huff_r16.hpp); it lists the blocks with more than 16
// distinct symbols again (work2) for the wave / lane passes.  Shorter lists
// skip it: one CAP-64 round takes the whole list, and there the extra pass
// measured slower (profiles/r3g_*).
#ifndef MYYUV_R16_GATE
#define MYYUV_R16_GATE (MYYUV_WIDE_GRID * MYYUV_WIDE_LANES)
#endif
constexpr uint32_t kR16Gate = MYYUV_R16_GATE;
// Single frames: past two rounds of k_huff_encode_wave (a wave per block,
// ~25 us a round), the tier and then the wave pass over what it leaves
// (8192^2 q50: 55 + 26 us against 94 us in one CAP-64 lane round;
// chef-big q90: 50 + 35 against 98 us in the wave pass; profiles/r6n_*).
#ifndef MYYUV_R16_GATE_SINGLE
#define MYYUV_R16_GATE_SINGLE (2 * 8192)
#endif
constexpr uint32_t kR16GateSingle = MYYUV_R16_GATE_SINGLE;
constexpr uint32_t kR16Grid = 4096;  // workgroups of k_huff_encode_r16 (grid-stride, 64 blocks each)
#ifndef MYYUV_K2_GROUP
#define MYYUV_K2_GROUP 256
#endif
constexpr uint32_t kK2Group = MYYUV_K2_GROUP;  // blocks per workgroup of k_huff_encode
__host__ __device__ __forceinline__ uint32_t coef_quad(uint32_t g, uint32_t c) {
  return ((g >> 6) * 8u + c) * 64u + (g & 63u);
}

// K2 works on windows of kWinTiles consecutive batch tiles (window w = batch
// tiles [w * kWinTiles, (w + 1) * kWinTiles)): one workgroup classifies the
// window's blocks and sorts them by class over the whole window, so its 64-block
// runs are more uniform than a single tile's would be.
#ifndef MYYUV_K2_WIN
#define MYYUV_K2_WIN 4
#endif
constexpr uint32_t kWinTiles = MYYUV_K2_WIN;
static_assert((kWinTiles & (kWinTiles - 1)) == 0 && kWinTiles >= 1 && kWinTiles <= 8, "kWinTiles: 1, 2, 4 or 8");
// Launches of at least kWinBigTiles batch tiles (the bench's 24-frame groups:
// 26.6k) use windows of kWinTilesBig tiles: twice the runs per workgroup
// share one classification and sort (bench +1.25 %), while smaller launches
// (a single 8192x8192 frame: 6,144 tiles) keep kWinTiles, whose grid fills
// the chip (K2 there 72 against 100 us with 8-tile windows, profiles/r5ba_*).
// K2 and K4 of one launch use the same window (k2_win), the fused encoder
// kWinTiles.
#ifndef MYYUV_K2_WIN_BIG
#define MYYUV_K2_WIN_BIG 8
#endif
#ifndef MYYUV_K2_WIN_BIG_TILES
#define MYYUV_K2_WIN_BIG_TILES 16384
#endif
constexpr uint32_t kWinTilesBig = MYYUV_K2_WIN_BIG;
constexpr uint32_t kWinBigTiles = MYYUV_K2_WIN_BIG_TILES;
static_assert((kWinTilesBig & (kWinTilesBig - 1)) == 0 && kWinTilesBig >= kWinTiles && kWinTilesBig <= 8,
              "kWinTilesBig: a power of two, kWinTiles .. 8");
__host__ __device__ __forceinline__ uint32_t k2_win(uint32_t ntiles) {
  return ntiles >= kWinBigTiles ? kWinTilesBig : kWinTiles;
}
__host__ __device__ __forceinline__ uint32_t win_first_tile(uint32_t T, uint32_t W) { return T & ~(W - 1u); }

// K2 -> K4 hand-off, per window of batch tiles:
//   stage:  kTileCap bytes per batch tile (the window's tiles' regions are
//           contiguous), one kWaveRun-byte region per 64-block run: the chunks
//           of the run's blocks with at most 8 distinct symbols, back to back
//           in the run's (class-sorted) order (a "dense run");
//   srcoff: u32 per block: the chunk's byte offset from its window's first
//           tile's stage region, kSrcOverflow for a block with more symbols,
//           whose chunk the overflow passes write to oslots at g * kMaxChunk;
//   tinfo:  kTInfoWords u32 per tile: [0] overflow chunk bytes (the overflow
//           passes add to it), [1 .. 4] the tile's dense-chunk bytes (k_huff_encode:
//           all in [1]; k_encode_tile: per wave), [8] the tile's exclusive
//           prefix in its frame's content (k_tile_scan).
constexpr uint32_t kTileCap = kK2Group * kMaxChunk;
constexpr uint32_t kWaveRun = kWave * kMaxChunk;
constexpr uint32_t kTInfoWords = 16;
constexpr uint32_t kTInfoPrefix = 8;
constexpr uint32_t kSrcOverflow = 0xFFFFFFFFu;
// The hand-off is laid out for exactly four K2 waves per tile: k_tile_scan sums
// tinfo words 1..4, k_stream_out keeps four run totals, k_encode_tile's
// phase 1 covers 4 waves x 4 units x 16 blocks, and tinfo word kTInfoPrefix
// must lie past the run words.
static_assert(kK2Group == 4 * kWave, "the K2 -> K4 hand-off assumes 4 waves per tile");
static_assert(1 + kK2Group / kWave <= kTInfoPrefix, "tinfo run words overlap the tile prefix");

// Batch tiles rounded up to whole windows (the stage buffer's extent).
__host__ __device__ __forceinline__ uint32_t win_tiles_alloc(uint32_t ntiles) {
  return (ntiles + kWinTilesBig - 1u) & ~(kWinTilesBig - 1u);
}

// Plane, first block (frame-local) and block count of tile t of a frame.
__host__ __device__ __forceinline__ int tile_plane(const FrameGeom& G, uint32_t t) {
  return t >= G.tcum[1] ? (t >= G.tcum[2] ? 2 : 1) : 0;
}
__host__ __device__ __forceinline__ uint32_t tile_first(const FrameGeom& G, int p, uint32_t t) {
  return G.cum[p] + (t - G.tcum[p]) * kK2Group;
}
// Batch tile of batch-global block g.
__host__ __device__ __forceinline__ uint32_t tile_of_block(const FrameGeom& G, uint32_t g) {
  const uint32_t f = G.nframes > 1 ? g / G.cum[3] : 0u;
  const uint32_t l = g - f * G.cum[3];
  const int p = l >= G.cum[1] ? (l >= G.cum[2] ? 2 : 1) : 0;
  return f * G.tcum[3] + G.tcum[p] + (l - G.cum[p]) / kK2Group;
}

// list c of K1's unproven blocks (see fix_count)
__host__ __device__ __forceinline__ uint32_t* fix_list(uint32_t* fix, const FrameGeom& G, uint32_t c) {
  return fix + kFixHeader + (size_t)c * fix_list_cap(G.ucum[3] * G.nframes);
}

}  // namespace myyuv_gpu
