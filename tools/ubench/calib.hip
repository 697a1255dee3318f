// FETCH_SIZE / WRITE_SIZE calibration for the codec's own access shapes
// (MI355X_MICROARCH.md §HBM: only 16-B-per-lane streams are calibrated by the
// guide).  Each kernel moves a known number of bytes with the addressing of
// one codec kernel, over buffers larger than the 256 MiB Infinity Cache:
//   k1_read   K1's pixel loads: lane (b, q) of a 16-block unit reads rows 2q,
//             2q+1 of block b, 8 B each (128-B runs per row)
//   k1_write  K1's coefficient stores: quads 2q, 2q+1 of block b, 16 B each, in
//             the block-interleaved quad layout (256-B runs)
//   k6_read   K6's coefficient loads (the same quads, read)
//   k6_write  K6's pixel stores (the same rows, written)
//   k2_scatter_read  K2's run loads (round 4): per 1024-block window (4 K2
//             tiles), lanes take the window's blocks in a scattered order (a
//             bijection standing in for the class sort) and load all 8 quads
//             of their block, 16 B per lane per load: every quad read once
//   k2_dc_read  K2's single-class runs: the DC word (4 B) of quad 0 of every
//             block, scattered the same way (line coverage: the quad-0 region)
//   k2_twophase_read  K2's whole read pattern: the window's quads coalesced
//             (classify), a workgroup barrier, then the scattered run loads
//             again, at K2's occupancy (5 workgroups of 256 per CU); known
//             bytes = the buffer once, so factor ~0.5 x the scatter factor
//             means the run loads miss L2 (the buffer is read twice)
//   k4_gather_read  K4's chunk loads: 12-B chunks packed back to back in
//             1024-chunk windows, lanes of a 256-lane tile read their chunk's
//             dwords (a 1-4 word gather) in a scattered order within the window
// Run under `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` (separate
// passes); tools/calib_report.py divides the counters by the printed bytes.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

namespace {
constexpr uint32_t W = 8192, H = 40960;  // 320 MiB of pixels, 640 MiB of coefficients
constexpr uint32_t BW = W / 8, NB = (W / 8) * (H / 8), NU = NB / 16;

__device__ __forceinline__ uint32_t coef_quad(uint32_t g, uint32_t c) { return ((g >> 6) * 8u + c) * 64u + (g & 63u); }
__device__ __forceinline__ uint32_t row_off(uint32_t g, uint32_t r) {
  const uint32_t by = g / BW, bx = g - by * BW;
  return (by * 8u + r) * W + bx * 8u;
}

__global__ __launch_bounds__(256) void k1_read(const uint8_t* __restrict__ px, uint32_t* __restrict__ sink) {
  const uint32_t lane = threadIdx.x & 63u, q = lane & 3u, b = lane >> 2;
  const uint32_t u = blockIdx.x * 4u + (threadIdx.x >> 6);
  if (u >= NU) return;
  const uint32_t g = u * 16u + b, off = row_off(g, 2u * q);
  const uint2 r0 = *reinterpret_cast<const uint2*>(px + off);
  const uint2 r1 = *reinterpret_cast<const uint2*>(px + off + W);
  const uint32_t x = r0.x ^ r0.y ^ r1.x ^ r1.y;
  if (x == 0x9e3779b9u) sink[lane] = x;  // never: keeps the loads
}

__global__ __launch_bounds__(256) void k1_write(uint4* __restrict__ coef) {
  const uint32_t lane = threadIdx.x & 63u, q = lane & 3u, b = lane >> 2;
  const uint32_t u = blockIdx.x * 4u + (threadIdx.x >> 6);
  if (u >= NU) return;
  const uint32_t g = u * 16u + b;
  coef[coef_quad(g, 2u * q)] = make_uint4(g, q, 1u, 2u);
  coef[coef_quad(g, 2u * q + 1u)] = make_uint4(g, q, 3u, 4u);
}

__global__ __launch_bounds__(256) void k6_read(const uint4* __restrict__ coef, uint32_t* __restrict__ sink) {
  const uint32_t lane = threadIdx.x & 63u, q = lane & 3u, b = lane >> 2;
  const uint32_t u = blockIdx.x * 4u + (threadIdx.x >> 6);
  if (u >= NU) return;
  const uint32_t g = u * 16u + b;
  const uint4 a = coef[coef_quad(g, 2u * q)], c = coef[coef_quad(g, 2u * q + 1u)];
  const uint32_t x = a.x ^ a.y ^ a.z ^ a.w ^ c.x ^ c.y ^ c.z ^ c.w;
  if (x == 0x9e3779b9u) sink[lane] = x;
}

// the window slot of sorted position e (a bijection on 0..1023 standing in
// for K2's class sort)
__device__ __forceinline__ uint32_t scat(uint32_t e) { return (e * 617u + 129u) & 1023u; }

__global__ __launch_bounds__(256) void k2_scatter_read(const uint4* __restrict__ coef, uint32_t* __restrict__ sink) {
  const uint32_t tid = threadIdx.x;
  uint32_t x = 0;
  for (uint32_t r = 0; r < 4; r++) {
    const uint32_t g = blockIdx.x * 1024u + scat(r * 256u + tid);
#pragma unroll
    for (uint32_t c = 0; c < 8; c++) {
      const uint4 a = coef[coef_quad(g, c)];
      x ^= a.x ^ a.y ^ a.z ^ a.w;
    }
  }
  if (x == 0x9e3779b9u) sink[tid & 63u] = x;
}

__global__ __launch_bounds__(256) void k2_dc_read(const uint4* __restrict__ coef, uint32_t* __restrict__ sink) {
  const uint32_t tid = threadIdx.x;
  uint32_t x = 0;
  for (uint32_t r = 0; r < 4; r++) {
    const uint32_t g = blockIdx.x * 1024u + scat(r * 256u + tid);
    x ^= reinterpret_cast<const uint32_t*>(coef)[coef_quad(g, 0) * 4u];
  }
  if (x == 0x9e3779b9u) sink[tid & 63u] = x;
}

__global__ __launch_bounds__(256, 5) void k2_twophase_read(const uint4* __restrict__ coef, uint32_t* __restrict__ sink) {
  const uint32_t tid = threadIdx.x;
  uint32_t x = 0;
  for (uint32_t r = 0; r < 4; r++) {  // classify: block tid of each tile, coalesced
    const uint32_t g = blockIdx.x * 1024u + r * 256u + tid;
#pragma unroll
    for (uint32_t c = 0; c < 8; c++) {
      const uint4 a = coef[coef_quad(g, c)];
      x += a.x ^ a.y ^ a.z ^ a.w;
    }
  }
  __syncthreads();
  for (uint32_t r = 0; r < 4; r++) {  // runs: scattered
    const uint32_t g = blockIdx.x * 1024u + scat(r * 256u + tid);
#pragma unroll
    for (uint32_t c = 0; c < 8; c++) {
      const uint4 a = coef[coef_quad(g, c)];
      x ^= a.x ^ a.y ^ a.z ^ a.w;
    }
  }
  if (x == 0x9e3779b9u) sink[tid & 63u] = x;
}

// K4: chunk k of a window (12 B, back to back) read by lane scat(k)
__global__ __launch_bounds__(256) void k4_gather_read(const uint32_t* __restrict__ stage, uint32_t* __restrict__ sink) {
  const uint32_t tid = threadIdx.x;
  uint32_t x = 0;
  for (uint32_t r = 0; r < 4; r++) {
    const uint32_t k = scat(r * 256u + tid);
    const uint32_t b0 = (blockIdx.x * 1024u + k) * 12u;  // byte offset
    const uint32_t w0 = b0 >> 2, nw = ((b0 & 3u) + 12u + 3u) >> 2;
    for (uint32_t i = 0; i < nw; i++) x ^= stage[w0 + i];
  }
  if (x == 0x9e3779b9u) sink[tid & 63u] = x;
}

__global__ __launch_bounds__(256) void k6_write(uint8_t* __restrict__ px) {
  const uint32_t lane = threadIdx.x & 63u, q = lane & 3u, b = lane >> 2;
  const uint32_t u = blockIdx.x * 4u + (threadIdx.x >> 6);
  if (u >= NU) return;
  const uint32_t g = u * 16u + b, off = row_off(g, 2u * q);
  *reinterpret_cast<uint2*>(px + off) = make_uint2(g, q);
  *reinterpret_cast<uint2*>(px + off + W) = make_uint2(q, g);
}
}  // namespace

int main() {
  const size_t pbytes = (size_t)W * H, cbytes = 2 * pbytes;
  uint8_t* px = nullptr;
  uint4* coef = nullptr;
  uint32_t* sink = nullptr;
  if (hipMalloc(&px, pbytes) != hipSuccess || hipMalloc(&coef, cbytes) != hipSuccess ||
      hipMalloc(&sink, 256) != hipSuccess)
    return 1;
  (void)hipMemset(px, 1, pbytes);
  (void)hipMemset(coef, 2, cbytes);
  const dim3 grid(NU / 4), block(256);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[8] = {"k1_read", "k1_write", "k6_read", "k6_write",
                          "k2_scatter_read", "k2_dc_read", "k2_twophase_read", "k4_gather_read"};
  // k2_dc_read: line coverage of the quad-0 region (NB x 16 B); k4: NB x 12 B of chunks
  const double bytes[8] = {(double)pbytes, (double)cbytes, (double)cbytes, (double)pbytes,
                           (double)cbytes, (double)NB * 16, (double)cbytes, (double)NB * 12};
  const dim3 gwin(NB / 1024);
  for (int k = 0; k < 8; k++) {
    float best = 1e9f;
    for (int rep = 0; rep < 3; rep++) {
      (void)hipEventRecord(e0);
      if (k == 0) k1_read<<<grid, block>>>(px, sink);
      if (k == 1) k1_write<<<grid, block>>>(coef);
      if (k == 2) k6_read<<<grid, block>>>(coef, sink);
      if (k == 3) k6_write<<<grid, block>>>(px);
      if (k == 4) k2_scatter_read<<<gwin, block>>>(coef, sink);
      if (k == 5) k2_dc_read<<<gwin, block>>>(coef, sink);
      if (k == 6) k2_twophase_read<<<gwin, block>>>(coef, sink);
      if (k == 7) k4_gather_read<<<gwin, block>>>(reinterpret_cast<const uint32_t*>(px), sink);
      (void)hipEventRecord(e1);
      if (hipEventSynchronize(e1) != hipSuccess) return 2;
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    printf("{\"kernel\": \"%s\", \"bytes_per_launch\": %.0f, \"best_us\": %.2f, \"TBps\": %.3f}\n", names[k],
           bytes[k], best * 1e3, bytes[k] / (best * 1e-3) / 1e12);
  }
  return 0;
}
