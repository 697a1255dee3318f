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
  const char* names[4] = {"k1_read", "k1_write", "k6_read", "k6_write"};
  const double bytes[4] = {(double)pbytes, (double)cbytes, (double)cbytes, (double)pbytes};
  for (int k = 0; k < 4; k++) {
    float best = 1e9f;
    for (int rep = 0; rep < 3; rep++) {
      (void)hipEventRecord(e0);
      if (k == 0) k1_read<<<grid, block>>>(px, sink);
      if (k == 1) k1_write<<<grid, block>>>(coef);
      if (k == 2) k6_read<<<grid, block>>>(coef, sink);
      if (k == 3) k6_write<<<grid, block>>>(px);
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
