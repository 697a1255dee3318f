// Microbenchmark: issue rate of independent f32 VALU ops on gfx950, scalar
// (v_mul_f32/v_add_f32) vs packed (v_pk_mul_f32/v_pk_add_f32), at several
// waves per SIMD.  Prints ns per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

template <int W>
__global__ __launch_bounds__(64) void k_scalar(float* out, float a, float b, int iters) {
  float v[16];
#pragma unroll
  for (int i = 0; i < 16; i++) v[i] = threadIdx.x * 0.001f + i;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = v[i] * a + b;  // contract off: mul + add
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) s += v[i];
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

__global__ __launch_bounds__(64) void k_packed(float* out, float a, float b, int iters) {
  f2 v[8];
#pragma unroll
  for (int i = 0; i < 8; i++) v[i] = f2{threadIdx.x * 0.001f + i, threadIdx.x * 0.002f + i};
  const f2 a2 = {a, a}, b2 = {b, b};
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = v[i] * a2 + b2;
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s += v[i].x + v[i].y;
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

int main() {
  float* out;
  hipMalloc(&out, 1 << 24);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 4096;
  for (int wps : {1, 2, 4, 8}) {
    const int grid = 1024 * wps;  // 256 CUs x 4 SIMDs
    for (int pk = 0; pk < 2; pk++) {
      float best = 1e9;
      for (int rep = 0; rep < 3; rep++) {
        hipEventRecord(e0);
        if (pk) k_packed<<<grid, 64>>>(out, 0.999f, 0.001f, iters);
        else k_scalar<1><<<grid, 64>>>(out, 0.999f, 0.001f, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      // instructions per wave: scalar 32 per iter (16 mul + 16 add), packed 16 per iter
      const double insts = (double)iters * (pk ? 16 : 32) * wps;  // per SIMD
      const double ops = (double)iters * 32 * wps;                   // f32 ops per lane per SIMD
      printf("waves/SIMD %d %s: %.3f ms, %.3f ns/inst/SIMD, %.3f ns per 64-lane op-pair\n", wps,
             pk ? "packed" : "scalar", best, best * 1e6 / insts, best * 1e6 / ops);
    }
  }
  return 0;
}
