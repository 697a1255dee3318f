// The transform's stage-1 instruction stream in isolation: per k, 2 byte->f32
// conversions, 16 v_mul_f32 by literals, 16 v_add_f32 into 16 accumulators.
// Grid and block shape as K1 (4443 x 256), iterated to amplify.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr float D[64] = {0.3535533845424652f,   0.3535533845424652f,  0.3535533845424652f,  0.3535533845424652f,
   0.3535533845424652f,   0.3535533845424652f,  0.3535533845424652f,  0.3535533845424652f,
   0.4903925955295563f,   0.4157347679138184f,  0.277785062789917f,   0.09754510968923569f,
   -0.09754515439271927f, -0.2777851521968842f, -0.4157347977161407f, -0.4903926253318787f,
   0.4619397222995758f,   0.1913416981697083f,  -0.1913417428731918f, -0.4619397819042206f,
   -0.4619397222995758f,  -0.1913415491580963f, 0.1913417875766754f,  0.4619397521018982f,
   0.4157347679138184f,   -0.09754515439271927f, -0.4903926253318787f, -0.2777849733829498f,
   0.2777851819992065f,   0.4903925955295563f,  0.09754502773284912f, -0.4157348573207855f,
   0.3535533547401428f,   -0.3535533547401428f, -0.353553295135498f,  0.3535534739494324f,
   0.3535533547401428f,   -0.3535535931587219f, -0.3535532355308533f, 0.3535533845424652f,
   0.277785062789917f,    -0.4903926253318787f, 0.09754519909620285f, 0.4157346487045288f,
   -0.4157348573207855f,  -0.09754510223865509f, 0.4903926253318787f, -0.2777853906154633f,
   0.1913416981697083f,   -0.4619397222995758f, 0.4619397521018982f,  -0.1913419365882874f,
   -0.1913414746522903f,  0.4619396328926086f,  -0.4619398415088654f, 0.1913419365882874f,
   0.09754510968923569f,  -0.2777849733829498f, 0.4157346487045288f,  -0.4903925657272339f,
   0.4903926849365234f,   -0.4157347679138184f, 0.2777855396270752f,  -0.09754576534032822f};

__device__ __forceinline__ void fence16(float (&a)[16]) {
  asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
               "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]),
               "+v"(a[12]), "+v"(a[13]), "+v"(a[14]), "+v"(a[15]));
}

template <int BS>
__global__ __launch_bounds__(BS) void k_stage(float* out, uint32_t seed, int reps) {
  uint32_t xr = (blockIdx.x * BS + threadIdx.x) * 2654435761u ^ seed;
  float T[16];
#pragma unroll
  for (int j = 0; j < 16; j++) T[j] = 0.0f;
  for (int r = 0; r < reps; r++) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const float x0 = (float)(int)(int8_t)(xr >> (8 * (k & 3)));
      const float x1 = (float)(int)(int8_t)(xr >> (8 * ((k + 1) & 3)));
      float pr[16];
#pragma unroll
      for (int i = 0; i < 8; i++) {
        pr[2 * i] = D[i * 8 + k] * x0;
        pr[2 * i + 1] = D[i * 8 + k] * x1;
      }
#pragma unroll
      for (int j = 0; j < 16; j++) T[j] = T[j] + pr[j];
      fence16(T);
    }
    xr = xr * 1664525u + 1013904223u;
  }
  float s = 0;
#pragma unroll
  for (int j = 0; j < 16; j++) s += T[j];
  out[blockIdx.x * BS + threadIdx.x] = s;
}

int main() {
  float* out;
  (void)hipMalloc(&out, 4443 * 256 * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int reps : {1, 8, 64}) {
    for (int bs : {64, 256}) {
      const int grid = 4443 * 256 / bs;
      float best = 1e9;
      for (int rep = 0; rep < 5; rep++) {
        if (bs == 64) hipExtLaunchKernelGGL(k_stage<64>, dim3(grid), dim3(64), 0, 0, e0, e1, 0, out, 7u, reps);
        else hipExtLaunchKernelGGL(k_stage<256>, dim3(grid), dim3(256), 0, 0, e0, e1, 0, out, 7u, reps);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      // per wave per rep: 8 x (16 mul + 16 add + ~3 cvt/shift) ~ 280 VALU
      const double waves_per_simd = 4443.0 * 256 / 64 / 1024;
      printf("reps %2d block %3d: %8.2f us  (%.3f ns per VALU per SIMD, ~280 VALU/wave/rep)\n", reps, bs,
             best * 1e3, best * 1e6 / (waves_per_simd * 280.0 * reps));
    }
  }
  return 0;
}
