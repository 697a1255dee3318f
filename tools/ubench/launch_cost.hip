// Event-timed cost of a launch vs its grid size, and of a grid-stride copy
// with K1's byte shape at a few persistent grid sizes.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void k_empty(uint32_t* out) {
  if (threadIdx.x == 1024) out[0] = 1;
}
__global__ __launch_bounds__(256) void k_rw8s(const uint2* __restrict__ in, uint2* __restrict__ out, uint32_t n8) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n8; i += gridDim.x * 256) {
    const uint2 v = in[i];
    out[2 * i] = v;
    out[2 * i + 1] = make_uint2(v.y, v.x);
  }
}

// dispatch-stamped (hipExtLaunchKernel) timing of a launch
template <class K, class... A>
float time_ext(K k, int grid, A... a) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e9;
  for (int rep = 0; rep < 20; rep++) {
    hipExtLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, e0, e1, 0, a...);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  return best * 1e3f;
}

template <class F>
float time_it(F f) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e9;
  for (int rep = 0; rep < 20; rep++) {
    (void)hipEventRecord(e0);
    f();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  return best * 1e3f;
}

int main() {
  const size_t N = 18192384;
  void *in, *out;
  (void)hipMalloc(&in, N);
  (void)hipMalloc(&out, 2 * N);
  (void)hipMemset(in, 1, N);
  for (int g : {1, 256, 1024, 2048, 4443, 8886, 17772})
    printf("empty grid %5d x 256: %.2f us\n", g, time_it([&] { k_empty<<<g, 256>>>((uint32_t*)out); }));
  for (int g : {512, 1024, 2048, 3072, 4096, 8886})
    printf("copy (8 B/lane, grid-stride) grid %5d: %.2f us -> %.2f TB/s\n", g,
           time_it([&] { k_rw8s<<<g, 256>>>((const uint2*)in, (uint2*)out, N / 8); }),
           3.0 * N / (time_it([&] { k_rw8s<<<g, 256>>>((const uint2*)in, (uint2*)out, N / 8); }) * 1e-6) / 1e12);
  for (int g : {1, 4443})
    printf("[ext] empty grid %5d x 256: %.2f us\n", g, time_ext(k_empty, g, (uint32_t*)out));
  for (int g : {1024, 2048, 8886}) {
    const float us = time_ext(k_rw8s, g, (const uint2*)in, (uint2*)out, (uint32_t)(N / 8));
    printf("[ext] copy (8 B/lane, grid-stride) grid %5d: %.2f us -> %.2f TB/s\n", g, us, 3.0 * N / (us * 1e-6) / 1e12);
  }
  return 0;
}
