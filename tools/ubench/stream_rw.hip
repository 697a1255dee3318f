// Reference streaming rates for K1's byte shape: read N bytes, write 2N bytes
// (N = 18,192,384, the 4032x3008 IYUV frame), 16 B per lane, one pass, timed
// with events around each launch (as the codec's kernel stats are).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void k_rw(const uint4* __restrict__ in, uint4* __restrict__ out, uint32_t n16) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n16) {
    const uint4 v = in[i];
    out[2 * i] = v;
    out[2 * i + 1] = make_uint4(v.y, v.z, v.w, v.x);
  }
}
// same bytes, 8 B per lane
__global__ __launch_bounds__(256) void k_rw8(const uint2* __restrict__ in, uint2* __restrict__ out, uint32_t n8) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n8) {
    const uint2 v = in[i];
    out[2 * i] = v;
    out[2 * i + 1] = make_uint2(v.y, v.x);
  }
}
__global__ __launch_bounds__(256) void k_empty(uint32_t* out) {
  if (threadIdx.x == 1024) out[0] = 1;
}

int main() {
  const size_t N = 18192384;
  void *in, *out;
  (void)hipMalloc(&in, N);
  (void)hipMalloc(&out, 2 * N);
  (void)hipMemset(in, 1, N);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int k = 0; k < 3; k++) {
    float best = 1e9, sum = 0;
    for (int rep = 0; rep < 20; rep++) {
      (void)hipEventRecord(e0);
      if (k == 0) k_rw<<<(N / 16 + 255) / 256, 256>>>((const uint4*)in, (uint4*)out, N / 16);
      if (k == 1) k_rw8<<<(N / 8 + 255) / 256, 256>>>((const uint2*)in, (uint2*)out, N / 8);
      if (k == 2) k_empty<<<4443, 256>>>((uint32_t*)out);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep >= 2) sum += ms;
      if (ms < best) best = ms;
    }
    printf("%-28s best %.2f us  mean %.2f us  -> %.2f TB/s (best)\n",
           k == 0 ? "read N + write 2N, 16 B/lane" : k == 1 ? "read N + write 2N, 8 B/lane" : "empty 4443 x 256 grid",
           best * 1e3, sum / 18 * 1e3, k == 2 ? 0.0 : 3.0 * N / (best * 1e-3) / 1e12);
  }
  return 0;
}
