// Checks the DPP wave helpers of codec_common.hpp (wave_incl_add,
// wave_max_nonneg) and K1's quad_perm exchange against a host computation
// on random data.  hipcc --offload-arch=gfx950 -O3 -std=c++17 -I yuv-manipulations-2_amd/csrc
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "codec_common.hpp"

using namespace myyuv_gpu;

__global__ void k(const uint32_t* in, uint32_t* scan, uint32_t* mx, uint32_t* quad) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t v = in[i];
  scan[i] = wave_incl_add(v);
  mx[i] = (uint32_t)wave_max_nonneg((int)(v & 0xFFFF));
  uint32_t rm = 1u << (threadIdx.x & 3u);
  rm |= (uint32_t)__builtin_amdgcn_mov_dpp((int)rm, 0xB1, 0xF, 0xF, false);
  rm |= (uint32_t)__builtin_amdgcn_mov_dpp((int)rm, 0x4E, 0xF, 0xF, false);
  quad[i] = rm | ((v & 0xF0u) << 4);
}

int main() {
  const int n = 256 * 64;
  std::vector<uint32_t> h(n), s(n), m(n), q(n);
  srand(5);
  for (auto& x : h) x = (uint32_t)rand() & 0xFFFFF;
  uint32_t *d_in, *d_s, *d_m, *d_q;
  hipMalloc(&d_in, n * 4); hipMalloc(&d_s, n * 4); hipMalloc(&d_m, n * 4); hipMalloc(&d_q, n * 4);
  hipMemcpy(d_in, h.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, d_in, d_s, d_m, d_q);
  hipMemcpy(s.data(), d_s, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(m.data(), d_m, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(q.data(), d_q, n * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int w = 0; w < n / 64; w++) {
    uint32_t acc = 0, mm = 0;
    for (int l = 0; l < 64; l++) mm = std::max(mm, h[w * 64 + l] & 0xFFFF);
    for (int l = 0; l < 64; l++) {
      acc += h[w * 64 + l];
      if (s[w * 64 + l] != acc) { if (bad++ < 5) printf("scan wave %d lane %d: %u != %u\n", w, l, s[w * 64 + l], acc); }
      if (m[w * 64 + l] != mm) { if (bad++ < 5) printf("max wave %d lane %d: %u != %u\n", w, l, m[w * 64 + l], mm); }
      if ((q[w * 64 + l] & 0xF) != 0xF) { if (bad++ < 5) printf("quad wave %d lane %d: %x\n", w, l, q[w * 64 + l]); }
    }
  }
  printf("dpp_check: %s (%d mismatches)\n", bad ? "FAILED" : "ok", bad);
  return bad ? 1 : 0;
}
