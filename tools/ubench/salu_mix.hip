// Microbenchmark: does re-materialising a constant with s_mov before each
// packed multiply (what the compiler emits for pk ops on literals) cost issue
// throughput?  A: 8 x (s_mov_b32 lit; v_pk_mul_f32 with that SGPR);
// B: 8 x v_pk_mul_f32 with SGPRs held across the loop.  Also C: scalar
// v_mul_f32 with a literal (VOP2) x 16 (same lane-ops as 8 pk).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(64) void kA(float* out, int iters) {
  float a0 = threadIdx.x, a1 = a0 + 1, b0 = a0 + 2, b1 = a0 + 3;
  for (int it = 0; it < iters; it++) {
    asm volatile(
        "s_mov_b32 s40, 0x3eb504f3\n v_pk_mul_f32 v[%0:%1], v[%0:%1], s[40:41] op_sel_hi:[1,0]\n"
        "s_mov_b32 s42, 0x3efb14bd\n v_pk_mul_f32 v[%2:%3], v[%2:%3], s[42:43] op_sel_hi:[1,0]\n"
        "s_mov_b32 s44, 0x3eec835d\n v_pk_mul_f32 v[%0:%1], v[%0:%1], s[44:45] op_sel_hi:[1,0]\n"
        "s_mov_b32 s46, 0x3ed4db30\n v_pk_mul_f32 v[%2:%3], v[%2:%3], s[46:47] op_sel_hi:[1,0]\n"
        "s_mov_b32 s40, 0x3e8e39d8\n v_pk_mul_f32 v[%0:%1], v[%0:%1], s[40:41] op_sel_hi:[1,0]\n"
        "s_mov_b32 s42, 0x3dc7c5bb\n v_pk_mul_f32 v[%2:%3], v[%2:%3], s[42:43] op_sel_hi:[1,0]\n"
        "s_mov_b32 s44, 0x3e43ef14\n v_pk_mul_f32 v[%0:%1], v[%0:%1], s[44:45] op_sel_hi:[1,0]\n"
        "s_mov_b32 s46, 0x3f000001\n v_pk_mul_f32 v[%2:%3], v[%2:%3], s[46:47] op_sel_hi:[1,0]\n"
        : : "n"(0), "n"(1), "n"(2), "n"(3) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "v0", "v1", "v2", "v3");
  }
  out[blockIdx.x * 64 + threadIdx.x] = a0 + a1 + b0 + b1;
}

__global__ __launch_bounds__(64) void kB(float* out, int iters) {
  asm volatile("s_mov_b32 s40, 0x3eb504f3\n s_mov_b32 s42, 0x3efb14bd\n s_mov_b32 s44, 0x3eec835d\n s_mov_b32 s46, 0x3ed4db30\n" ::: "s40", "s42", "s44", "s46");
  for (int it = 0; it < iters; it++) {
    asm volatile(
        "v_pk_mul_f32 v[0:1], v[0:1], s[40:41] op_sel_hi:[1,0]\n"
        "v_pk_mul_f32 v[2:3], v[2:3], s[42:43] op_sel_hi:[1,0]\n"
        "v_pk_mul_f32 v[0:1], v[0:1], s[44:45] op_sel_hi:[1,0]\n"
        "v_pk_mul_f32 v[2:3], v[2:3], s[46:47] op_sel_hi:[1,0]\n"
        "v_pk_mul_f32 v[0:1], v[0:1], s[40:41] op_sel_hi:[1,0]\n"
        "v_pk_mul_f32 v[2:3], v[2:3], s[42:43] op_sel_hi:[1,0]\n"
        "v_pk_mul_f32 v[0:1], v[0:1], s[44:45] op_sel_hi:[1,0]\n"
        "v_pk_mul_f32 v[2:3], v[2:3], s[46:47] op_sel_hi:[1,0]\n"
        ::: "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "v0", "v1", "v2", "v3");
  }
  out[blockIdx.x * 64 + threadIdx.x] = 1.0f;
}

__global__ __launch_bounds__(64) void kC(float* out, int iters) {
  for (int it = 0; it < iters; it++) {
    asm volatile(
        "v_mul_f32 v0, 0x3eb504f3, v0\n v_mul_f32 v1, 0x3eb504f3, v1\n"
        "v_mul_f32 v2, 0x3efb14bd, v2\n v_mul_f32 v3, 0x3efb14bd, v3\n"
        "v_mul_f32 v0, 0x3eec835d, v0\n v_mul_f32 v1, 0x3eec835d, v1\n"
        "v_mul_f32 v2, 0x3ed4db30, v2\n v_mul_f32 v3, 0x3ed4db30, v3\n"
        "v_mul_f32 v0, 0x3e8e39d8, v0\n v_mul_f32 v1, 0x3e8e39d8, v1\n"
        "v_mul_f32 v2, 0x3dc7c5bb, v2\n v_mul_f32 v3, 0x3dc7c5bb, v3\n"
        "v_mul_f32 v0, 0x3e43ef14, v0\n v_mul_f32 v1, 0x3e43ef14, v1\n"
        "v_mul_f32 v2, 0x3f000001, v2\n v_mul_f32 v3, 0x3f000001, v3\n"
        ::: "v0", "v1", "v2", "v3");
  }
  out[blockIdx.x * 64 + threadIdx.x] = 1.0f;
}

int main() {
  float* out;
  (void)hipMalloc(&out, 1 << 24);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int iters = 4096;
  for (int wps : {2, 4, 8}) {
    const int grid = 1024 * wps;
    for (int k = 0; k < 3; k++) {
      float best = 1e9;
      for (int rep = 0; rep < 3; rep++) {
        (void)hipEventRecord(e0);
        if (k == 0) kA<<<grid, 64>>>(out, iters);
        if (k == 1) kB<<<grid, 64>>>(out, iters);
        if (k == 2) kC<<<grid, 64>>>(out, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      const double lane_op_pairs = (double)iters * 8 * wps;  // 8 pk-equivalents per iter per wave, per SIMD
      printf("waves/SIMD %d %s: %.3f ms, %.3f ns per pk-equivalent per SIMD\n", wps,
             k == 0 ? "A s_mov+pk" : k == 1 ? "B pk (SGPR held)" : "C 2x VOP2 literal", best,
             best * 1e6 / lane_op_pairs);
    }
  }
  return 0;
}
