// Instruction-fetch sensitivity: a long straight-line body (N independent
// f32 multiplies over 16 accumulators, no loop reuse inside the body) in
// 8-byte form (VOP2 with a 32-bit literal) vs 4-byte form (VOP2, VGPR
// operand) vs 8-byte packed form (v_pk_mul_f32, two multiplies), 8 waves per
// SIMD, timed per instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)
#define LIT(i) "v_mul_f32 v" #i ", 0x3f7ffffe, v" #i "\n"
#define VGP(i) "v_mul_f32 v" #i ", v40, v" #i "\n"
#define PKM(i) "v_pk_mul_f32 v[" #i "*2+0:" #i "*2+1], v[" #i "*2+0:" #i "*2+1], v[40:41]\n"
#define B16(X) REP16(X)
#define B256(X) B16(X) B16(X) B16(X) B16(X) B16(X) B16(X) B16(X) B16(X) B16(X) B16(X) B16(X) B16(X) B16(X) B16(X) B16(X) B16(X)
#define B1K(X) B256(X) B256(X) B256(X) B256(X)
#define CLOB "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31","v40","v41"

template <int K>
__global__ __launch_bounds__(256) void kern(float* out, int iters) {
  asm volatile("v_mov_b32 v40, 1.0\n v_mov_b32 v41, 1.0\n" ::: "v40", "v41");
  for (int it = 0; it < iters; it++) {
    if (K == 0) asm volatile(B1K(LIT) B1K(LIT) ::: CLOB);
    if (K == 1) asm volatile(B1K(VGP) B1K(VGP) ::: CLOB);
    if (K == 2) asm volatile(B1K(PKM) ::: CLOB);
    if (K == 3) asm volatile(B256(LIT) ::: CLOB);
    if (K == 4) asm volatile(B256(VGP) ::: CLOB);
  }
  out[blockIdx.x * 256 + threadIdx.x] = 1.0f;
}

int main() {
  float* out;
  (void)hipMalloc(&out, 1 << 26);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[5] = {"2048 x VOP2 literal (8 B)", "2048 x VOP2 vgpr (4 B)", "1024 x pk_mul (8 B, 2 ops)",
                          "256 x VOP2 literal (8 B)", "256 x VOP2 vgpr (4 B)"};
  const int body[5] = {2048, 2048, 1024, 256, 256};
  for (int wps : {4, 8}) {
    for (int k = 0; k < 5; k++) {
      const int iters = k >= 3 ? 64 : 8;
      float best = 1e9;
      for (int rep = 0; rep < 3; rep++) {
        const int grid = 256 * wps;  // 256-thread WGs: 4 waves, one per SIMD
        (void)hipEventRecord(e0);
        if (k == 0) kern<0><<<grid, 256>>>(out, iters);
        if (k == 1) kern<1><<<grid, 256>>>(out, iters);
        if (k == 2) kern<2><<<grid, 256>>>(out, iters);
        if (k == 3) kern<3><<<grid, 256>>>(out, iters);
        if (k == 4) kern<4><<<grid, 256>>>(out, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      const double insts = (double)iters * body[k] * wps;  // per SIMD
      printf("waves/SIMD %d %-28s %.3f ns/inst/SIMD (%.1f us)\n", wps, names[k], best * 1e6 / insts, best * 1e3);
    }
  }
  return 0;
}
