// Issue throughput of the f32 instruction forms the transforms use, with 8
// independent chains per wave (no dependency stalls), 1..8 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
// scalar VOP2 multiply by a literal
#define MUL_LIT(i) "v_mul_f32 v" #i ", 0x3f7ffffe, v" #i "\n"
// packed multiply by an SGPR pair (broadcast lo)
#define PK_MUL_S(i) "v_pk_mul_f32 v[" #i "*2+8:" #i "*2+9], v[" #i "*2+8:" #i "*2+9], s[40:41] op_sel_hi:[1,0]\n"
// scalar add vgpr+vgpr
#define ADD_V(i) "v_add_f32 v" #i ", v" #i ", v30\n"
// packed add vgpr+vgpr
#define PK_ADD_V(i) "v_pk_add_f32 v[" #i "*2+8:" #i "*2+9], v[" #i "*2+8:" #i "*2+9], v[30:31]\n"

template <int K>
__global__ __launch_bounds__(64) void kern(float* out, int iters) {
  asm volatile("s_mov_b32 s40, 0x3f7ffffe\n s_mov_b32 s41, 0x3f7ffffe\n v_mov_b32 v30, 0\n v_mov_b32 v31, 0\n" ::: "s40", "s41", "v30", "v31");
  for (int it = 0; it < iters; it++) {
    if (K == 0) asm volatile(R8(MUL_LIT) R8(MUL_LIT) ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7");
    if (K == 1) asm volatile(R8(PK_MUL_S) R8(PK_MUL_S) ::: "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23");
    if (K == 2) asm volatile(R8(ADD_V) R8(ADD_V) ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7");
    if (K == 3) asm volatile(R8(PK_ADD_V) R8(PK_ADD_V) ::: "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23");
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
  const char* names[4] = {"v_mul_f32 literal", "v_pk_mul_f32 sgpr", "v_add_f32 vgpr", "v_pk_add_f32 vgpr"};
  for (int wps : {1, 2, 4, 8}) {
    for (int k = 0; k < 4; k++) {
      float best = 1e9;
      for (int rep = 0; rep < 3; rep++) {
        (void)hipEventRecord(e0);
        const int grid = 1024 * wps;
        if (k == 0) kern<0><<<grid, 64>>>(out, iters);
        if (k == 1) kern<1><<<grid, 64>>>(out, iters);
        if (k == 2) kern<2><<<grid, 64>>>(out, iters);
        if (k == 3) kern<3><<<grid, 64>>>(out, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      const double insts = (double)iters * 16 * wps;  // per SIMD
      printf("waves/SIMD %d %-20s %.3f ns/inst/SIMD\n", wps, names[k], best * 1e6 / insts);
    }
  }
  return 0;
}
