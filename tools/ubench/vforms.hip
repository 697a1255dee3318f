// Issue cost of the instruction forms K1's quantisation and conversion use,
// and of dependency distance, 8 waves per SIMD, 16 accumulators per wave.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)
#define B(X) REP16(X) REP16(X) REP16(X) REP16(X)
#define MUL(i) "v_mul_f32 v" #i ", 0x3f7ffffe, v" #i "\n"
#define ADDV(i) "v_add_f32 v" #i ", v" #i ", v40\n"
#define FMA3(i) "v_fma_f32 v" #i ", v" #i ", v40, v41\n"
#define FMAABS(i) "v_fma_f32 v" #i ", |v" #i "|, s40, |v41|\n"
#define MAX3(i) "v_max3_f32 v" #i ", v" #i ", v40, v41\n"
#define SDWA(i) "v_cvt_f32_i32_sdwa v" #i ", sext(v" #i ") dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1\n"
#define CVT(i) "v_cvt_f32_i32 v" #i ", v" #i "\n"
#define PAIR1(i) "v_mul_f32 v" #i ", 0x3f7ffffe, v" #i "\n v_add_f32 v" #i ", v" #i ", v40\n"
#define SUBSB(i) "v_sub_f32 v" #i ", v" #i ", v" #i "\n"
#define PERM(i) "v_perm_b32 v" #i ", v" #i ", v40, s41\n"
#define BFE(i) "v_bfe_i32 v" #i ", v" #i ", 8, 8\n"
#define CLOB "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","v40","v41","s40","s41"

template <int K>
__global__ __launch_bounds__(256) void kern(float* out, int iters) {
  asm volatile("v_mov_b32 v40, 1.0\n v_mov_b32 v41, 1.0\n s_mov_b32 s40, 1.0\n s_mov_b32 s41, 0x05040100\n" ::: "v40", "v41", "s40", "s41");
  for (int it = 0; it < iters; it++) {
    if (K == 0) asm volatile(B(MUL) B(ADDV) ::: CLOB);
    if (K == 1) asm volatile(B(FMA3) ::: CLOB);
    if (K == 2) asm volatile(B(FMAABS) ::: CLOB);
    if (K == 3) asm volatile(B(MAX3) ::: CLOB);
    if (K == 4) asm volatile(B(SDWA) ::: CLOB);
    if (K == 5) asm volatile(B(CVT) ::: CLOB);
    if (K == 6) asm volatile(B(PAIR1) ::: CLOB);
    if (K == 7) asm volatile(B(SUBSB) ::: CLOB);
    if (K == 8) asm volatile(B(PERM) ::: CLOB);
    if (K == 9) asm volatile(B(BFE) ::: CLOB);
  }
  out[blockIdx.x * 256 + threadIdx.x] = 1.0f;
}

int main() {
  float* out;
  (void)hipMalloc(&out, 1 << 26);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[10] = {"mul lit + add (dist 16)", "v_fma_f32 3 vgpr", "v_fma_f32 |v|,s,|v|", "v_max3_f32",
                           "v_cvt_f32_i32_sdwa", "v_cvt_f32_i32", "mul;add dependent (dist 1)",
                           "v_sub_f32 same reg", "v_perm_b32", "v_bfe_i32"};
  const int per[10] = {128, 64, 64, 64, 64, 64, 128, 64, 64, 64};
  for (int wps : {2, 4, 8}) {
    for (int k = 0; k < 10; k++) {
      const int iters = 512;
      float best = 1e9;
      for (int rep = 0; rep < 3; rep++) {
        const int grid = 256 * wps;
        (void)hipEventRecord(e0);
        switch (k) {
          case 0: kern<0><<<grid, 256>>>(out, iters); break;
          case 1: kern<1><<<grid, 256>>>(out, iters); break;
          case 2: kern<2><<<grid, 256>>>(out, iters); break;
          case 3: kern<3><<<grid, 256>>>(out, iters); break;
          case 4: kern<4><<<grid, 256>>>(out, iters); break;
          case 5: kern<5><<<grid, 256>>>(out, iters); break;
          case 6: kern<6><<<grid, 256>>>(out, iters); break;
          case 7: kern<7><<<grid, 256>>>(out, iters); break;
          case 8: kern<8><<<grid, 256>>>(out, iters); break;
          case 9: kern<9><<<grid, 256>>>(out, iters); break;
        }
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      const double insts = (double)iters * per[k] * wps;
      printf("waves/SIMD %d %-28s %.3f ns/inst/SIMD\n", wps, names[k], best * 1e6 / insts);
    }
  }
  return 0;
}
