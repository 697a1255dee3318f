// Issue cost of the integer / mixed instruction forms the decoder's symbol
// loop, K2 and K1's stores use (VOP3 64-bit, SDWA, 24-bit multiplies, bit
// counts, compares into SGPR pairs), 4 and 8 waves per SIMD, 16 independent
// registers per wave (8 pairs for the 64-bit forms).  Build:
//   hipcc --offload-arch=gfx950 -O2 -o tools/ubench/iforms tools/ubench/iforms.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)
#define REP8P(X) X(0, 1) X(2, 3) X(4, 5) X(6, 7) X(8, 9) X(10, 11) X(12, 13) X(14, 15)
#define B16(X) REP16(X) REP16(X) REP16(X) REP16(X)
#define B8P(X) REP8P(X) REP8P(X) REP8P(X) REP8P(X) REP8P(X) REP8P(X) REP8P(X) REP8P(X)

#define ADD(i) "v_add_u32 v" #i ", v" #i ", v40\n"
#define MAD64(a, b) "v_mad_u64_u32 v[" #a ":" #b "], s[42:43], v" #a ", v40, v[" #a ":" #b "]\n"
#define MAD24(i) "v_mad_u32_u24 v" #i ", v" #i ", v40, v41\n"
#define MUL24(i) "v_mul_u32_u24 v" #i ", v" #i ", v40\n"
#define MUL24S(i) "v_mul_u32_u24_sdwa v" #i ", v" #i ", v40 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD\n"
#define SHL64(a, b) "v_lshlrev_b64 v[" #a ":" #b "], v40, v[" #a ":" #b "]\n"
#define ALIGN(i) "v_alignbit_b32 v" #i ", v" #i ", v40, v41\n"
#define BCNT(i) "v_bcnt_u32_b32 v" #i ", v" #i ", 0\n"
#define CMPS(i) "v_cmp_lt_u32_sdwa s[42:43], v" #i ", v40 src0_sel:DWORD src1_sel:WORD_0\n"
#define CMPE(i) "v_cmp_lt_u32_e64 s[42:43], v" #i ", v40\n"
#define ANDOR(i) "v_and_or_b32 v" #i ", v" #i ", v40, v41\n"
#define ADD3(i) "v_add3_u32 v" #i ", v" #i ", v40, v41\n"
#define CND(i) "v_cndmask_b32_e64 v" #i ", v" #i ", v40, s[44:45]\n"
#define MULLO(i) "v_mul_lo_u32 v" #i ", v" #i ", v40\n"
#define SHR(i) "v_lshrrev_b32 v" #i ", v40, v" #i "\n"
#define MINS(i) "v_min_u32_sdwa v" #i ", v" #i ", v40 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:DWORD\n"
#define PKADD(i) "v_pk_add_u16 v" #i ", v" #i ", v40\n"
#define DPP(i) "v_mov_b32_dpp v" #i ", v" #i " quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
#define LSHLOR(i) "v_lshl_or_b32 v" #i ", v" #i ", 16, v40\n"
#define BFEU(i) "v_bfe_u32 v" #i ", v" #i ", 8, 8\n"
#define CMPX(i) "v_cmp_lt_u32 vcc, v" #i ", v40\n"
#define CLOB "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","v40","v41","s42","s43","vcc"

constexpr int kN = 21;
template <int K>
__global__ __launch_bounds__(256) void kern(unsigned* out, int iters) {
  asm volatile("v_mov_b32 v40, 3\n v_mov_b32 v41, 5\n s_mov_b64 s[44:45], exec\n" ::: "v40", "v41", "s44", "s45");
  for (int it = 0; it < iters; it++) {
    if (K == 0) asm volatile(B16(ADD) ::: CLOB);
    if (K == 1) asm volatile(B8P(MAD64) ::: CLOB);
    if (K == 2) asm volatile(B16(MAD24) ::: CLOB);
    if (K == 3) asm volatile(B16(MUL24) ::: CLOB);
    if (K == 4) asm volatile(B16(MUL24S) ::: CLOB);
    if (K == 5) asm volatile(B8P(SHL64) ::: CLOB);
    if (K == 6) asm volatile(B16(ALIGN) ::: CLOB);
    if (K == 7) asm volatile(B16(BCNT) ::: CLOB);
    if (K == 8) asm volatile(B16(CMPS) ::: CLOB);
    if (K == 9) asm volatile(B16(CMPE) ::: CLOB);
    if (K == 10) asm volatile(B16(ANDOR) ::: CLOB);
    if (K == 11) asm volatile(B16(ADD3) ::: CLOB);
    if (K == 12) asm volatile(B16(CND) ::: CLOB);
    if (K == 13) asm volatile(B16(MULLO) ::: CLOB);
    if (K == 14) asm volatile(B16(SHR) ::: CLOB);
    if (K == 15) asm volatile(B16(MINS) ::: CLOB);
    if (K == 16) asm volatile(B16(PKADD) ::: CLOB);
    if (K == 17) asm volatile(B16(DPP) ::: CLOB);
    if (K == 18) asm volatile(B16(LSHLOR) ::: CLOB);
    if (K == 19) asm volatile(B16(BFEU) ::: CLOB);
    if (K == 20) asm volatile(B16(CMPX) ::: CLOB);
  }
  out[blockIdx.x * 256 + threadIdx.x] = 1u;
}

template <int K>
void launch(int grid, unsigned* out, int iters) {
  kern<K><<<grid, 256>>>(out, iters);
}
typedef void (*Fn)(int, unsigned*, int);
template <int... Ks>
struct Table {
  static constexpr Fn f[sizeof...(Ks)] = {launch<Ks>...};
};

int main() {
  unsigned* out;
  (void)hipMalloc(&out, 1 << 26);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const Fn fns[kN] = {launch<0>,  launch<1>,  launch<2>,  launch<3>,  launch<4>,  launch<5>,  launch<6>,
                      launch<7>,  launch<8>,  launch<9>,  launch<10>, launch<11>, launch<12>, launch<13>,
                      launch<14>, launch<15>, launch<16>, launch<17>, launch<18>, launch<19>, launch<20>};
  const char* names[kN] = {"v_add_u32 (VOP2)",        "v_mad_u64_u32",        "v_mad_u32_u24",
                           "v_mul_u32_u24 (VOP2)",    "v_mul_u32_u24_sdwa",   "v_lshlrev_b64",
                           "v_alignbit_b32",          "v_bcnt_u32_b32",       "v_cmp_lt_u32_sdwa -> s[]",
                           "v_cmp_lt_u32_e64 -> s[]", "v_and_or_b32",         "v_add3_u32",
                           "v_cndmask_b32_e64 s[]",   "v_mul_lo_u32",         "v_lshrrev_b32 (VOP2)",
                           "v_min_u32_sdwa",          "v_pk_add_u16",         "v_mov_b32_dpp quad_perm",
                           "v_lshl_or_b32",           "v_bfe_u32",            "v_cmp_lt_u32_e32 -> vcc"};
  for (int wps : {4, 8}) {
    for (int k = 0; k < kN; k++) {
      const int iters = 512;
      float best = 1e9;
      for (int rep = 0; rep < 3; rep++) {
        (void)hipEventRecord(e0);
        fns[k](256 * wps, out, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      const double insts = (double)iters * 64 * wps;
      printf("waves/SIMD %d %-26s %.3f ns/inst/SIMD\n", wps, names[k], best * 1e6 / insts);
    }
  }
  return 0;
}
