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
#define CNDV(i) "v_cndmask_b32_e32 v" #i ", v" #i ", v40, vcc\n"
#define BITOP3(i) "v_bitop3_b32 v" #i ", v" #i ", v40, v41 bitop3:0xc8\n"
#define BFI(i) "v_bfi_b32 v" #i ", v" #i ", v40, v41\n"
#define MAXU(i) "v_max_u32 v" #i ", v" #i ", v40\n"
#define CVTUB(i) "v_cvt_f32_ubyte1 v" #i ", v" #i "\n"
#define FRACT(i) "v_fract_f32 v" #i ", v" #i "\n"
#define RNDNE(i) "v_rndne_f32 v" #i ", v" #i "\n"
#define MED3(i) "v_med3_f32 v" #i ", v" #i ", v40, v41\n"
#define CMPROT(i) "v_cmp_lt_u32_e64 s[" #i "*2+40:" #i "*2+41], v" #i ", v40\n"
#define XOR(i) "v_xor_b32 v" #i ", v" #i ", v40\n"
#define MULHI24(i) "v_mul_hi_u32_u24 v" #i ", v" #i ", v40\n"
#define ASHR(i) "v_ashrrev_i32 v" #i ", v40, v" #i "\n"
#define SUBREV(i) "v_subrev_u32 v" #i ", v" #i ", v40\n"
#define CMPCLASS(i) "v_cmp_class_f32_e64 s[42:43], v" #i ", v40\n"
#define MAXF(i) "v_max_f32 v" #i ", v" #i ", v40\n"
#define MINF(i) "v_min_f32 v" #i ", v" #i ", v40\n"
#define ANDV(i) "v_and_b32 v" #i ", v" #i ", v40\n"
#define ORV(i) "v_or_b32 v" #i ", v" #i ", v40\n"
#define ADDCO(i) "v_add_co_u32 v" #i ", vcc, v" #i ", v40\n"
#define SELPAIR(i) "v_cmp_lt_u32 vcc, v" #i ", v40\n v_cndmask_b32 v" #i ", v" #i ", v41, vcc\n"
#define MAXI(i) "v_max_i32 v" #i ", v" #i ", v40\n"
#define MINU(i) "v_min_u32 v" #i ", v" #i ", v40\n"
#define CLOB "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","v40","v41","s42","s43","vcc","s40","s41","s44","s45","s46","s47","s48","s49","s50","s51","s52","s53","s54","s55","s56","s57","s58","s59","s60","s61","s62","s63","s64","s65","s66","s67","s68","s69","s70","s71"

constexpr int kN = 43;
template <int K>
__global__ __launch_bounds__(256) void kern(unsigned* out, int iters) {
  asm volatile("v_mov_b32 v40, 3\n v_mov_b32 v41, 5\n s_mov_b64 s[44:45], exec\n s_mov_b64 vcc, exec\n" ::: "v40", "v41", "s44", "s45", "vcc");
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
    if (K == 21) asm volatile(B16(CNDV) ::: CLOB);
    if (K == 22) asm volatile(B16(BITOP3) ::: CLOB);
    if (K == 23) asm volatile(B16(BFI) ::: CLOB);
    if (K == 24) asm volatile(B16(MAXU) ::: CLOB);
    if (K == 25) asm volatile(B16(CVTUB) ::: CLOB);
    if (K == 26) asm volatile(B16(FRACT) ::: CLOB);
    if (K == 27) asm volatile(B16(RNDNE) ::: CLOB);
    if (K == 28) asm volatile(B16(MED3) ::: CLOB);
    if (K == 29) asm volatile(B16(CMPROT) ::: CLOB);
    if (K == 30) asm volatile(B16(XOR) ::: CLOB);
    if (K == 31) asm volatile(B16(MULHI24) ::: CLOB);
    if (K == 32) asm volatile(B16(ASHR) ::: CLOB);
    if (K == 33) asm volatile(B16(SUBREV) ::: CLOB);
    if (K == 34) asm volatile(B16(CMPCLASS) ::: CLOB);
    if (K == 35) asm volatile(B16(MAXF) ::: CLOB);
    if (K == 36) asm volatile(B16(MINF) ::: CLOB);
    if (K == 37) asm volatile(B16(ANDV) ::: CLOB);
    if (K == 38) asm volatile(B16(ORV) ::: CLOB);
    if (K == 39) asm volatile(B16(ADDCO) ::: CLOB);
    if (K == 40) asm volatile(B16(SELPAIR) ::: CLOB);
    if (K == 41) asm volatile(B16(MAXI) ::: CLOB);
    if (K == 42) asm volatile(B16(MINU) ::: CLOB);
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
                      launch<14>, launch<15>, launch<16>, launch<17>, launch<18>, launch<19>, launch<20>,
                      launch<21>, launch<22>, launch<23>, launch<24>, launch<25>, launch<26>, launch<27>,
                      launch<28>, launch<29>, launch<30>, launch<31>, launch<32>, launch<33>, launch<34>,
                      launch<35>, launch<36>, launch<37>, launch<38>, launch<39>, launch<40>, launch<41>,
                      launch<42>};
  const char* names[kN] = {"v_add_u32 (VOP2)",        "v_mad_u64_u32",        "v_mad_u32_u24",
                           "v_mul_u32_u24 (VOP2)",    "v_mul_u32_u24_sdwa",   "v_lshlrev_b64",
                           "v_alignbit_b32",          "v_bcnt_u32_b32",       "v_cmp_lt_u32_sdwa -> s[]",
                           "v_cmp_lt_u32_e64 -> s[]", "v_and_or_b32",         "v_add3_u32",
                           "v_cndmask_b32_e64 s[]",   "v_mul_lo_u32",         "v_lshrrev_b32 (VOP2)",
                           "v_min_u32_sdwa",          "v_pk_add_u16",         "v_mov_b32_dpp quad_perm",
                           "v_lshl_or_b32",           "v_bfe_u32",            "v_cmp_lt_u32_e32 -> vcc",
                           "v_cndmask_b32_e32 (vcc)", "v_bitop3_b32",         "v_bfi_b32",
                           "v_max_u32 (VOP2)",        "v_cvt_f32_ubyte1",     "v_fract_f32",
                           "v_rndne_f32",             "v_med3_f32",           "v_cmp_lt_u32_e64 rot s[]",
                           "v_xor_b32 (VOP2)",        "v_mul_hi_u32_u24",     "v_ashrrev_i32 (VOP2)",
                           "v_subrev_u32 (VOP2)",     "v_cmp_class_f32_e64",  "v_max_f32 (VOP2)",
                           "v_min_f32 (VOP2)",        "v_and_b32 (VOP2)",     "v_or_b32 (VOP2)",
                           "v_add_co_u32 -> vcc",     "cmp->vcc + cndmask (per pair)", "v_max_i32 (VOP2)",
                           "v_min_u32 (VOP2)"};
  for (int wps : {8}) {
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
      const double insts = (double)iters * (k == 40 ? 128 : 64) * wps;
      printf("waves/SIMD %d %-26s %.3f ns/inst/SIMD\n", wps, names[k], best * 1e6 / insts);
    }
  }
  return 0;
}
