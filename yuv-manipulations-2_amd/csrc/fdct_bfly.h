// fdct_bfly.h — K1's fast forward transform (round 5): the 8-point DCT of
// the reference's literal basis (DCT.cpp:221-230) evaluated as an even/odd
// butterfly over a NOMINAL basis N (the literal one made exactly symmetric),
// plus the error bound that decides per unit whether the result is provably
// the reference's.  Shared, operation for operation, by the gfx950 kernel
// (xform_common.hpp fdct_fast) and the host check tools/diag/
// fdct_bfly_check.cpp (tests/test_numerics.py), which emulates the kernel's
// arithmetic and compares every unit that passes the bound with the
// reference transform.
//
// The reference: T = D X (k-ascending sums of rounded products), Y = T D^T,
// coefficient roundf(fl(Y / Q)) (DCT.cpp:232-254, 269-277).  The fast path:
//   stage 1, columns: x = pixel (unsigned; the -128 of DCT.cpp:303 folded
//     into the DC term), s/d butterflies in exact integer-valued floats, then
//     T0 = c0 (E0 - 1024), T4 = c4 E4, T2/T6 two-term, odd rows four-term
//     FMA chains: at most 4 roundings per output;
//   stage 2, rows: the same butterfly on float T, every operation rounded:
//     at most 5 roundings per output.
// With N the matrix this computes in exact arithmetic, delta = max|N - D|
// (<= 5.5 u, u = 2^-24), A = sum |x - 128| over the block, n = d = 0.4904:
//   |T_f - T*| <= (g4 n + delta) A_k =: e1 A_k          (T* = D X exactly)
//   |Y_f - Y*| <= (g5 n (d + e1) + n e1 + delta d) A    (Y* = T* D^T)
//   |Y_ref - Y*| <= g8 d^2 (2 + g8) A
// (g_k = k u / (1 - k u), Higham), so |Y_f - Y_ref| <= kappa A with kappa =
// 11.41 u; |Y_f| <= 0.2406 A.  The quantised value t = fl(Y_f * fl(1/Q))
// then lies within beta = A * r_max * (kappa (1 + 2^-20) + 0.2406 * 2^-21)
// of fl(Y_ref / Q) (the second term: the divide's and the reciprocal's
// roundings), r_max the largest 1/Q of the output's row.  kBflyK = 7.946e-7
// (13.33 u) is that factor with margin (tools/diag/fdct_bfly_derive.py
// computes N, delta and K from the literal basis); kb[row] = kBflyK r_max
// (1 + 2^-20) covers the float evaluation of A * kb.  An output whose t is
// further than beta from every half-integer rounds (half-even, magic add) to
// the reference's roundf of fl(Y_ref / Q): fl(Y_ref / Q) lies strictly inside
// the same (n - 1/2, n + 1/2).  A unit with any closer output goes to the
// reference-order transform (k_fdct_fix).
#pragma once

#if defined(__HIPCC__)
#define MYYUV_BF_HD __host__ __device__ __forceinline__
#else
#include <math.h>
#define MYYUV_BF_HD static inline
#endif

namespace myyuv_bfly {

// N: row 0 = c0 (the literal row 0 exactly), row 4 = c4 (+ - - + + - - +),
// rows 2 / 6 = (a, b, -b, -a, -a, -b, b, a) / (b, -a, a, -b, -b, a, -a, b),
// odd rows antisymmetric (N[i][7 - m] = -N[i][m]); each value the midpoint of
// the literal entries it stands for (fdct_bfly_derive.py)
constexpr float kC0 = 0.3535533845424652f, kC4 = 0.3535534143447876f;
constexpr float kA2 = 0.4619397521018982f, kB2 = 0.19134166836738586f;
constexpr float kA6 = 0.4619397521018982f, kB6 = 0.19134169816970825f;
constexpr float kO1[4] = {0.49039262533187866f, 0.41573476791381836f, 0.27778512239456177f, 0.09754513204097748f};
constexpr float kO3[4] = {0.41573482751846313f, -0.0975450873374939f, -0.49039262533187866f, -0.277785062789917f};
constexpr float kO5[4] = {0.2777852416038513f, -0.49039262533187866f, 0.09754514694213867f, 0.41573476791381836f};
constexpr float kO7[4] = {0.09754543751478195f, -0.2777852416038513f, 0.4157347083091736f, -0.49039262533187866f};
constexpr float kBflyK = 7.946e-7f;

MYYUV_BF_HD float odd4(const float (&o)[4], float d0, float d1, float d2, float d3) {
  return fmaf(o[3], d3, fmaf(o[2], d2, fmaf(o[1], d1, o[0] * d0)));
}

// Column transform of one block column: p[m] = pixel of row m (0..255, as
// float); t[i] = T[i][k].  Everything before the last products is exact.
MYYUV_BF_HD void bfly_cols(const float (&p)[8], float (&t)[8]) {
  const float s0 = p[0] + p[7], s1 = p[1] + p[6], s2 = p[2] + p[5], s3 = p[3] + p[4];
  const float d0 = p[0] - p[7], d1 = p[1] - p[6], d2 = p[2] - p[5], d3 = p[3] - p[4];
  const float ss0 = s0 + s3, ss1 = s1 + s2, ds0 = s0 - s3, ds1 = s1 - s2;
  t[0] = kC0 * ((ss0 + ss1) - 1024.0f);
  t[4] = kC4 * (ss0 - ss1);
  t[2] = fmaf(kA2, ds0, kB2 * ds1);
  t[6] = fmaf(kB6, ds0, -kA6 * ds1);
  t[1] = odd4(kO1, d0, d1, d2, d3);
  t[3] = odd4(kO3, d0, d1, d2, d3);
  t[5] = odd4(kO5, d0, d1, d2, d3);
  t[7] = odd4(kO7, d0, d1, d2, d3);
}

// Row transform of one row of T: x[k] = T[i][k]; y[v] = Y[i][v].
MYYUV_BF_HD void bfly_rows(const float (&x)[8], float (&y)[8]) {
  const float s0 = x[0] + x[7], s1 = x[1] + x[6], s2 = x[2] + x[5], s3 = x[3] + x[4];
  const float d0 = x[0] - x[7], d1 = x[1] - x[6], d2 = x[2] - x[5], d3 = x[3] - x[4];
  const float ss0 = s0 + s3, ss1 = s1 + s2, ds0 = s0 - s3, ds1 = s1 - s2;
  y[0] = kC0 * (ss0 + ss1);
  y[4] = kC4 * (ss0 - ss1);
  y[2] = fmaf(kA2, ds0, kB2 * ds1);
  y[6] = fmaf(kB6, ds0, -kA6 * ds1);
  y[1] = odd4(kO1, d0, d1, d2, d3);
  y[3] = odd4(kO3, d0, d1, d2, d3);
  y[5] = odd4(kO5, d0, d1, d2, d3);
  y[7] = odd4(kO7, d0, d1, d2, d3);
}

// kb[i] for the rows of one plane: kBflyK * max_v r[i][v] * (1 + 2^-20),
// rounded up (r: the plane's 1 / Q table, natural order).
MYYUV_BF_HD void bfly_row_bounds(const float* r, float* kb) {
  for (int i = 0; i < 8; i++) {
    double m = 0.0;
    for (int v = 0; v < 8; v++) m = r[i * 8 + v] > m ? r[i * 8 + v] : m;
    kb[i] = (float)((double)kBflyK * m * (1.0 + 0x1p-20) * (1.0 + 0x1p-22));
  }
}

#if !defined(__HIPCC__)
// The kernel's arithmetic for one whole block (host check): coefficients in
// natural order; returns 0 when some output is not provably the reference's.
static inline int bfly_block(const unsigned char* px, const float* R, const float* kb, short* out) {
  unsigned a = 0;
  for (int i = 0; i < 64; i++) a += px[i] > 128 ? px[i] - 128u : 128u - px[i];
  const float af = (float)a;
  float T[8][8];
  for (int k = 0; k < 8; k++) {
    float p[8], t[8];
    for (int m = 0; m < 8; m++) p[m] = (float)px[m * 8 + k];
    bfly_cols(p, t);
    for (int i = 0; i < 8; i++) T[i][k] = t[i];
  }
  int ok = 1;
  for (int i = 0; i < 8; i++) {
    float y[8];
    bfly_rows(T[i], y);
    float em = 0.0f;
    for (int v = 0; v < 8; v++) {
      const float t = y[v] * R[i * 8 + v];
      const float uu = t + 0x1.8p23f;
      const float e = t - (uu - 0x1.8p23f);
      em = fmaxf(em, fabsf(e));
      out[i * 8 + v] = (short)(int)(uu - 0x1.8p23f);
    }
    if (fmaf(af, kb[i], em) >= 0.5f) ok = 0;  // (the kernel: one fma, max over the rows)
  }
  return ok;
}
#endif

}  // namespace myyuv_bfly
