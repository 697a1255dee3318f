/* Host check of the division- and roundf-free arithmetic in k_transform.hip
 * (IEEE binary32, round-to-nearest-even: the same operations the GPU runs).
 *
 *  1. roundf(x) == truncf(x + copysignf(0x1.fffffep-2f, x)) for every finite
 *     float (all 2^32 encodings with "all"; sampled otherwise).
 *  2. K1 quantisation: for every Q in 1..255 and every y within 256 ulps of
 *     each tie point h*Q (h a half-integer, |h*Q| <= 1100), plus random y in
 *     [-1100, 1100]: whenever the fast path's near-tie test says "far"
 *     (fma(|t|, 2^-21, |e|) < 0.5), its integer (low 16 bits of
 *     t + 1.5*2^23) equals (int)roundf(y / Q) — the reference's divide.
 *  3. K6 rounding: for s' in [-128, 127] near every half-integer and at
 *     random, when |s' - rint(s')| < 0.5 the low byte of s' + 1.5*2^23 + 128
 *     equals 128 + (int)roundf(s').
 * Prints "ok <checks>" or the first failure; exit status 0 on success.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static uint32_t bits(float x) { uint32_t u; memcpy(&u, &x, 4); return u; }
static float fl(uint32_t u) { float x; memcpy(&x, &u, 4); return x; }
static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(void) { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return (uint32_t)(rng >> 11); }

static const float kHalfDown = 0x1.fffffep-2f;
static const float kMagic = 0x1.8p23f;
static const float kMagicPx = 0x1.8p23f + 128.0f;
static const float kNearRel = 0x1p-21f;

static int check_roundf(int all, uint64_t* n) {
  const uint64_t step = all ? 1 : 257;  /* a prime stride samples every exponent */
  for (uint64_t u = 0; u <= 0xFFFFFFFFull; u += step) {
    volatile float x = fl((uint32_t)u);
    if (!isfinite(x)) continue;
    volatile float s = x + copysignf(kHalfDown, x);
    if (truncf(s) != roundf(x)) { printf("roundf %a\n", (double)x); return 1; }
    (*n)++;
  }
  return 0;
}

static int quant_one(float y, int Q, uint64_t* n) {
  const float q = (float)Q;
  const float r = 1.0f / q;
  volatile float t = y * r;
  volatile float u = t + kMagic;
  volatile float rt = u - kMagic;
  volatile float e = t - rt;
  volatile float nt = fmaf(fabsf(t), kNearRel, fabsf(e));
  (*n)++;
  if (nt < 0.5f) {  /* fast path */
    const int16_t fast = (int16_t)(bits(u) & 0xFFFF);
    const int ref = (int)roundf(y / q);
    if (fast != (int16_t)ref) { printf("quant y=%a Q=%d fast=%d ref=%d\n", (double)y, Q, fast, ref); return 1; }
  }
  return 0;
}

static int check_quant(uint64_t* n) {
  for (int Q = 1; Q <= 255; Q++) {
    for (int k = -2 * 1100 / Q - 1; k <= 2 * 1100 / Q + 1; k++) {
      if ((k & 1) == 0) continue;
      const float tie = 0.5f * (float)k * (float)Q;  /* y with y/Q a half-integer */
      if (fabsf(tie) > 1100.0f) continue;
      uint32_t b = bits(tie);
      for (int d = -256; d <= 256; d++) {
        const float y = fl(b + (uint32_t)d);
        if (isfinite(y) && quant_one(y, Q, n)) return 1;
      }
    }
    for (int i = 0; i < 200000; i++) {
      const float y = ((float)(rnd() & 0xFFFFFF) / 16777216.0f * 2.0f - 1.0f) * 1100.0f;
      if (quant_one(y, Q, n)) return 1;
    }
  }
  return 0;
}

static int px_one(float s, uint64_t* n) {
  volatile float c = fminf(fmaxf(s, -128.0f), 127.0f);
  volatile float u = c + kMagicPx;
  volatile float e = c - (u - kMagicPx);
  (*n)++;
  if (fabsf(e) < 0.5f) {
    const int fast = (int)(bits(u) & 0xFF);
    int ref = (int)roundf(s) + 128;
    ref = ref < 0 ? 0 : (ref > 255 ? 255 : ref);
    if (fast != ref) { printf("pixel s=%a fast=%d ref=%d\n", (double)s, fast, ref); return 1; }
  }
  return 0;
}

static int check_pixels(uint64_t* n) {
  for (int k = -300; k <= 300; k++) {
    const uint32_t b = bits(0.5f * (float)k);
    for (int d = -4096; d <= 4096; d++) {
      const float s = fl(b + (uint32_t)d);
      if (isfinite(s) && px_one(s, n)) return 1;
    }
  }
  for (int i = 0; i < 4000000; i++) {
    const float s = ((float)(rnd() & 0xFFFFFF) / 16777216.0f * 2.0f - 1.0f) * 200.0f;
    if (px_one(s, n)) return 1;
  }
  return 0;
}

int main(int argc, char** argv) {
  const int all = argc > 1 && strcmp(argv[1], "all") == 0;
  uint64_t n = 0;
  if (check_roundf(all, &n) || check_quant(&n) || check_pixels(&n)) return 1;
  printf("ok %llu\n", (unsigned long long)n);
  return 0;
}
