// Host harness (test infrastructure): runs K2's register-resident encoders
// (huff_common.hpp, compiled for the host) on blocks read from stdin and
// writes the chunks to stdout, for tests/test_r8_host.py to compare with the
// oracle.  argv[1]: "4" / "8" = encode_block_r<CAP> on every block; "auto" =
// the kernel's class dispatch (block_class).
//   in:  u32 n, then n x 64 int16 coefficients in natural order
//   out: per block u8 ok, u8 size, then `size` chunk bytes (ok = 1)
#include <cstdio>
#include <cstring>
#include <vector>

#include "huff_common.hpp"

using namespace myyuv_gpu;

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "auto";
  uint32_t n = 0;
  if (fread(&n, 4, 1, stdin) != 1) return 2;
  std::vector<int16_t> c((size_t)n * 64);
  if (fread(c.data(), 2, c.size(), stdin) != c.size()) return 2;
  std::vector<uint32_t> slot(kSlotWords * kWave);
  for (uint32_t b = 0; b < n; b++) {
    CoefRegs R;
    for (int w = 0; w < 32; w++)
      R.w[w] = (uint16_t)c[b * 64 + 2 * w] | ((uint32_t)(uint16_t)c[b * 64 + 2 * w + 1] << 16);
    std::fill(slot.begin(), slot.end(), 0u);
    uint8_t size = 0;
    const int msz = R.msz();
    bool ok;
    if (mode[0] == '4') {
      ok = encode_block_r<4>(R, msz, 64, slot.data(), &size);
    } else if (mode[0] == '8') {
      ok = encode_block_r<8>(R, msz, 64, slot.data(), &size);
    } else {
      const uint32_t cls = block_class(R, msz);
      if (cls == kClassSingle) {
        encode_block_single(R, slot.data(), &size);
        ok = true;
      } else if (cls == kClassR4) {
        ok = encode_block_r<4>(R, msz, 64, slot.data(), &size);
      } else {
        ok = encode_block_r<8>(R, msz, 64, slot.data(), &size);
      }
    }
    const uint8_t hdr[2] = {(uint8_t)ok, ok ? size : (uint8_t)0};
    fwrite(hdr, 1, 2, stdout);
    if (ok) {
      uint8_t bytes[kMaxChunk];
      for (int w = 0; w < kSlotWords; w++) memcpy(bytes + 4 * w, &slot[(size_t)w * kWave], 4);
      fwrite(bytes, 1, size, stdout);
    }
  }
  return 0;
}
