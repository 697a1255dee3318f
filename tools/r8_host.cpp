// Host harness (test infrastructure): runs K2's register-resident encoders
// (huff_common.hpp, compiled for the host) on blocks read from stdin and
// writes the chunks to stdout, for tests/test_r8_host.py to compare with the
// oracle.  argv[1]: "4" / "8" = build_r<CAP> + emit_chunk on every block;
// "auto" = the kernel's class dispatch (block_class); "dense" = "auto" packed
// the way k_huff_encode packs a tile (DenseWriter); "16" = build_r16 +
// emit_chunk16 (the CAP-16 overflow tier, huff_r16.hpp).
//   in:  u32 n, then n x 64 int16 coefficients in natural order
//   out: per block u8 ok, u8 size, then `size` chunk bytes (ok = 1);
//        "dense": u32 run bytes, then the run
#include <cstdio>
#include <cstring>
#include <vector>

#include "huff_common.hpp"
#include "huff_r16.hpp"

using namespace myyuv_gpu;

// Host writer with the put / align_byte interface emit_chunk expects.
struct HostWriter {
  uint8_t* out;
  uint64_t acc = 0;
  int nacc = 0;
  int pos = 0;
  void put(uint32_t v, int n) {
    acc |= (uint64_t)v << nacc;
    nacc += n;
    while (nacc >= 8) {
      out[pos++] = (uint8_t)acc;
      acc >>= 8;
      nacc -= 8;
    }
  }
  void align_byte() {
    if (nacc > 0) put(0, 8 - nacc);
  }
};

static bool build(const CoefRegs& R, const char* mode, EncState& S) {
  const int msz = R.msz();
  if (mode[0] == '4') return build_r<4>(R, msz, 64, S);
  if (mode[0] == '8') return build_r<8>(R, msz, 64, S);
  const uint32_t cls = block_class(R, msz);
  if (cls == kClassOvf) return false;  // straight to the overflow worklist
  if (cls == kClassSingle) {
    build_single(R, S);
    return true;
  }
  return cls == kClassR4 ? build_r<4>(R, msz, 64, S) : build_r<8>(R, msz, 64, S);
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "auto";
  uint32_t n = 0;
  if (fread(&n, 4, 1, stdin) != 1) return 2;
  std::vector<int16_t> c((size_t)n * 64);
  if (fread(c.data(), 2, c.size(), stdin) != c.size()) return 2;
  std::vector<EncState> st(n);
  std::vector<uint8_t> ok(n);
  for (uint32_t b = 0; b < n; b++) {
    CoefRegs R;
    for (int w = 0; w < 32; w++)
      R.w[w] = (uint16_t)c[b * 64 + 2 * w] | ((uint32_t)(uint16_t)c[b * 64 + 2 * w + 1] << 16);
    ok[b] = build(R, mode[0] == 'd' ? "auto" : mode, st[b]);
  }
  if (mode[0] == '1') {  // "16": the CAP-16 tier
    for (uint32_t b = 0; b < n; b++) {
      CoefRegs R;
      for (int w = 0; w < 32; w++)
        R.w[w] = (uint16_t)c[b * 64 + 2 * w] | ((uint32_t)(uint16_t)c[b * 64 + 2 * w + 1] << 16);
      EncState16 S16;
      uint32_t col[16] = {0};  // "16l": the kernel's LDS-column heap over a local column
      const bool ok16 = mode[2] == 'l' ? build_r16(R, R.msz(), 64, S16, r16::LdsHeap16<1>{col})
                                       : build_r16(R, R.msz(), 64, S16);
      const uint8_t hdr[2] = {(uint8_t)ok16, ok16 ? (uint8_t)S16.size : (uint8_t)0};
      fwrite(hdr, 1, 2, stdout);
      if (ok16) {
        uint8_t bytes[kMaxChunk] = {0};
        HostWriter hw{bytes};
        emit_chunk16(S16, 64, hw);
        hw.align_byte();
        if (hw.pos != (int)S16.size) return 3;
        fwrite(bytes, 1, S16.size, stdout);
      }
    }
    return 0;
  }
  if (mode[0] == 'd') {
    // "dense": K2's tile run — the accepted blocks' chunks back to back in
    // block order, each written by DenseWriter at its offset with the next
    // accepted chunk's header; out: u32 run bytes, the run
    std::vector<uint32_t> off(n + 1, 0);
    for (uint32_t b = 0; b < n; b++) off[b + 1] = off[b] + (ok[b] ? st[b].size : 0);
    std::vector<uint32_t> run(off[n] / 4 + 2, 0xA5A5A5A5u);  // canary: every dword must be stored
    for (uint32_t b = 0; b < n; b++) {
      if (!ok[b]) continue;
      uint32_t next = 0;
      for (uint32_t k = b + 1; k < n; k++)
        if (ok[k]) {
          next = st[k].hdr | 0x80000000u;
          break;
        }
      DenseWriter dw;
      dw.init(run.data(), off[b]);
      emit_chunk(st[b], 64, dw);
      dw.finish(next);
    }
    const uint32_t total = off[n];
    fwrite(&total, 4, 1, stdout);
    fwrite(run.data(), 1, total, stdout);
    return 0;
  }
  for (uint32_t b = 0; b < n; b++) {
    const uint8_t hdr[2] = {ok[b], ok[b] ? (uint8_t)st[b].size : (uint8_t)0};
    fwrite(hdr, 1, 2, stdout);
    if (ok[b]) {
      uint8_t bytes[kMaxChunk] = {0};
      HostWriter hw{bytes};
      emit_chunk(st[b], 64, hw);
      hw.align_byte();
      if (hw.pos != (int)st[b].size) return 3;
      fwrite(bytes, 1, st[b].size, stdout);
    }
  }
  return 0;
}
