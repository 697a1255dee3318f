// ref_harness.cpp — C entry points over the REFERENCE library's public API.
//
// TEST INFRASTRUCTURE ONLY.  oracle/Makefile compiles the reference sources
// where they lie (/root/reference/myyuv_lib/*.cpp, never copied) together with
// this file into oracle/_ref/libmyyuv_ref_{serial,omp}.so.  Tests use it to pin
// the CPU restatement (oracle/myyuv_oracle.c) and the HIP path against the
// reference itself; bench.py times it as the "reference" cpu_baseline.
//
// Calls only the reference's public surface: myyuv::YUV (myyuv_yuv.hpp:37-350),
// YUV::compress / YUV::decompress (myyuv_yuv.cpp:454-483), which dispatch through
// YUV::compress_map / decompress_map to myyuvDCT::compress_DCT_planar /
// decompress_DCT_planar (DCT.cpp:371-488).
#include <myyuv.hpp>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <exception>
#include <string>

namespace {

thread_local std::string g_last_error;

myyuv::YUV make_raw(const uint8_t* iyuv, uint32_t w, uint32_t h) {
  myyuv::YUV y;
  y.header.fourcc_format = myyuv::YUV::FourccFormats::IYUV;
  y.header.width = w;
  y.header.height = h;
  y.header.data_pos = sizeof(myyuv::YUVHeader);
  y.header.data_size = w * h * 3 / 2;
  y.data = new uint8_t[y.header.data_size];
  std::memcpy(y.data, iyuv, y.header.data_size);
  return y;
}

myyuv::YUV make_compressed(const uint8_t* payload, uint32_t size, uint32_t w, uint32_t h,
                           const uint8_t q[3]) {
  myyuv::YUV y;
  y.header.fourcc_format = myyuv::YUV::FourccFormats::IYUV;
  y.header.width = w;
  y.header.height = h;
  y.header.compression = myyuv::YUV::Compressions::DCT;
  y.header.compression_params_size = 3;
  y.header.compression_params_pos = sizeof(myyuv::YUVHeader);
  y.header.data_pos = sizeof(myyuv::YUVHeader) + 3;
  y.header.data_size = size;
  y.compression_params = new uint8_t[3];
  std::memcpy(y.compression_params, q, 3);
  y.data = new uint8_t[size];
  std::memcpy(y.data, payload, size);
  return y;
}

}  // namespace

extern "C" {

const char* ref_last_error() { return g_last_error.c_str(); }

// Returns 0 on success, 1 on exception (message in ref_last_error()), 2 if cap too small.
int ref_compress(const uint8_t* iyuv, uint32_t w, uint32_t h, const uint8_t q[3], uint8_t* out,
                 uint32_t cap, uint32_t* out_size) {
  try {
    myyuv::YUV in = make_raw(iyuv, w, h);
    myyuv::YUV c = in.compress(myyuv::YUV::Compressions::DCT, q, 3);
    *out_size = c.header.data_size;
    if (c.header.data_size > cap) return 2;
    std::memcpy(out, c.data, c.header.data_size);
    return 0;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return 1;
  }
}

int ref_decompress(const uint8_t* payload, uint32_t size, uint32_t w, uint32_t h, const uint8_t q[3],
                   uint8_t* iyuv) {
  try {
    myyuv::YUV in = make_compressed(payload, size, w, h, q);
    myyuv::YUV d = in.decompress();
    std::memcpy(iyuv, d.data, d.header.data_size);
    return 0;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return 1;
  }
}

// Times `iters` in-process compress and decompress calls of the public API
// (file I/O excluded, as SURVEY.md §6 measured); writes per-call medians in ms.
int ref_bench(const uint8_t* iyuv, uint32_t w, uint32_t h, const uint8_t q[3], int iters,
              double* comp_ms, double* decomp_ms) {
  try {
    myyuv::YUV in = make_raw(iyuv, w, h);
    double tc[64], td[64];
    iters = std::max(1, std::min(iters, 64));
    for (int i = 0; i < iters; i++) {
      auto t0 = std::chrono::steady_clock::now();
      myyuv::YUV c = in.compress(myyuv::YUV::Compressions::DCT, q, 3);
      auto t1 = std::chrono::steady_clock::now();
      myyuv::YUV d = c.decompress();
      auto t2 = std::chrono::steady_clock::now();
      tc[i] = std::chrono::duration<double, std::milli>(t1 - t0).count();
      td[i] = std::chrono::duration<double, std::milli>(t2 - t1).count();
    }
    std::sort(tc, tc + iters);
    std::sort(td, td + iters);
    *comp_ms = tc[iters / 2];
    *decomp_ms = td[iters / 2];
    return 0;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return 1;
  }
}

// BMP -> IYUV through the reference's public surface: myyuv::BMP(path)
// (myyuv_bmp.cpp:9-11, 141-166) and YUV(const BMP&, IYUV) (myyuv_yuv.cpp:186-188,
// 512-523 -> bmp_to_yuv_map, :88-128).  Writes W*H*3/2 bytes (cap checked),
// the frame size, and the header fields the conversion sets.
int ref_bmp_to_iyuv(const char* path, uint8_t* out, uint32_t cap, uint32_t* w, uint32_t* h) {
  try {
    myyuv::BMP bmp(path);
    myyuv::YUV y(bmp, myyuv::YUV::FourccFormats::IYUV);
    *w = y.header.width;
    *h = y.header.height;
    if (y.header.data_size > cap) return 2;
    std::memcpy(out, y.data, y.header.data_size);
    return 0;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return 1;
  }
}

}  // extern "C"
