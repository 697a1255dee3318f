// myyuv_hip_plugin.cpp — Seam 1 of INTEGRATION.md: added to the reference's
// own myyuv_lib (its sources untouched), this translation unit replaces the CPU
// entries of the plugin tables at static-init time with the MI355X codec's C
// ABI (include/myyuv_hip.h, libmyyuv_hip.so):
//   YUV::compress_map[DCT][IYUV] / decompress_map[DCT][IYUV]  myyuv_yuv.hpp:111,116 (myyuv_yuv.cpp:130-160)
//   YUV::bmp_to_yuv_map[IYUV]                                  myyuv_yuv.hpp:106 (myyuv_yuv.cpp:88-128)
// Link it after the reference's objects (its initializer must run after the
// maps' own, myyuv_yuv.cpp:130: static initialization follows link order).
// oracle/Makefile `hipref` builds the reference CLI and library this way;
// tests/test_reference_binding.py runs them.  MYYUV_HIP_PLUGIN_TRACE=1 logs
// each dispatch to stderr.
#include "myyuv_hip.h"          // this repo's include/
#include "myyuv_yuv.hpp"        // the reference's myyuv_lib/

#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <vector>

namespace {
thread_local struct Ctx {
  myyuv_hip_handle h = nullptr;
  ~Ctx() { if (h) myyuv_hip_destroy(h); }
  myyuv_hip_handle get() {
    if (!h) { int rc = myyuv_hip_create(0, &h); if (rc) throw std::runtime_error(myyuv_hip_strerror(rc)); }
    return h;
  }
} ctx;

void trace(const char* what) {
  if (std::getenv("MYYUV_HIP_PLUGIN_TRACE")) std::fprintf(stderr, "myyuv_hip plugin: %s\n", what);
}

myyuv::YUV gpu_compress(const myyuv::YUV& yuv, const void* params, uint32_t n) {
  trace("compress");
  if (n != 3) throw std::runtime_error("Error compression: incorrect parameters count. 3 parameters required");
  const uint8_t* q = static_cast<const uint8_t*>(params);
  std::vector<uint8_t> buf(myyuv_dct_payload_bound(yuv.header.width, yuv.header.height));
  uint32_t size = 0;
  int rc = myyuv_gpu_dct_compress(ctx.get(), yuv.data, yuv.header.width, yuv.header.height, q,
                                  buf.data(), (uint32_t)buf.size(), &size);
  if (rc) throw std::runtime_error(myyuv_hip_strerror(rc));
  myyuv::YUV res;                                   // header rewrite as DCT.cpp:389-396
  res.header = yuv.header;
  res.header.compression = myyuv::YUV::Compressions::DCT;
  res.header.compression_params_size = 3;
  res.header.compression_params_pos = sizeof(res.header);
  res.header.data_pos = sizeof(res.header) + 3;
  res.header.data_size = size;
  res.compression_params = new uint8_t[3]{q[0], q[1], q[2]};
  res.data = new uint8_t[size];                     // YUV owns new[] memory
  std::copy(buf.begin(), buf.begin() + size, res.data);
  return res;
}

myyuv::YUV gpu_decompress(const myyuv::YUV& yuv) {
  trace("decompress");
  if (yuv.header.compression_params_size != 3)
    throw std::runtime_error("Error decompression: incorrect parameters count. 3 parameters required");
  myyuv::YUV res;                                   // header rewrite as DCT.cpp:446-453
  res.header = yuv.header;
  res.header.compression = myyuv::YUV::Compressions::NONE;
  res.header.compression_params_size = 0;
  res.header.compression_params_pos = 0;
  res.header.data_pos = sizeof(res.header);
  res.header.data_size = res.getImageSize();
  res.data = new uint8_t[res.header.data_size];
  int64_t bad = -1;
  int rc = myyuv_gpu_dct_decompress(ctx.get(), yuv.data, yuv.header.data_size, yuv.header.width,
                                    yuv.header.height, yuv.compression_params, res.data, &bad);
  if (rc) throw std::runtime_error(myyuv_hip_strerror(rc));
  return res;
}

myyuv::YUV gpu_bmp_to_iyuv(const myyuv::BMP& bmp) {
  trace("bmp_to_iyuv");
  myyuv::YUV res;                                   // raw-image header as the reference's lambda
  const uint32_t w = bmp.trueWidth(), h = bmp.trueHeight();
  res.header.fourcc_format = myyuv::YUV::FourccFormats::IYUV;
  res.header.width = w;
  res.header.height = h;
  res.header.data_size = w * h * 3 / 2;
  res.header.data_pos = sizeof(myyuv::YUVHeader);
  res.data = new uint8_t[res.header.data_size];
  int rc = myyuv_gpu_bmp_to_iyuv(ctx.get(), bmp.data, bmp.header.width, bmp.header.height,
                                 bmp.header.bit_count, res.data);
  if (rc) throw std::runtime_error(myyuv_hip_strerror(rc));
  return res;
}

const bool registered = [] {
  using Y = myyuv::YUV;
  Y::compress_map[Y::Compressions::DCT][Y::FourccFormats::IYUV] = gpu_compress;
  Y::decompress_map[Y::Compressions::DCT][Y::FourccFormats::IYUV] = gpu_decompress;
  Y::bmp_to_yuv_map[Y::FourccFormats::IYUV] = gpu_bmp_to_iyuv;
  return true;
}();
}  // namespace
