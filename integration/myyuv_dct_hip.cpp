// myyuv_dct_hip.cpp — Seam 2 of INTEGRATION.md: the link-time replacement of
// the reference's DCT codec.  It defines the two functions myyuv_DCT/DCT.hpp:16,25
// declares (and myyuv_yuv.cpp:9-14 declares extern) on top of the MI355X
// codec's C ABI, so the reference's own myyuv_yuv.cpp, myyuv_bmp.cpp and CLI
// link against it instead of myyuv_DCT/DCT.cpp + Huffman.cpp.  Same checks and
// messages as DCT.cpp:371-382 / :432-441; the header rewrites of :389-396 /
// :446-453.  oracle/Makefile `hipref` builds the reference CLI this way;
// tests/test_reference_binding.py runs it.  MYYUV_HIP_PLUGIN_TRACE=1 logs
// each call to stderr.
#include "myyuv_hip.h"            // this repo's include/
#include "myyuv_DCT/DCT.hpp"      // the reference's myyuv_lib/

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
  if (std::getenv("MYYUV_HIP_PLUGIN_TRACE")) std::fprintf(stderr, "myyuv_dct_hip: %s\n", what);
}

void check_quality(const std::array<uint8_t, 3>& params) {
  for (uint32_t i = 0; i < 3; i++)
    if (params[i] < 1 || params[i] > 100) throw std::runtime_error("Level of quality must be between 1 and 100");
}
}  // namespace

namespace myyuvDCT {

myyuv::YUV compress_DCT_planar(const myyuv::YUV& yuv, const std::array<uint8_t, 3>& params) {
  trace("compress_DCT_planar");
  if (yuv.getFormatGroup() != myyuv::YUV::FormatGroup::PLANAR)
    throw std::runtime_error("Error compressing: YUV must be planar");
  if (yuv.getCompression() != myyuv::YUV::Compressions::NONE)
    throw std::runtime_error("Error compressing: can't compress uncompressed YUV");
  check_quality(params);
  std::vector<uint8_t> buf(myyuv_dct_payload_bound(yuv.header.width, yuv.header.height));
  uint32_t size = 0;
  const int rc = myyuv_gpu_dct_compress(ctx.get(), yuv.data, yuv.header.width, yuv.header.height,
                                        params.data(), buf.data(), (uint32_t)buf.size(), &size);
  if (rc) throw std::runtime_error(myyuv_hip_strerror(rc));
  myyuv::YUV res;
  res.header = yuv.header;
  res.header.compression = static_cast<uint16_t>(myyuv::YUV::Compressions::DCT);
  res.header.compression_params_size = 3;
  res.header.compression_params_pos = sizeof(res.header);
  res.header.data_pos = sizeof(res.header) + 3;
  res.header.data_size = size;
  res.compression_params = new uint8_t[3];
  std::copy(params.data(), params.data() + 3, res.compression_params);
  res.data = new uint8_t[size];
  std::copy(buf.begin(), buf.begin() + size, res.data);
  return res;
}

myyuv::YUV decompress_DCT_planar(const myyuv::YUV& yuv, const std::array<uint8_t, 3>& params) {
  trace("decompress_DCT_planar");
  if (yuv.getFormatGroup() != myyuv::YUV::FormatGroup::PLANAR)
    throw std::runtime_error("Error decompressing: YUV must be planar");
  check_quality(params);
  myyuv::YUV res;
  res.header = yuv.header;
  res.header.compression = static_cast<uint16_t>(myyuv::YUV::Compressions::NONE);
  res.header.compression_params_size = 0;
  res.header.compression_params_pos = 0;
  res.header.data_pos = sizeof(yuv.header);
  res.compression_params = nullptr;
  res.header.data_size = yuv.getImageSize();
  res.data = new uint8_t[res.header.data_size];
  int64_t bad = -1;
  const int rc = myyuv_gpu_dct_decompress(ctx.get(), yuv.data, yuv.header.data_size, yuv.header.width,
                                          yuv.header.height, params.data(), res.data, &bad);
  if (rc) throw std::runtime_error(myyuv_hip_strerror(rc));
  return res;
}

}  // namespace myyuvDCT
