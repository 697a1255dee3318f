// myyuv_yuv.hpp — C++ host surface of the MI355X codec, API-compatible with the
// reference's myyuv::YUV (myyuv_lib/myyuv_yuv.hpp:13-350) for everything on the
// DCT path: the 64-byte header, load/dump, plane geometry, and the codec
// registry (compress_map / decompress_map, myyuv_yuv.hpp:111,116) whose
// [DCT][IYUV] entries here run the HIP kernels through the C ABI
// (include/myyuv_hip.h), and BMP input (bmp_to_yuv_map[IYUV], YUV(const BMP&),
// myyuv_yuv.hpp:106,143,343), whose colour conversion runs on the GPU too
// (K7).  Out of scope: per-pixel access (getPixel).
#pragma once

#include <array>
#include <cstdint>
#include <functional>
#include <string>
#include <unordered_map>
#include <vector>

#include "myyuv_bmp.hpp"

namespace myyuv {

#pragma pack(push, 1)
// On-disk header of a .myyuv file (64 bytes, little endian).
struct YUVHeader {
  uint8_t type[2] = {'Y', 'U'};
  uint32_t fourcc_format = 0;
  uint32_t data_size = 0;            // payload bytes
  uint16_t compression = 0;          // 0 = none, 1 = DCT
  uint32_t compression_params_size = 0;
  uint32_t compression_params_pos = 0;
  uint32_t width = 0;
  uint32_t height = 0;
  uint32_t data_pos = 0;
  uint8_t unused[32] = {0};
};
#pragma pack(pop)
static_assert(sizeof(YUVHeader) == 64, "YUVHeader must be 64 bytes");

class YUV {
 public:
  YUVHeader header;
  uint8_t* compression_params = nullptr;  // owned, new[]
  uint8_t* data = nullptr;                // owned, new[]

  enum class FormatGroup { UNKNOWN = 0, PACKED, PLANAR, SEMI_PLANAR };
  using FourccFormat = uint32_t;
  struct FourccFormats {
    static constexpr const FourccFormat UNKNOWN = 0;
    static constexpr const FourccFormat IYUV = 0x56555949;
  };
  using Compression = uint16_t;
  struct Compressions {
    static constexpr const Compression NONE = 0;
    static constexpr const Compression DCT = 1;
  };
  static constexpr const uint32_t max_planes = 4;
  static constexpr const uint8_t no_plane = 0xff;

  static std::unordered_map<FourccFormat, FormatGroup> yuv_format_group_map;
  static std::unordered_map<FourccFormat, std::array<uint8_t, max_planes>> yuv_order_planes_map;
  static std::unordered_map<FourccFormat, std::array<uint32_t, 2>> yuv_resolution_fraction_map;
  static std::unordered_map<FourccFormat, std::function<YUV(const BMP&)>> bmp_to_yuv_map;
  static std::unordered_map<Compression,
                            std::unordered_map<FourccFormat, std::function<YUV(const YUV&, const void*, uint32_t)>>>
      compress_map;
  static std::unordered_map<Compression, std::unordered_map<FourccFormat, std::function<YUV(const YUV&)>>>
      decompress_map;

  YUV() {}
  explicit YUV(const std::string& path);
  explicit YUV(const BMP& bmp, FourccFormat format);
  YUV(const YUV& yuv);
  YUV& operator=(const YUV& yuv);
  YUV(YUV&& yuv) noexcept;
  YUV& operator=(YUV&& yuv) noexcept;
  ~YUV();

  bool isValid() const noexcept;
  bool isValidHeader() const noexcept;
  static bool isImplementedFormat(FourccFormat format, Compression compression = Compressions::NONE) noexcept;
  FourccFormat getFourccFormat() const noexcept { return header.fourcc_format; }
  Compression getCompression() const noexcept { return header.compression; }
  uint32_t getWidth() const noexcept { return header.width; }
  uint32_t getHeight() const noexcept { return header.height; }
  uint32_t getDataSize() const noexcept { return header.data_size; }
  std::array<uint32_t, 2> getResolutionFraction() const;
  std::array<uint32_t, 2> getWidthHeightChannel(uint8_t channel) const;
  std::array<uint32_t, max_planes> getFormatSizeBits() const;
  std::array<uint8_t, max_planes> getYUVPlanesOrder() const;
  uint32_t getImageSize() const;
  std::array<const uint8_t*, max_planes> getYUVPlanes() const;
  std::array<uint8_t*, max_planes> getYUVPlanes();
  FormatGroup getFormatGroup() const noexcept { return getFormatGroup(getFourccFormat()); }
  static FormatGroup getFormatGroup(FourccFormat format) noexcept;
  YUV compress(Compression compression, const void* params, uint32_t params_size) const;
  YUV decompress() const;
  bool isCompressed() const noexcept { return getCompression() != Compressions::NONE; }
  void load(const std::string& path);
  void load(const BMP& bmp, FourccFormat format);
  void dump(const std::string& path) const;
};

}  // namespace myyuv

namespace myyuvDCT {
// myyuv_DCT/DCT.hpp:16,25 — same signatures, HIP implementation.
myyuv::YUV compress_DCT_planar(const myyuv::YUV& yuv, const std::array<uint8_t, 3>& params);
myyuv::YUV decompress_DCT_planar(const myyuv::YUV& yuv, const std::array<uint8_t, 3>& params);
// Many frames per call: frames of one geometry share
// one batched launch of every kernel; result i is compress_DCT_planar(*frames[i]).
std::vector<myyuv::YUV> compress_DCT_planar_batch(const std::vector<const myyuv::YUV*>& frames,
                                                  const std::array<uint8_t, 3>& params);
// The same over several devices: frame i on devices[i % n] (frames sharded
// one per GPU round-robin), one host thread and context per
// entry (an id may repeat: several contexts on one device).
std::vector<myyuv::YUV> compress_DCT_planar_batch(const std::vector<const myyuv::YUV*>& frames,
                                                  const std::array<uint8_t, 3>& params,
                                                  const std::vector<int>& devices);
// Many compressed frames per call: result i is frames[i]->decompress(); the
// DCT frames of one geometry and quality go through one pipelined host batch.
std::vector<myyuv::YUV> decompress_DCT_planar_batch(const std::vector<const myyuv::YUV*>& frames);
}  // namespace myyuvDCT
