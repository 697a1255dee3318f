// myyuv_bmp.hpp — BMP input for the BMP -> IYUV step,
// API-compatible with the reference's myyuv::BMP (myyuv_lib/myyuv_bmp.hpp:8-95):
// the packed file header, the 32-bit colour header, load / dump, and the
// validity rules the conversion relies on.  The colour conversion itself runs
// on the GPU (K7, csrc/k_color.hip) through myyuv_gpu_bmp_to_iyuv; colorData()
// is kept for callers that want the re-oriented pixels on the host.
#pragma once

#include <cstdint>
#include <string>

namespace myyuv {

#pragma pack(push, 1)
struct BMPHeader {  // BITMAPFILEHEADER + BITMAPINFOHEADER, 54 bytes
  uint8_t type[2] = {'B', 'M'};
  uint32_t file_size = 0;
  uint16_t reserved1 = 0;
  uint16_t reserved2 = 0;
  uint32_t data_pos = 0;
  uint32_t header_size = 0;
  int32_t width = 0;
  int32_t height = 0;
  uint16_t planes = 0;
  uint16_t bit_count = 0;
  uint32_t compression = 0;
  uint32_t size_image_for_compression = 0;
  int32_t x_pixels_per_meter = 0;
  int32_t y_pixels_per_meter = 0;
  uint32_t colors_used = 0;
  uint32_t colors_important = 0;
};

struct BMPColorHeader {  // present for 32-bit images, 84 bytes
  uint32_t red_mask = 0x00ff0000;
  uint32_t green_mask = 0x0000ff00;
  uint32_t blue_mask = 0x000000ff;
  uint32_t alpha_mask = 0xff000000;
  uint32_t color_space = 0x73524742;  // sRGB
  uint32_t unused[16] = {0};
};
#pragma pack(pop)
static_assert(sizeof(BMPHeader) == 54, "BMPHeader must be 54 bytes");
static_assert(sizeof(BMPColorHeader) == 84, "BMPColorHeader must be 84 bytes");

class BMP {
 public:
  BMPHeader header;
  BMPColorHeader color_header;
  uint8_t* data = nullptr;  // owned, new[]; the pixel array as stored in the file

  BMP() {}
  explicit BMP(const std::string& path);
  BMP(const BMP& bmp);
  BMP& operator=(const BMP& bmp);
  BMP(BMP&& bmp) noexcept;
  BMP& operator=(BMP&& bmp) noexcept;
  ~BMP();

  uint32_t trueWidth() const noexcept;
  uint32_t trueHeight() const noexcept;
  uint32_t imageSize() const noexcept;  // |w| * |h| * bit_count / 8 (u32, as the reference)
  uint8_t* colorData() const;           // new[] copy, top-down rows, left to right
  uint8_t* colorDataFlipped() const;    // new[] copy, bottom-up rows
  bool isValid() const noexcept;
  bool isValidHeader() const noexcept;
  void load(const std::string& path);
  void dump(const std::string& path) const;
};

}  // namespace myyuv
