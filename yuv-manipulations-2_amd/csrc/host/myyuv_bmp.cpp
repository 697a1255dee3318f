// myyuv_bmp.cpp — myyuv::BMP (see myyuv_bmp.hpp).  Behaviour and messages
// follow the reference (myyuv_lib/myyuv_bmp.cpp:9-179): load reads the 54-byte
// header, the colour header only for 32-bit images, then imageSize() bytes at
// data_pos, and normalises data_pos / file_size to what dump() writes.
#include "myyuv_bmp.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <stdexcept>
#include <utility>

namespace myyuv {

BMP::BMP(const std::string& path) { load(path); }

BMP::BMP(const BMP& bmp) { *this = bmp; }

BMP& BMP::operator=(const BMP& bmp) {
  if (this == &bmp) return *this;
  uint8_t* d = nullptr;
  if (bmp.data) {
    const uint32_t n = bmp.imageSize();
    d = new uint8_t[n];
    std::memcpy(d, bmp.data, n);
  }
  delete[] data;
  data = d;
  header = bmp.header;
  color_header = bmp.color_header;
  return *this;
}

BMP::BMP(BMP&& bmp) noexcept { *this = std::move(bmp); }

BMP& BMP::operator=(BMP&& bmp) noexcept {
  std::swap(header, bmp.header);
  std::swap(color_header, bmp.color_header);
  std::swap(data, bmp.data);
  return *this;
}

BMP::~BMP() { delete[] data; }

uint32_t BMP::trueWidth() const noexcept { return (uint32_t)std::abs(header.width); }
uint32_t BMP::trueHeight() const noexcept { return (uint32_t)std::abs(header.height); }
uint32_t BMP::imageSize() const noexcept { return trueWidth() * trueHeight() * header.bit_count / 8; }

// The three orientations colorData accepts (myyuv_bmp.cpp:77-101): width > 0,
// height < 0 is already top-down; height > 0 stores rows bottom-up; width < 0
// (with height > 0) stores the pixels in fully reversed order.
uint8_t* BMP::colorData() const {
  if (!isValid()) throw std::runtime_error("BMP data is invalid");
  const uint32_t n = imageSize(), bpp = header.bit_count / 8, w = trueWidth(), h = trueHeight();
  uint8_t* out = new uint8_t[n];
  if (header.width > 0 && header.height < 0) {
    std::memcpy(out, data, n);
  } else if (header.width < 0 && header.height > 0) {
    for (uint32_t i = 0; i < n; i += bpp) std::memcpy(out + i, data + (n - bpp - i), bpp);
  } else if (header.width > 0 && header.height > 0) {
    const size_t row = (size_t)w * bpp;
    for (uint32_t r = 0; r < h; r++) std::memcpy(out + r * row, data + (size_t)(h - 1 - r) * row, row);
  } else {
    delete[] out;
    throw std::runtime_error("Unaccounted width and height sign");
  }
  return out;
}

uint8_t* BMP::colorDataFlipped() const {
  if (!isValid()) throw std::runtime_error("BMP data is invalid");
  const uint32_t n = imageSize(), bpp = header.bit_count / 8, h = trueHeight();
  uint8_t* out = new uint8_t[n];
  if (header.width > 0 && header.height > 0) {
    std::memcpy(out, data, n);
  } else if (header.width > 0 && header.height < 0) {
    const size_t row = (size_t)trueWidth() * bpp;
    for (uint32_t r = 0; r < h; r++) std::memcpy(out + r * row, data + (size_t)(h - 1 - r) * row, row);
  } else {
    delete[] out;
    throw std::runtime_error("Unaccounted width and height sign");
  }
  return out;
}

bool BMP::isValid() const noexcept { return data != nullptr && isValidHeader(); }

// myyuv_bmp.cpp:125-139: unpadded rows (width % 4 == 0), uncompressed (BI_RGB
// or BI_BITFIELDS with the standard masks), no palette, sRGB.
bool BMP::isValidHeader() const noexcept {
  const BMPColorHeader& c = color_header;
  return header.type[0] == 'B' && header.type[1] == 'M' && header.width % 4 == 0 && header.bit_count > 0 &&
         header.header_size > 0 && (header.compression == 0 || header.compression == 3) &&
         header.colors_used == 0 && header.colors_important == 0 && c.red_mask == 0x00ff0000 &&
         c.green_mask == 0x0000ff00 && c.blue_mask == 0x000000ff &&
         (c.alpha_mask == 0xff000000 || c.alpha_mask == 0) && c.color_space == 0x73524742;
}

void BMP::load(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("Error opening file to read " + path);
  BMP res;
  f.read(reinterpret_cast<char*>(&res.header), sizeof(res.header));
  if (res.header.bit_count == 32) f.read(reinterpret_cast<char*>(&res.color_header), sizeof(res.color_header));
  f.clear();
  f.seekg(res.header.data_pos, std::ios::beg);
  res.header.data_pos = (uint32_t)(sizeof(BMPHeader) + (res.header.bit_count == 32 ? sizeof(BMPColorHeader) : 0));
  const uint32_t n = res.imageSize();
  res.header.file_size = res.header.data_pos + n;
  if (!res.isValidHeader()) throw std::runtime_error("Error bad header " + path);
  res.data = new uint8_t[n]();
  f.read(reinterpret_cast<char*>(res.data), n);
  *this = std::move(res);
}

void BMP::dump(const std::string& path) const {
  if (!isValid()) throw std::runtime_error("BMP data is invalid");
  std::ofstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("Error opening file to write " + path);
  f.write(reinterpret_cast<const char*>(&header), sizeof(header));
  if (header.bit_count == 32) f.write(reinterpret_cast<const char*>(&color_header), sizeof(color_header));
  f.write(reinterpret_cast<const char*>(data), imageSize());
}

}  // namespace myyuv
