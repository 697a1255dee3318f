// myyuv_yuv.cpp — the C++ host surface (myyuv::YUV + the DCT codec entry
// points) over the gfx950 C ABI.  Behaviour follows the reference
// (myyuv_lib/myyuv_yuv.cpp:130-536, myyuv_DCT/DCT.cpp:371-488): same header
// normalisation on load, same header rewrites on compress/decompress, same
// std::runtime_error messages.  The per-block work runs on the GPU; this file
// only validates, allocates (new[], as YUV's destructor expects) and copies.
#include "myyuv_yuv.hpp"

#include <cstdlib>
#include <cstring>
#include <fstream>
#include <stdexcept>
#include <vector>

#include <exception>
#include <thread>

#include "myyuv_hip.h"

namespace {

// One codec context per host thread (the C ABI contexts are not shared
// across threads); device from MYYUV_HIP_DEVICE, default 0.
struct ThreadCodec {
  myyuv_hip_handle h = nullptr;
  ~ThreadCodec() {
    if (h) myyuv_hip_destroy(h);
  }
  myyuv_hip_handle get() {
    if (!h) {
      const char* dev = std::getenv("MYYUV_HIP_DEVICE");
      const int rc = myyuv_hip_create(dev ? std::atoi(dev) : 0, &h);
      if (rc) throw std::runtime_error(myyuv_hip_strerror(rc));
    }
    return h;
  }
};
thread_local ThreadCodec t_codec;

[[noreturn]] void fail(int rc) { throw std::runtime_error(myyuv_hip_strerror(rc)); }

uint8_t* dup(const uint8_t* src, size_t n) {
  if (!src) return nullptr;
  uint8_t* p = new uint8_t[n];
  std::memcpy(p, src, n);
  return p;
}

}  // namespace

namespace myyuv {

std::unordered_map<YUV::FourccFormat, YUV::FormatGroup> YUV::yuv_format_group_map = {
    {FourccFormats::IYUV, FormatGroup::PLANAR},
};
std::unordered_map<YUV::FourccFormat, std::array<uint8_t, YUV::max_planes>> YUV::yuv_order_planes_map = {
    {FourccFormats::IYUV, {0, 1, 2, no_plane}},
};
std::unordered_map<YUV::FourccFormat, std::array<uint32_t, 2>> YUV::yuv_resolution_fraction_map = {
    {FourccFormats::IYUV, {2, 2}},
};

// BMP -> IYUV (myyuv_yuv.cpp:88-128): K7 on the GPU (myyuv_gpu_bmp_to_iyuv);
// the raw-image header as the reference's lambda sets it.
std::unordered_map<YUV::FourccFormat, std::function<YUV(const BMP&)>> YUV::bmp_to_yuv_map = {
    {FourccFormats::IYUV,
     [](const BMP& bmp) -> YUV {
       YUV res;
       const uint32_t w = bmp.trueWidth(), h = bmp.trueHeight();
       res.header.fourcc_format = FourccFormats::IYUV;
       res.header.width = w;
       res.header.height = h;
       res.header.data_size = w * h * 3 / 2;
       res.header.data_pos = sizeof(YUVHeader);
       res.data = new uint8_t[res.header.data_size];
       const int rc = myyuv_gpu_bmp_to_iyuv(t_codec.get(), bmp.data, bmp.header.width, bmp.header.height,
                                            bmp.header.bit_count, res.data);
       if (rc) fail(rc);
       return res;
     }},
};

// Registry: the [DCT][IYUV] entries are the drop-in (myyuv_yuv.cpp:130-160).
std::unordered_map<YUV::Compression,
                   std::unordered_map<YUV::FourccFormat, std::function<YUV(const YUV&, const void*, uint32_t)>>>
    YUV::compress_map = {
        {Compressions::DCT,
         {{FourccFormats::IYUV,
           [](const YUV& yuv, const void* params, uint32_t params_size) -> YUV {
             if (params_size != 3)
               throw std::runtime_error("Error compression: incorrect parameters count. 3 parameters required");
             const uint8_t* p = static_cast<const uint8_t*>(params);
             return myyuvDCT::compress_DCT_planar(yuv, {p[0], p[1], p[2]});
           }}}},
};
std::unordered_map<YUV::Compression, std::unordered_map<YUV::FourccFormat, std::function<YUV(const YUV&)>>>
    YUV::decompress_map = {
        {Compressions::DCT,
         {{FourccFormats::IYUV,
           [](const YUV& yuv) -> YUV {
             if (yuv.header.compression_params_size != 3)
               throw std::runtime_error(
                   "Error decompression: incorrect parameters count. 3 parameters required");
             const uint8_t* p = yuv.compression_params;
             return myyuvDCT::decompress_DCT_planar(yuv, {p[0], p[1], p[2]});
           }}}},
};

YUV::YUV(const std::string& path) { load(path); }

YUV::YUV(const BMP& bmp, FourccFormat format) { load(bmp, format); }

// myyuv_yuv.cpp:512-523
void YUV::load(const BMP& bmp, FourccFormat format) {
  if (!bmp.isValid()) throw std::runtime_error("BMP is invalid");
  auto it = bmp_to_yuv_map.find(format);
  if (it == bmp_to_yuv_map.end()) throw std::runtime_error("Incorrect format");
  YUV tmp = it->second(bmp);
  *this = std::move(tmp);
}

YUV::YUV(const YUV& yuv) { *this = yuv; }

YUV& YUV::operator=(const YUV& yuv) {
  if (this == &yuv) return *this;
  uint8_t* d = dup(yuv.data, yuv.header.data_size);
  uint8_t* p = nullptr;
  try {
    p = dup(yuv.compression_params, yuv.header.compression_params_size);
  } catch (...) {
    delete[] d;
    throw;
  }
  delete[] data;
  delete[] compression_params;
  data = d;
  compression_params = p;
  header = yuv.header;
  return *this;
}

YUV::YUV(YUV&& yuv) noexcept { *this = std::move(yuv); }

YUV& YUV::operator=(YUV&& yuv) noexcept {
  std::swap(header, yuv.header);
  std::swap(compression_params, yuv.compression_params);
  std::swap(data, yuv.data);
  return *this;
}

YUV::~YUV() {
  delete[] data;
  delete[] compression_params;
}

bool YUV::isValid() const noexcept {
  const bool params_ok = (header.compression_params_size > 0 && compression_params != nullptr) ||
                         (header.compression == Compressions::NONE && compression_params == nullptr) ||
                         (header.compression_params_size == 0 && compression_params == nullptr);
  return data != nullptr && params_ok && isValidHeader();
}

bool YUV::isValidHeader() const noexcept {
  return header.type[0] == 'Y' && header.type[1] == 'U' &&
         isImplementedFormat(getFourccFormat(), getCompression()) && header.width > 0 &&
         header.height > 0 && header.data_pos >= sizeof(YUVHeader) + header.compression_params_size &&
         header.data_size > 0;
}

bool YUV::isImplementedFormat(FourccFormat format, Compression compression) noexcept {
  if (!yuv_format_group_map.count(format) || !yuv_resolution_fraction_map.count(format)) return false;
  if (compression == Compressions::NONE) return true;
  const auto c = compress_map.find(compression);
  const auto d = decompress_map.find(compression);
  return c != compress_map.end() && d != decompress_map.end() && c->second.count(format) &&
         d->second.count(format);
}

std::array<uint32_t, 2> YUV::getResolutionFraction() const {
  if (!isImplementedFormat(getFourccFormat(), Compressions::NONE))
    throw std::runtime_error("Error. Unimplemented format.");
  return yuv_resolution_fraction_map.at(getFourccFormat());
}

std::array<uint8_t, YUV::max_planes> YUV::getYUVPlanesOrder() const {
  if (!isImplementedFormat(getFourccFormat(), Compressions::NONE))
    throw std::runtime_error("Error. Unimplemented format.");
  const auto it = yuv_order_planes_map.find(getFourccFormat());
  if (it == yuv_order_planes_map.end()) throw std::runtime_error("Error. Planar type unimplemented (?)");
  return it->second;
}

std::array<uint32_t, 2> YUV::getWidthHeightChannel(uint8_t channel) const {
  const auto order = getYUVPlanesOrder();
  if (channel >= max_planes || order[channel] == no_plane) return {0, 0};
  if (channel == 1 || channel == 2) {
    const auto f = getResolutionFraction();
    return {header.width / f[0], header.height / f[1]};
  }
  return {header.width, header.height};
}

std::array<uint32_t, YUV::max_planes> YUV::getFormatSizeBits() const {
  const auto f = getResolutionFraction();
  const auto order = getYUVPlanesOrder();
  const uint32_t frac = f[0] * f[1];
  std::array<uint32_t, max_planes> bits = {8, 8 / frac, 8 / frac, 8};
  for (uint32_t i = 0; i < max_planes; i++)
    if (order[i] == no_plane) bits[i] = 0;
  return bits;
}

uint32_t YUV::getImageSize() const {
  const auto bits = getFormatSizeBits();
  uint64_t total = 0;
  for (uint32_t b : bits) total += (uint64_t)header.width * header.height * b / 8;
  if (total > 0xFFFFFFFFull) throw std::runtime_error("Error. Image too large.");
  return (uint32_t)total;
}

std::array<const uint8_t*, YUV::max_planes> YUV::getYUVPlanes() const {
  const auto order = getYUVPlanesOrder();
  const auto bits = getFormatSizeBits();
  std::array<const uint8_t*, max_planes> res = {nullptr, nullptr, nullptr, nullptr};
  // planes are stored back to back in `order`
  const uint8_t* cur = data;
  for (uint32_t slot = 0; slot < max_planes; slot++) {
    for (uint32_t ch = 0; ch < max_planes; ch++) {
      if (order[ch] != slot) continue;
      if (bits[ch]) res[ch] = cur;
      cur += (size_t)header.width * header.height * bits[ch] / 8;
    }
  }
  return res;
}

std::array<uint8_t*, YUV::max_planes> YUV::getYUVPlanes() {
  const auto c = static_cast<const YUV*>(this)->getYUVPlanes();
  return {const_cast<uint8_t*>(c[0]), const_cast<uint8_t*>(c[1]), const_cast<uint8_t*>(c[2]),
          const_cast<uint8_t*>(c[3])};
}

YUV::FormatGroup YUV::getFormatGroup(FourccFormat format) noexcept {
  const auto it = yuv_format_group_map.find(format);
  return it == yuv_format_group_map.end() ? FormatGroup::UNKNOWN : it->second;
}

YUV YUV::compress(Compression compression, const void* params, uint32_t params_size) const {
  if (getCompression() != Compressions::NONE) throw std::runtime_error("Error already compressed");
  const auto c = compress_map.find(compression);
  if (c == compress_map.end()) throw std::runtime_error("Error this compression is unimplemented");
  const auto f = c->second.find(getFourccFormat());
  if (f == c->second.end()) throw std::runtime_error("Error compression for this format is unimplemented");
  return f->second(*this, params, params_size);
}

YUV YUV::decompress() const {
  if (getCompression() == Compressions::NONE) return *this;
  const auto c = decompress_map.find(getCompression());
  if (c == decompress_map.end()) throw std::runtime_error("Error this decompression is unimplemented");
  const auto f = c->second.find(getFourccFormat());
  if (f == c->second.end()) throw std::runtime_error("Error decompression for this format is unimplemented");
  return f->second(*this);
}

// YUV::load (myyuv_yuv.cpp:485-510): header, params at params_pos, data at
// data_pos; params_pos / data_pos normalised to 64 / 64 + params_size and a
// raw image's data_size recomputed from its geometry.
void YUV::load(const std::string& path) {
  YUV res;
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("Error opening file to read " + path);
  f.read(reinterpret_cast<char*>(&res.header), sizeof(res.header));
  if (!res.isValidHeader()) throw std::runtime_error("Error bad header " + path);
  if (res.header.compression_params_size > 0) {
    f.seekg(res.header.compression_params_pos, std::ios::beg);
    res.compression_params = new uint8_t[res.header.compression_params_size]();
    f.read(reinterpret_cast<char*>(res.compression_params), res.header.compression_params_size);
  }
  f.clear();
  f.seekg(res.header.data_pos, std::ios::beg);
  res.header.compression_params_pos = sizeof(res.header);
  res.header.data_pos = res.header.compression_params_pos + res.header.compression_params_size;
  if (res.getCompression() == Compressions::NONE) res.header.data_size = res.getImageSize();
  res.data = new uint8_t[res.header.data_size]();
  f.read(reinterpret_cast<char*>(res.data), res.header.data_size);
  *this = std::move(res);
}

void YUV::dump(const std::string& path) const {
  std::ofstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("Error opening file to write " + path);
  f.write(reinterpret_cast<const char*>(&header), sizeof(header));
  if (compression_params) f.write(reinterpret_cast<const char*>(compression_params), header.compression_params_size);
  f.write(reinterpret_cast<const char*>(data), header.data_size);
}

}  // namespace myyuv

namespace myyuvDCT {

// compress_DCT_planar (DCT.cpp:371-430): checks, header rewrite
// (compression=1, 3 quality bytes at 64, data at 67), payload from the GPU.
myyuv::YUV compress_DCT_planar(const myyuv::YUV& yuv, const std::array<uint8_t, 3>& params) {
  using myyuv::YUV;
  if (yuv.getFormatGroup() != YUV::FormatGroup::PLANAR)
    throw std::runtime_error("Error compressing: YUV must be planar");
  if (yuv.getCompression() != YUV::Compressions::NONE)
    throw std::runtime_error("Error compressing: can't compress uncompressed YUV");
  for (uint8_t q : params)
    if (q < 1 || q > 100) throw std::runtime_error("Level of quality must be between 1 and 100");
  const uint32_t w = yuv.header.width, h = yuv.header.height;
  std::vector<uint8_t> payload(myyuv_dct_payload_bound(w, h));
  uint32_t size = 0;
  const int rc = myyuv_gpu_dct_compress(t_codec.get(), yuv.data, w, h, params.data(), payload.data(),
                                        (uint32_t)payload.size(), &size);
  if (rc) fail(rc);
  YUV res;
  res.header = yuv.header;
  res.header.compression = YUV::Compressions::DCT;
  res.header.compression_params_size = 3;
  res.header.compression_params_pos = sizeof(myyuv::YUVHeader);
  res.header.data_pos = sizeof(myyuv::YUVHeader) + 3;
  res.header.data_size = size;
  res.compression_params = new uint8_t[3]{params[0], params[1], params[2]};
  res.data = new uint8_t[size];
  std::memcpy(res.data, payload.data(), size);
  return res;
}

namespace {

// Frames `idx` of `frames` (any geometries) on context h: frames of one
// geometry go through one pipelined host batch (myyuv_gpu_dct_compress_frames:
// uploads, kernels and downloads overlapped, one launch per kernel per chunk);
// each payload lands in its YUV's own new[] buffer, sized once its length is
// known.
struct PayloadSink {
  std::vector<myyuv::YUV>* out;
  const std::vector<size_t>* dst;  // batch frame -> index into *out
};
uint8_t* payload_sink(void* user, uint32_t frame, uint32_t size) {
  auto* ps = static_cast<PayloadSink*>(user);
  myyuv::YUV& res = (*ps->out)[(*ps->dst)[frame]];
  delete[] res.data;
  res.data = new uint8_t[size ? size : 1];
  return res.data;
}

void compress_share(myyuv_hip_handle h, const std::vector<const myyuv::YUV*>& frames,
                    const std::vector<size_t>& idx, const std::array<uint8_t, 3>& params,
                    std::vector<myyuv::YUV>& out) {
  using myyuv::YUV;
  std::vector<bool> done(idx.size(), false);
  for (size_t i = 0; i < idx.size(); i++) {
    if (done[i]) continue;
    const uint32_t w = frames[idx[i]]->header.width, hh = frames[idx[i]]->header.height;
    std::vector<size_t> dst;  // indices (into frames / out) of this geometry, in input order
    std::vector<const uint8_t*> src;
    for (size_t j = i; j < idx.size(); j++)
      if (!done[j] && frames[idx[j]]->header.width == w && frames[idx[j]]->header.height == hh) {
        dst.push_back(idx[j]);
        src.push_back(frames[idx[j]]->data);
        done[j] = true;
      }
    std::vector<uint32_t> sizes(dst.size());
    PayloadSink ps{&out, &dst};
    const int rc = myyuv_gpu_dct_compress_frames(h, src.data(), (uint32_t)src.size(), w, hh, params.data(),
                                                 payload_sink, &ps, sizes.data());
    if (rc) fail(rc);
    for (size_t k = 0; k < dst.size(); k++) {
      const YUV& in = *frames[dst[k]];
      YUV& res = out[dst[k]];
      res.header = in.header;  // header rewrite as compress_DCT_planar (DCT.cpp:389-396)
      res.header.compression = YUV::Compressions::DCT;
      res.header.compression_params_size = 3;
      res.header.compression_params_pos = sizeof(myyuv::YUVHeader);
      res.header.data_pos = sizeof(myyuv::YUVHeader) + 3;
      res.header.data_size = sizes[k];
      res.compression_params = new uint8_t[3]{params[0], params[1], params[2]};
    }
  }
}

void check_compressible(const std::vector<const myyuv::YUV*>& frames, const std::array<uint8_t, 3>& params) {
  using myyuv::YUV;
  for (uint8_t q : params)
    if (q < 1 || q > 100) throw std::runtime_error("Level of quality must be between 1 and 100");
  for (const YUV* y : frames) {
    if (y->getFormatGroup() != YUV::FormatGroup::PLANAR)
      throw std::runtime_error("Error compressing: YUV must be planar");
    if (y->getCompression() != YUV::Compressions::NONE)
      throw std::runtime_error("Error compressing: can't compress uncompressed YUV");
  }
}

}  // namespace

std::vector<myyuv::YUV> compress_DCT_planar_batch(const std::vector<const myyuv::YUV*>& frames,
                                                  const std::array<uint8_t, 3>& params) {
  check_compressible(frames, params);
  std::vector<myyuv::YUV> out(frames.size());
  std::vector<size_t> all(frames.size());
  for (size_t i = 0; i < frames.size(); i++) all[i] = i;
  compress_share(t_codec.get(), frames, all, params, out);
  return out;
}

// Frames dealt round-robin over `devices` (frame i -> devices[i % n], the
// multi-GPU sharding of SURVEY.md §8e), one host thread and codec context per
// entry; results in input order.  The first failure is rethrown.
std::vector<myyuv::YUV> compress_DCT_planar_batch(const std::vector<const myyuv::YUV*>& frames,
                                                  const std::array<uint8_t, 3>& params,
                                                  const std::vector<int>& devices) {
  if (devices.empty()) return compress_DCT_planar_batch(frames, params);
  check_compressible(frames, params);
  std::vector<myyuv::YUV> out(frames.size());
  const size_t n = devices.size();
  std::vector<std::exception_ptr> errs(n);
  std::vector<std::thread> th;
  for (size_t d = 0; d < n; d++) {
    th.emplace_back([&, d] {
      myyuv_hip_handle h = nullptr;
      try {
        const int rc = myyuv_hip_create(devices[d], &h);
        if (rc) fail(rc);
        std::vector<size_t> mine;
        for (size_t i = d; i < frames.size(); i += n) mine.push_back(i);
        compress_share(h, frames, mine, params, out);
      } catch (...) {
        errs[d] = std::current_exception();
      }
      if (h) myyuv_hip_destroy(h);
    });
  }
  for (auto& t : th) t.join();
  for (auto& e : errs)
    if (e) std::rethrow_exception(e);
  return out;
}

// decompress_DCT_planar (DCT.cpp:432-488): header rewrite (compression=0,
// params 0/0, data at 64, data_size = image size), planes from the GPU.
myyuv::YUV decompress_DCT_planar(const myyuv::YUV& yuv, const std::array<uint8_t, 3>& params) {
  using myyuv::YUV;
  if (yuv.getFormatGroup() != YUV::FormatGroup::PLANAR)
    throw std::runtime_error("Error decompressing: YUV must be planar");
  for (uint8_t q : params)
    if (q < 1 || q > 100) throw std::runtime_error("Level of quality must be between 1 and 100");
  YUV res;
  res.header = yuv.header;
  res.header.compression = YUV::Compressions::NONE;
  res.header.compression_params_size = 0;
  res.header.compression_params_pos = 0;
  res.header.data_pos = sizeof(myyuv::YUVHeader);
  res.header.data_size = res.getImageSize();
  res.data = new uint8_t[res.header.data_size];
  int64_t bad = -1;
  const int rc = myyuv_gpu_dct_decompress(t_codec.get(), yuv.data, yuv.header.data_size, yuv.header.width,
                                          yuv.header.height, params.data(), res.data, &bad);
  if (rc) fail(rc);
  return res;
}


// Many compressed frames per call.  Each frame is checked as YUV::decompress
// -> decompress_map[DCT][IYUV] -> decompress_DCT_planar would, in input order
// (frames that are not DCT / IYUV, or fail a check, take that single-frame
// path and its error); the DCT frames of one geometry and quality triple
// then go through one pipelined host batch (myyuv_gpu_dct_decompress_frames)
// straight into their results' planes.
std::vector<myyuv::YUV> decompress_DCT_planar_batch(const std::vector<const myyuv::YUV*>& frames) {
  using myyuv::YUV;
  std::vector<YUV> out(frames.size());
  std::vector<size_t> todo;
  for (size_t i = 0; i < frames.size(); i++) {
    const YUV& y = *frames[i];
    bool batchable = y.getCompression() == YUV::Compressions::DCT && y.getFourccFormat() == YUV::FourccFormats::IYUV &&
                     y.header.compression_params_size == 3 && y.compression_params &&
                     y.getFormatGroup() == YUV::FormatGroup::PLANAR;
    for (int p = 0; batchable && p < 3; p++) batchable = y.compression_params[p] >= 1 && y.compression_params[p] <= 100;
    if (batchable)
      todo.push_back(i);
    else
      out[i] = y.decompress();
  }
  std::vector<bool> done(todo.size(), false);
  for (size_t i = 0; i < todo.size(); i++) {
    if (done[i]) continue;
    const YUV& y0 = *frames[todo[i]];
    const uint32_t w = y0.header.width, hh = y0.header.height;
    const uint8_t* q = y0.compression_params;
    std::vector<size_t> grp;
    for (size_t j = i; j < todo.size(); j++) {
      const YUV& y = *frames[todo[j]];
      if (!done[j] && y.header.width == w && y.header.height == hh && std::memcmp(y.compression_params, q, 3) == 0) {
        grp.push_back(todo[j]);
        done[j] = true;
      }
    }
    std::vector<const uint8_t*> src;
    std::vector<uint32_t> sizes;
    std::vector<uint8_t*> dstp;
    for (size_t k : grp) {
      const YUV& y = *frames[k];
      YUV& res = out[k];  // header rewrite as decompress_DCT_planar (DCT.cpp:446-453)
      res.header = y.header;
      res.header.compression = YUV::Compressions::NONE;
      res.header.compression_params_size = 0;
      res.header.compression_params_pos = 0;
      res.header.data_pos = sizeof(myyuv::YUVHeader);
      res.header.data_size = res.getImageSize();
      res.data = new uint8_t[res.header.data_size];
      src.push_back(y.data);
      sizes.push_back(y.header.data_size);
      dstp.push_back(res.data);
    }
    int64_t bad = -1;
    const int rc = myyuv_gpu_dct_decompress_frames(t_codec.get(), src.data(), sizes.data(), (uint32_t)grp.size(), w,
                                                   hh, q, dstp.data(), &bad);
    if (rc) fail(rc);
  }
  return out;
}

}  // namespace myyuvDCT
