// myyuv_cli.cpp — drop-in for the reference CLI's YUV commands
// (myyuv_cli/main.cpp:138-253) on the MI355X codec:
//   myyuv_cli in.myyuv -info
//   myyuv_cli in.myyuv -compress DCT q [q [q]] -o out.myyuv
//   myyuv_cli in.myyuv -decompress -o out.myyuv
// Same argument rules, quality fill (the last value repeats, main.cpp:64-75),
// same integer-millisecond timing line and "Success!" (main.cpp:11-41, 241),
// same failure mode (usage, then the exception propagates).  BMP input
// (main.cpp:100-136):
//   myyuv_cli in.bmp -info
//   myyuv_cli in.bmp -to_yuv IYUV -o out.myyuv   (conversion on the GPU, K7)
// and, beyond the reference CLI, many frames per invocation (SURVEY.md §8f
// row 2; frames of one geometry share batched kernel launches):
//   myyuv_cli -batch-compress DCT Q [Q [Q]] [-devices D0,D1,...] -o OUTDIR IN.myyuv...
//     (-devices: frames dealt round-robin over those GPUs, one host thread each)
//   myyuv_cli -batch-decompress -o OUTDIR IN.myyuv...
// each output is OUTDIR/<input file name>, byte-identical to the per-file
// command's.
#include <chrono>
#include <cstring>
#include <fstream>
#include <functional>
#include <iostream>
#include <stdexcept>
#include <string>
#include <vector>

#include "myyuv_yuv.hpp"

namespace {

float elapsed_ms(const std::function<void()>& f) {
  const auto t0 = std::chrono::high_resolution_clock::now();
  f();
  const auto t1 = std::chrono::high_resolution_clock::now();
  return (float)std::chrono::duration_cast<std::chrono::milliseconds>(t1 - t0).count();
}

void usage() {
  std::cout << "myyuv_cli (MI355X DCT codec): inspect and DCT-compress/decompress .myyuv images.\n"
            << "Usage:\n"
            << "  myyuv_cli IMAGE.myyuv -info\n"
            << "  myyuv_cli IMAGE.myyuv -compress DCT Q [Q [Q]] -o OUT.myyuv   (Q in 1..100, per plane Y U V)\n"
            << "  myyuv_cli IMAGE.myyuv -decompress -o OUT.myyuv\n"
            << "  myyuv_cli IMAGE.bmp -info\n"
            << "  myyuv_cli IMAGE.bmp -to_yuv IYUV -o OUT.myyuv\n"
            << "  myyuv_cli -batch-compress DCT Q [Q [Q]] [-devices D0,D1,...] -o OUTDIR IMAGE.myyuv...\n"
            << "  myyuv_cli -batch-decompress -o OUTDIR IMAGE.myyuv...\n"
            << "\nYUV formats:\nIYUV\n\nCompression formats for YUV:\nDCT\n"
            << "\nExample:\n  myyuv_cli image.myyuv -compress DCT 50 -o image-DCT-50.myyuv\n";
}

myyuv::YUV compress_dct(const myyuv::YUV& yuv, const std::vector<std::string>& params) {
  if (params.size() > 3)
    throw std::runtime_error("Error. Too many compression parameters. Can't be more than 3 parameters.");
  if (params.empty()) throw std::runtime_error("Error. Too few compression parameters. Must be at least one.");
  uint8_t q[3];
  for (size_t i = 0; i < 3; i++) {
    const int v = std::stoi(params[i < params.size() ? i : params.size() - 1]);
    if (v < 1 || v > 100)
      throw std::runtime_error("Error. Compression parameters for DCT must range between [1..100].");
    q[i] = (uint8_t)v;
  }
  return yuv.compress(myyuv::YUV::Compressions::DCT, q, 3);
}

int run_yuv(const myyuv::YUV& yuv, size_t a, const std::vector<std::string>& args) {
  const std::string& cmd = args[a];
  if (cmd == "-info") {
    const auto& h = yuv.header;
    std::cout << "Type: " << h.type[0] << h.type[1] << '\n'
              << "FourCC Format: 0x" << std::hex << h.fourcc_format << std::dec << '\n'
              << "File size: " << (sizeof(h) + h.compression_params_size + h.data_size) << '\n'
              << "Data size: " << h.data_size << '\n'
              << "Compression: " << h.compression << '\n'
              << "Compression params size: " << h.compression_params_size << '\n'
              << "Width: " << h.width << '\n'
              << "Height: " << h.height << '\n'
              << "Valid: " << yuv.isValid() << '\n';
    return 0;
  }
  if (cmd == "-compress") {
    a++;
    if (a >= args.size()) {
      std::cout << "Invalid arguments. Specify compression algorithm, compression parameters and output.\n";
      usage();
      return 1;
    }
    const std::string algo = args[a++];
    if (algo != "DCT") throw std::runtime_error("Compression not registered: " + algo);
    std::vector<std::string> params;
    while (a < args.size() && args[a] != "-o") params.push_back(args[a++]);
    a++;
    if (a >= args.size()) {
      std::cout << "Invalid argument, last arguments must be `-o /path/to/new_image.myyuv`\n";
      usage();
      return 1;
    }
    std::string label = " ";
    for (const auto& p : params) label += p + " ";
    myyuv::YUV out;
    const float ms = elapsed_ms([&] { out = compress_dct(yuv, params); });
    std::cout << "YUV DCT compression (" << label << ") : " << ms << " ms\n";
    out.dump(args[a]);
    return 0;
  }
  if (cmd == "-decompress") {
    if (!yuv.isCompressed()) {
      std::cout << "Nothing to decompress, image is not compressed\n";
      return 1;
    }
    a++;
    if (args.size() != a + 2) {
      std::cout << "Invalid arguments amount. " << (a + 2) << " is required\n";
      usage();
      return 1;
    }
    if (args[a] != "-o") {
      std::cout << a << " argument must be `-o` instead of " << args[a] << '\n';
      usage();
      return 1;
    }
    myyuv::YUV out;
    const float ms = elapsed_ms([&] { out = yuv.decompress(); });
    std::cout << "YUV DCT decompression : " << ms << " ms\n";
    out.dump(args[a + 1]);
    return 0;
  }
  std::cout << "Invalid command " << cmd << '\n';
  usage();
  return 1;
}

int run_bmp(const myyuv::BMP& bmp, size_t a, const std::vector<std::string>& args) {
  const std::string& cmd = args[a];
  if (cmd == "-info") {
    const auto& h = bmp.header;
    std::cout << "Type: " << h.type[0] << h.type[1] << '\n'
              << "File size: " << h.file_size << '\n'
              << "Data size: " << h.width * h.height * h.bit_count / 8 << '\n'
              << "Width: " << h.width << '\n'
              << "Height: " << h.height << '\n'
              << "Bit count: " << h.bit_count << '\n'
              << "Valid: " << bmp.isValid() << '\n';
    return 0;
  }
  if (cmd == "-to_yuv") {
    if (args.size() != a + 4) {
      std::cout << "Invalid arguments amount. " << (a + 4) << " is required\n";
      usage();
      return 1;
    }
    if (args[a + 1] != "IYUV") throw std::runtime_error("Format is not registered: " + args[a + 1]);
    if (args[a + 2] != "-o") {
      std::cout << (a + 2) << " argument must be `-o` instead of " << args[a + 2] << '\n';
      usage();
      return 1;
    }
    myyuv::YUV out;
    const float ms = elapsed_ms([&] { out = myyuv::YUV(bmp, myyuv::YUV::FourccFormats::IYUV); });
    std::cout << "BMP to YUV (" << args[a + 1] << ") : " << ms << " ms\n";
    out.dump(args[a + 3]);
    return 0;
  }
  std::cout << "Invalid command " << cmd << '\n';
  usage();
  return 1;
}

std::string base_name(const std::string& path) {
  const size_t k = path.find_last_of('/');
  return k == std::string::npos ? path : path.substr(k + 1);
}

// -batch-compress DCT Q [Q [Q]] -o OUTDIR FILES... / -batch-decompress -o OUTDIR FILES...
int run_batch(const std::vector<std::string>& args) {
  const bool comp = args[1] == "-batch-compress";
  size_t a = 2;
  std::vector<std::string> params;
  std::vector<int> devices;
  if (comp) {
    if (a >= args.size() || args[a] != "DCT")
      throw std::runtime_error("Compression not registered: " + (a < args.size() ? args[a] : std::string()));
    a++;
    while (a < args.size() && args[a] != "-o") {
      if (args[a] == "-devices" && a + 1 < args.size()) {  // frames dealt round-robin over these GPUs
        std::string list = args[a + 1];
        for (size_t k = 0; k <= list.size();) {
          const size_t e = list.find(',', k);
          devices.push_back(std::stoi(list.substr(k, e == std::string::npos ? std::string::npos : e - k)));
          if (e == std::string::npos) break;
          k = e + 1;
        }
        a += 2;
        continue;
      }
      params.push_back(args[a++]);
    }
  }
  if (a + 2 >= args.size() || args[a] != "-o") {
    std::cout << "Invalid arguments. Expected -o OUTDIR followed by input files\n";
    usage();
    return 1;
  }
  const std::string outdir = args[a + 1];
  std::vector<myyuv::YUV> in;
  std::vector<std::string> names;
  for (size_t i = a + 2; i < args.size(); i++) {
    names.push_back(base_name(args[i]));
    // outputs are OUTDIR/<input file name>: two inputs with one name would
    // overwrite each other
    for (size_t j = 0; j + 1 < names.size(); j++)
      if (names[j] == names.back())
        throw std::runtime_error("Error. Two batch inputs share the file name " + names.back());
  }
  for (size_t i = a + 2; i < args.size(); i++) in.emplace_back(args[i]);
  std::vector<myyuv::YUV> out;
  const float ms = elapsed_ms([&] {
    if (comp) {
      uint8_t q[3];
      if (params.empty()) throw std::runtime_error("Error. Too few compression parameters. Must be at least one.");
      if (params.size() > 3)
        throw std::runtime_error("Error. Too many compression parameters. Can't be more than 3 parameters.");
      for (size_t i = 0; i < 3; i++) {
        const int v = std::stoi(params[i < params.size() ? i : params.size() - 1]);
        if (v < 1 || v > 100)
          throw std::runtime_error("Error. Compression parameters for DCT must range between [1..100].");
        q[i] = (uint8_t)v;
      }
      std::vector<const myyuv::YUV*> ptrs;
      for (const auto& y : in) ptrs.push_back(&y);
      out = myyuvDCT::compress_DCT_planar_batch(ptrs, {q[0], q[1], q[2]}, devices);
    } else {
      std::vector<const myyuv::YUV*> ptrs;
      for (const auto& y : in) ptrs.push_back(&y);
      out = myyuvDCT::decompress_DCT_planar_batch(ptrs);
    }
  });
  std::cout << (comp ? "YUV DCT batch compression" : "YUV DCT batch decompression") << " (" << in.size()
            << " frames) : " << ms << " ms\n";
  for (size_t i = 0; i < out.size(); i++) out[i].dump(outdir + "/" + names[i]);
  return 0;
}

int run(int argc, char* argv[]) {
  if (argc <= 2) {
    usage();
    return 0;
  }
  const std::vector<std::string> args(argv, argv + argc);
  if (args[1] == "-batch-compress" || args[1] == "-batch-decompress") {
    const int rc = run_batch(args);
    if (rc == 0) std::cout << "Success!\n";
    return rc;
  }
  const std::string& path = args[1];
  char magic[2] = {0, 0};
  {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("Error opening file to read " + path);
    f.read(magic, 2);
  }
  int rc;
  if (magic[0] == 'Y' && magic[1] == 'U') {
    rc = run_yuv(myyuv::YUV(path), 2, args);
  } else if (magic[0] == 'B' && magic[1] == 'M') {
    rc = run_bmp(myyuv::BMP(path), 2, args);
  } else {
    throw std::runtime_error("Unknown image format (magic) " + path);
  }
  if (rc == 0) std::cout << "Success!\n";
  return rc;
}

}  // namespace

int main(int argc, char* argv[]) {
  try {
    return run(argc, argv);
  } catch (...) {
    usage();
    throw;
  }
}
