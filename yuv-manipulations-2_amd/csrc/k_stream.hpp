// k_stream.hpp — descriptors shared by the stream kernels and the host.
#pragma once
#include <stdint.h>

namespace myyuv_gpu {

#ifndef MYYUV_SCAN_PER_THREAD
#define MYYUV_SCAN_PER_THREAD 16
#endif
constexpr uint32_t kScanPerThread = MYYUV_SCAN_PER_THREAD;
constexpr uint32_t kScanTile = 256 * kScanPerThread;

// Where the u8 chunk-size bytes of each plane live in `src`.
struct ScanSrc {
  uint32_t cum[4];  // plane block boundaries (global block numbering)
  uint32_t pos[3];  // byte offset of plane p's size array in src
};

// Decode-side stream layout, produced on the device by k_parse.
struct StreamDesc {
  uint32_t bad;              // nonzero: header invalid, later kernels skip
  uint32_t sizes_pos[3];     // chunk_size[] of plane p
  uint32_t content_pos[3];   // content[] of plane p
  uint32_t content_size[3];  // declared content_size of plane p
};

}  // namespace myyuv_gpu
