// k_chain.hpp — device helpers for kernels that find their chunk offsets
// themselves instead of behind separate scan kernels:
//   * parse_stream: the DCTYUV / DCTYUVPlane header checks (DCT.cpp:130-159,
//     :39-62) in the reference's order, as k_parse did;
//   * chained_prefix: decoupled look-back (single-pass chained scan) over the
//     workgroups of one chain: each workgroup publishes its aggregate, then
//     its inclusive prefix, in a 64-bit status word tagged with the launch
//     epoch (so the status array is never cleared); a wave reads 512
//     predecessors per round.  The tile index is the workgroup index: a
//     workgroup waits only on lower ones, which the in-order dispatch has
//     already placed on the GPU (the scan grids here are a few hundred
//     workgroups, all resident).  (A ticket counter taken with a global atomic
//     instead cost ~60 us for 4,443 workgroups on one address.)
#pragma once
#include "codec_common.hpp"

namespace myyuv_gpu {

constexpr uint32_t kEpochMask = 0x3FFFFFFFu;  // 30-bit epoch in status bits 34..63

struct StreamPos {
  uint32_t sizes_pos[3], content_pos[3], content_size[3];
};

// Returns 0 or the MYYUV_E_* code of the first failing check (k_parse order).
__device__ __forceinline__ int parse_stream(const uint8_t* __restrict__ in, uint32_t size,
                                            const FrameGeom& G, StreamPos& S) {
  auto rd32 = [&](uint64_t a) -> uint32_t {
    return (uint32_t)in[a] | ((uint32_t)in[a + 1] << 8) | ((uint32_t)in[a + 2] << 16) |
           ((uint32_t)in[a + 3] << 24);
  };
  if (size <= 12) return 6;
  uint32_t ps[3];
  for (int p = 0; p < 3; p++) ps[p] = rd32(4 * p);
  // the three plane headers are loaded together (two load round trips in all,
  // not one per plane): positions clamped into the stream, the values used
  // only once the checks below have passed
  uint32_t hw[6];
  {
    const uint64_t last = size - 8ull;
    const uint64_t o[3] = {12ull, 12ull + ps[0], 12ull + ps[0] + ps[1]};
#pragma unroll
    for (int p = 0; p < 3; p++) {
      const uint64_t a = o[p] < last ? o[p] : last;
      hw[2 * p] = rd32(a);
      hw[2 * p + 1] = rd32(a + 4);
    }
  }
  if (12ull + ps[0] + ps[1] + ps[2] > size) return 6;
  uint64_t poff = 12;
  uint32_t hn[3];
  for (int p = 0; p < 3; p++) {
    if (ps[p] <= 8) return 7;
    hn[p] = hw[2 * p];
    const uint32_t hc = hw[2 * p + 1];
    if (hn[p] == 0) return 8;
    if (hc == 0) return 9;
    if (8ull + hn[p] + hc > ps[p]) return 7;
    S.sizes_pos[p] = (uint32_t)(poff + 8);
    S.content_pos[p] = (uint32_t)(poff + 8 + hn[p]);
    S.content_size[p] = hc;
    poff += ps[p];
  }
  for (int p = 0; p < 3; p++)
    if (hn[p] < G.cum[p + 1] - G.cum[p]) return 8;
  return 0;
}

// Exclusive prefix of tile t in the chain starting at tile t0 (wave-uniform
// result; agg = this tile's aggregate, uniform).  Every tile publishes its
// aggregate before looking back, so a look-back is limited by latency, not by
// its predecessors: each round reads the status of kLookBack predecessors at
// once (kLookBack / 64 independent loads per lane) and stops at the nearest
// inclusive prefix.
constexpr int kLookBackPerLane = 8;
__device__ __forceinline__ uint32_t chained_prefix(unsigned long long* status, uint32_t t,
                                                   uint32_t t0, uint32_t agg, uint32_t epoch) {
  const uint32_t lane = threadIdx.x & 63;
  const unsigned long long tag = (unsigned long long)(epoch & kEpochMask) << 34;
  if (lane == 0)
    __hip_atomic_store(&status[t], tag | ((t == t0 ? 2ull : 1ull) << 32) | agg, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  uint32_t excl = 0;
  if (t > t0) {
    int hi = (int)t - 1;  // nearest predecessor not yet accounted for
    while (true) {
      unsigned long long v[kLookBackPerLane];
      bool in[kLookBackPerLane];
#pragma unroll
      for (int k = 0; k < kLookBackPerLane; k++) {
        const int idx = hi - (int)lane - 64 * k;  // distance lane + 64k
        in[k] = idx >= (int)t0;
        v[k] = in[k] ? __hip_atomic_load(&status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                     : 0ull;
      }
      // nearest inclusive prefix (distance d), readiness of everything nearer
      int d = 64 * kLookBackPerLane;
      bool stall = false;
#pragma unroll
      for (int k = 0; k < kLookBackPerLane; k++) {
        const bool ready = in[k] && (v[k] >> 34) == (epoch & kEpochMask) && ((v[k] >> 32) & 3) != 0;
        const uint64_t inclm = __ballot(ready && ((v[k] >> 32) & 3) == 2);
        const uint64_t notready = __ballot(in[k] && !ready);
        const int dk = inclm ? 64 * k + __ffsll((long long)inclm) - 1 : 64 * kLookBackPerLane;
        // lanes of this row nearer than the nearest inclusive found so far
        const int lim = min(d, dk) - 64 * k;  // lanes [0, lim] matter
        const uint64_t need = lim >= 63 ? ~0ull : (lim < 0 ? 0ull : (2ull << lim) - 1ull);
        stall = stall || (notready & need) != 0;
        d = min(d, dk);
      }
      if (stall) {
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      uint32_t part = 0;
#pragma unroll
      for (int k = 0; k < kLookBackPerLane; k++)
        part += (in[k] && (int)lane + 64 * k <= d) ? (uint32_t)v[k] : 0u;
#pragma unroll
      for (int s = 1; s < 64; s <<= 1) part += (uint32_t)__shfl_xor((int)part, s, 64);
      excl += part;
      if (d < 64 * kLookBackPerLane) break;
      hi -= 64 * kLookBackPerLane;
    }
    if (lane == 0)
      __hip_atomic_store(&status[t], tag | (2ull << 32) | (excl + agg), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  return excl;
}

}  // namespace myyuv_gpu
