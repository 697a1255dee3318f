// Host <-> device copy strategies for the host-buffer entry points
// (myyuv_gpu_dct_compress / _decompress): an 18 MB frame (4032x3008 IYUV) and
// a 3.4 MB payload between pageable host memory (allocated once, pre-faulted)
// and HBM.
//   direct     hipMemcpyAsync from/to the pageable buffer + stream sync
//   pinned     the DMA alone between a pinned buffer and HBM (the link rate)
//   staged T/C two pinned chunks of C MB, CPU copies between the pageable
//              buffer and the chunk by T threads while the DMA engine moves
//              the other chunk
// Build: hipcc -O2 -std=c++17 -pthread tools/ubench/pcie_copy.cpp -o tools/ubench/pcie_copy
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#define CK(x)                                                          \
  do {                                                                 \
    if ((x) != hipSuccess) {                                           \
      std::fprintf(stderr, "%s failed at %d\n", #x, __LINE__);         \
      std::exit(1);                                                    \
    }                                                                  \
  } while (0)

// a minimal persistent pool: run(dst, src, n) splits one memcpy over T threads
struct Pool {
  int T;
  std::vector<std::thread> th;
  std::mutex mu;
  std::condition_variable cv;
  uint64_t gen = 0;
  bool stop = false;
  uint8_t* dst = nullptr;
  const uint8_t* src = nullptr;
  size_t n = 0;
  std::atomic<int> left{0};
  explicit Pool(int t) : T(t) {
    for (int i = 1; i < T; i++)
      th.emplace_back([this, i] {
        uint64_t seen = 0;
        for (;;) {
          std::unique_lock<std::mutex> lk(mu);
          cv.wait(lk, [&] { return stop || gen != seen; });
          if (stop) return;
          seen = gen;
          lk.unlock();
          part(i);
          left.fetch_sub(1, std::memory_order_release);
        }
      });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto& t : th) t.join();
  }
  void part(int i) {
    const size_t per = (n / T + 63) & ~size_t(63);
    const size_t a = std::min(n, per * i), b = std::min(n, per * (i + 1));
    if (b > a) std::memcpy(dst + a, src + a, b - a);
  }
  void run(uint8_t* d, const uint8_t* s, size_t bytes) {
    if (T == 1) {
      std::memcpy(d, s, bytes);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu);
      dst = d;
      src = s;
      n = bytes;
      left.store(T - 1, std::memory_order_relaxed);
      gen++;
    }
    cv.notify_all();
    part(0);
    while (left.load(std::memory_order_acquire) > 0) std::this_thread::yield();
  }
};

double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const size_t sizes[2] = {18192384, 3363749};
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  uint8_t* dev;
  CK(hipMalloc(&dev, sizes[0]));
  uint8_t* host = static_cast<uint8_t*>(std::aligned_alloc(4096, sizes[0]));
  std::memset(host, 1, sizes[0]);
  uint8_t* pinfull;
  CK(hipHostMalloc(reinterpret_cast<void**>(&pinfull), sizes[0], hipHostMallocDefault));
  std::memset(pinfull, 1, sizes[0]);
  const int reps = 20;
  auto best = [&](auto fn) {
    double b = 1e9;
    for (int r = 0; r < reps; r++) {
      const double t0 = now();
      fn();
      b = std::min(b, now() - t0);
    }
    return b;
  };
  for (size_t n : sizes) {
    std::printf("== %zu bytes\n", n);
    const double th2d = best([&] {
      CK(hipMemcpyAsync(dev, host, n, hipMemcpyHostToDevice, s));
      CK(hipStreamSynchronize(s));
    });
    const double td2h = best([&] {
      CK(hipMemcpyAsync(host, dev, n, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
    });
    std::printf("direct      H2D %7.3f ms %6.1f GB/s   D2H %7.3f ms %6.1f GB/s\n", th2d * 1e3, n / th2d / 1e9,
                td2h * 1e3, n / td2h / 1e9);
    // a fresh buffer per call (what a caller that allocates per frame hands
    // over): pre-faulted by memset for H2D, untouched for D2H; the first call,
    // the median and the best of `reps`
    for (int mode = 0; mode < 2; mode++) {
      std::vector<double> ts;
      for (int r = 0; r < reps; r++) {
        uint8_t* fb = static_cast<uint8_t*>(std::malloc(n));
        if (mode == 0) std::memset(fb, 2, n);
        const double t0 = now();
        CK(hipMemcpyAsync(mode == 0 ? dev : fb, mode == 0 ? fb : dev, n,
                          mode == 0 ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        ts.push_back(now() - t0);
        std::free(fb);
      }
      const double first = ts[0];
      std::sort(ts.begin(), ts.end());
      std::printf("fresh buffer %s first %7.3f ms, median %7.3f ms, best %7.3f ms\n", mode == 0 ? "H2D" : "D2H",
                  first * 1e3, ts[ts.size() / 2] * 1e3, ts[0] * 1e3);
    }
    {  // the reused buffer: first call after allocation, then the rest
      uint8_t* fb = static_cast<uint8_t*>(std::malloc(n));
      std::memset(fb, 3, n);
      std::vector<double> ts;
      for (int r = 0; r < reps; r++) {
        const double t0 = now();
        CK(hipMemcpyAsync(dev, fb, n, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        ts.push_back(now() - t0);
      }
      std::printf("reused buffer H2D: calls 1..4 %7.3f %7.3f %7.3f %7.3f ms, last %7.3f ms\n", ts[0] * 1e3,
                  ts[1] * 1e3, ts[2] * 1e3, ts[3] * 1e3, ts.back() * 1e3);
      std::free(fb);
    }
    for (size_t off : {size_t(1), size_t(16), size_t(32), size_t(64), size_t(4096)}) {
      // a pageable buffer starting `off` bytes past a page boundary (a
      // Python bytes object's data sits 32 bytes into the object)
      uint8_t* base = static_cast<uint8_t*>(std::aligned_alloc(4096, n + 8192));
      std::memset(base, 4, n + 8192);
      const double a = best([&] {
        CK(hipMemcpyAsync(dev, base + off, n, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
      });
      const double b = best([&] {
        CK(hipMemcpyAsync(base + off, dev, n, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
      });
      std::printf("offset %4zu  H2D %7.3f ms   D2H %7.3f ms\n", off, a * 1e3, b * 1e3);
      std::free(base);
    }
    const double ph2d = best([&] {
      CK(hipMemcpyAsync(dev, pinfull, n, hipMemcpyHostToDevice, s));
      CK(hipStreamSynchronize(s));
    });
    const double pd2h = best([&] {
      CK(hipMemcpyAsync(pinfull, dev, n, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
    });
    std::printf("pinned      H2D %7.3f ms %6.1f GB/s   D2H %7.3f ms %6.1f GB/s\n", ph2d * 1e3, n / ph2d / 1e9,
                pd2h * 1e3, n / pd2h / 1e9);
    const double tm = best([&] { std::memcpy(host, pinfull, n); });
    std::printf("memcpy pinned->pageable (1 thread) %7.3f ms %6.1f GB/s\n", tm * 1e3, n / tm / 1e9);
    for (int T : {1, 2, 4, 8}) {
      Pool pool(T);
      for (size_t C : {size_t(1) << 20, size_t(2) << 20, size_t(4) << 20}) {
        uint8_t* pin;
        CK(hipHostMalloc(reinterpret_cast<void**>(&pin), 2 * C, hipHostMallocDefault));
        std::memset(pin, 0, 2 * C);
        hipEvent_t ev[2];
        for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        const double sh2d = best([&] {
          for (size_t off = 0, i = 0; off < n; off += C, i++) {
            const size_t len = std::min(C, n - off);
            uint8_t* b = pin + (i & 1) * C;
            if (i >= 2) CK(hipEventSynchronize(ev[i & 1]));
            pool.run(b, host + off, len);
            CK(hipMemcpyAsync(dev + off, b, len, hipMemcpyHostToDevice, s));
            CK(hipEventRecord(ev[i & 1], s));
          }
          CK(hipStreamSynchronize(s));
        });
        const double sd2h = best([&] {
          const size_t nc = (n + C - 1) / C;
          auto issue = [&](size_t i) {
            const size_t off = i * C, len = std::min(C, n - off);
            CK(hipMemcpyAsync(pin + (i & 1) * C, dev + off, len, hipMemcpyDeviceToHost, s));
            CK(hipEventRecord(ev[i & 1], s));
          };
          issue(0);
          if (nc > 1) issue(1);
          for (size_t i = 0; i < nc; i++) {
            CK(hipEventSynchronize(ev[i & 1]));
            const size_t off = i * C, len = std::min(C, n - off);
            pool.run(host + off, pin + (i & 1) * C, len);
            if (i + 2 < nc) issue(i + 2);
          }
        });
        std::printf("staged T=%d C=%zuMB H2D %7.3f ms %6.1f GB/s   D2H %7.3f ms %6.1f GB/s\n", T, C >> 20,
                    sh2d * 1e3, n / sh2d / 1e9, sd2h * 1e3, n / sd2h / 1e9);
        for (auto& e : ev) CK(hipEventDestroy(e));
        CK(hipHostFree(pin));
      }
    }
  }
  return 0;
}
