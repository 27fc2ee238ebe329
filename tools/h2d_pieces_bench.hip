// Host -> HBM upload of a partition made of many pinned pieces (the
// out-of-core convert's upload: ~40 pieces of ~1.6 MB from ~40 pinned chunk
// buffers), three ways:
//   big     one hipMemcpyAsync of the same bytes from one pinned buffer (the floor)
//   pieces  one hipMemcpyAsync per piece (what ooc.cpp does)
//   kernel  one zero-copy gather kernel per partition: the GPU reads every
//           piece straight from pinned host memory (no copy-engine commands)
// measured fresh, then again after the process touched `big_gb` GB of HBM
// (the state after an in-HBM job of ~180 GB, where the pieces path was seen
// to slow down ~4x).
//
//   hipcc --offload-arch=gfx950 -O3 tools/h2d_pieces_bench.hip -o tools/bin/h2d_pieces_bench
//   tools/bin/h2d_pieces_bench [pieces=40] [piece_mb=1.6] [partitions=40] [big_gb=180]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                            \
    }                                                                                          \
  } while (0)

constexpr int MAXP = 64;
struct Table {
  const uint32_t* src[MAXP];
  int64_t dst_off[MAXP];  // in dwords
  int64_t words[MAXP];
  int n;
};

// grid (blocks_per_piece, n): block (x, p) copies its stride of piece p,
// 4 dwords in flight per thread
__global__ __launch_bounds__(256) void k_gather(Table t, uint32_t* __restrict__ dst) {
  const int p = blockIdx.y;
  if (p >= t.n) return;
  const uint32_t* __restrict__ s = t.src[p];
  uint32_t* __restrict__ d = dst + t.dst_off[p];
  const int64_t n = t.words[p];
  const int64_t stride = (int64_t)gridDim.x * 256 * 4;
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += stride) {
    if (i + 3 < n) {
      const uint32_t a = __builtin_nontemporal_load(s + i), b = __builtin_nontemporal_load(s + i + 1);
      const uint32_t c = __builtin_nontemporal_load(s + i + 2), e = __builtin_nontemporal_load(s + i + 3);
      d[i] = a;
      d[i + 1] = b;
      d[i + 2] = c;
      d[i + 3] = e;
    } else {
      for (int64_t j = i; j < n; ++j) d[j] = s[j];
    }
  }
}

double now_ms() {
  using namespace std::chrono;
  return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const int np = argc > 1 ? std::atoi(argv[1]) : 40;
  const double piece_mb = argc > 2 ? std::atof(argv[2]) : 1.6;
  const int nparts = argc > 3 ? std::atoi(argv[3]) : 40;
  const double big_gb = argc > 4 ? std::atof(argv[4]) : 180.0;
  const int64_t pw = ((int64_t)(piece_mb * 1e6) / 4 + 63) / 64 * 64;  // dwords per piece
  const int64_t chunk_words = pw * nparts;                              // one pinned "chunk" per piece index
  std::printf("# %d pieces of %.2f MB per partition, %d partitions (%.2f GB per pass)\n", np, pw * 4 / 1e6, nparts,
              (double)np * nparts * pw * 4 / 1e9);
  std::vector<uint32_t*> chunks(np);
  for (auto& c : chunks) {
    CK(hipHostMalloc((void**)&c, chunk_words * 4, hipHostMallocDefault));
    for (int64_t i = 0; i < chunk_words; i += 1024) c[i] = (uint32_t)i;
  }
  uint32_t* one = nullptr;
  CK(hipHostMalloc((void**)&one, np * pw * 4, hipHostMallocDefault));
  uint32_t* dev = nullptr;
  CK(hipMalloc((void**)&dev, np * pw * 4 * 2));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  auto pass = [&](int mode) {  // one pass over all partitions, ms
    CK(hipStreamSynchronize(s));
    const double t0 = now_ms();
    for (int d = 0; d < nparts; ++d) {
      uint32_t* dst = dev + (d & 1) * np * pw;
      if (mode == 0) {
        CK(hipMemcpyAsync(dst, one, np * pw * 4, hipMemcpyHostToDevice, s));
      } else if (mode == 1) {
        for (int p = 0; p < np; ++p)
          CK(hipMemcpyAsync(dst + p * pw, chunks[p] + d * pw, pw * 4, hipMemcpyHostToDevice, s));
      } else {
        for (int p0 = 0; p0 < np; p0 += MAXP) {
          Table t{};
          t.n = std::min(MAXP, np - p0);
          for (int i = 0; i < t.n; ++i) {
            t.src[i] = chunks[p0 + i] + d * pw;
            t.dst_off[i] = (int64_t)(p0 + i) * pw;
            t.words[i] = pw;
          }
          hipLaunchKernelGGL(k_gather, dim3(16, t.n), dim3(256), 0, s, t, dst);
        }
      }
    }
    const double t1 = now_ms();
    CK(hipStreamSynchronize(s));
    return std::make_pair(now_ms() - t0, t1 - t0);
  };
  auto report = [&](const char* state) {
    const char* names[] = {"big", "pieces", "kernel"};
    for (int mode = 0; mode < 3; ++mode) {
      pass(mode);
      auto [ms, host] = pass(mode);
      const double gb = (double)np * nparts * pw * 4 / 1e9;
      std::printf("%-8s %-7s %8.2f ms  %6.1f GB/s  (host issue %.2f ms)\n", state, names[mode], ms, gb / ms * 1e3, host);
      std::fflush(stdout);
    }
  };
  report("fresh");
  // touch big_gb of HBM in 2 GiB blocks, free it again
  std::vector<void*> blocks;
  const int64_t blk = int64_t(2) << 30;
  for (double got = 0; got < big_gb * 1e9; got += blk) {
    void* p = nullptr;
    if (hipMalloc(&p, blk) != hipSuccess) break;
    CK(hipMemsetAsync(p, 1, blk, s));
    blocks.push_back(p);
  }
  CK(hipStreamSynchronize(s));
  std::printf("# touched %.1f GB of HBM\n", blocks.size() * (double)blk / 1e9);
  report("held");
  for (void* p : blocks) CK(hipFree(p));
  report("freed");
  return 0;
}
