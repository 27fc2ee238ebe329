// Random 4-byte gather ceiling on MI355X (gfx950): the access pattern of the
// PageRank pull gather (csrc/kernels/wavesegred.h k_ws_gather_reduce) without
// its segmented reduce, so its measured rate can be put against what the
// hardware gives for the same pattern.
//
// Every block b serves XCD slot b % 8 (workgroups are dispatched round-robin
// over the 8 XCDs, as the real kernel's schedule assumes), and every slot
// gathers from its own slice of x of `slice` bytes (3 MiB: the real kernel's
// L2 budget per XCD range). A wave owns tiles of 64 lanes x 16 edges; a lane
// issues its 16 gathers at once.
//
// Modes (one line each):
//   stream   : read the int32 index stream only (nontemporal, 16 B per load)
//   gather   : gathers at indices hashed in registers (no index stream) —
//              the pure random-gather rate from an L2-resident slice
//   both     : index stream + gathers (the real kernel's memory traffic)
// Sizes: slice 3 MiB (L2-resident per XCD), 16 KiB (vL1D-resident), 64 MiB
// (past the L2: MALL / HBM).
//
//   hipcc --offload-arch=gfx950 -O3 tools/l2_gather_bench.hip -o tools/bin/l2_gather_bench
//   tools/bin/l2_gather_bench [edges=1073741824]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

constexpr int IT = 16;
constexpr int NT = 256;
constexpr int TILE = 64 * IT;
typedef int v4i __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// uniform in [0, m): multiply-high of a 32-bit hash
__device__ __forceinline__ int32_t in_range(uint32_t h, uint32_t m) { return (int32_t)(((uint64_t)h * m) >> 32); }

__global__ void k_init_idx(int32_t* idx, int64_t n, uint32_t m) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    idx[i] = in_range(mix((uint32_t)i * 2654435761u + 12345u), m);
}

__global__ void k_init_x(float* x, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    x[i] = (float)(i & 1023) * 0.001f;
}

// MODE 0 stream, 1 gather, 2 both. tiles_per_slot tiles of TILE edges per slot;
// slot s reads idx[s * tiles_per_slot * TILE ...) and x + s * slice_elems
template <int MODE>
__global__ __launch_bounds__(NT) void k_bench(const int32_t* __restrict__ idx, const float* __restrict__ x,
                                              int64_t tiles_per_slot, int64_t slice_elems, uint32_t mask,
                                              float* __restrict__ out) {
  const int slot = blockIdx.x & 7;
  const int64_t blocks_per_slot = gridDim.x >> 3;
  const int64_t wave = (int64_t)(blockIdx.x >> 3) * (NT / 64) + (threadIdx.x >> 6);
  const int64_t waves = blocks_per_slot * (NT / 64);
  const int lane = threadIdx.x & 63;
  const float* xs = x + (int64_t)slot * slice_elems;
  const int32_t* is = idx + (int64_t)slot * tiles_per_slot * TILE;
  float acc = 0.f;
  for (int64_t t = wave; t < tiles_per_slot; t += waves) {
    const int64_t L0 = t * TILE + (int64_t)lane * IT;
    int id[IT];
    if (MODE == 1) {
#pragma unroll
      for (int j = 0; j < IT; ++j) id[j] = in_range(mix((uint32_t)(L0 + j)), mask);
    } else {
      const v4i* p = reinterpret_cast<const v4i*>(is + L0);
#pragma unroll
      for (int q = 0; q < IT / 4; ++q) {
        v4i v = __builtin_nontemporal_load(p + q);
        id[4 * q] = v.x;
        id[4 * q + 1] = v.y;
        id[4 * q + 2] = v.z;
        id[4 * q + 3] = v.w;
      }
    }
    if (MODE == 0) {
#pragma unroll
      for (int j = 0; j < IT; ++j) acc += (float)id[j];
    } else {
      float v[IT];
#pragma unroll
      for (int j = 0; j < IT; ++j) v[j] = xs[id[j]];
#pragma unroll
      for (int j = 0; j < IT; ++j) acc += v[j];
    }
  }
  if (acc == 1234.5f) out[blockIdx.x * NT + threadIdx.x] = acc;  // keeps the loads; never true in practice
}

int main(int argc, char** argv) {
  const int64_t edges = argc > 1 ? std::atoll(argv[1]) : (int64_t(1) << 30);
  const int64_t tiles_per_slot = edges / 8 / TILE;
  const int64_t n = tiles_per_slot * TILE * 8;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  std::printf("# %s, %d CUs, %lld edges, IT=%d, %d threads/block, block b -> XCD slot b %% 8\n", prop.gcnArchName, cus,
              (long long)n, IT, NT);
  int32_t* idx;
  float *x, *out;
  const int64_t max_slice = int64_t(64) << 20;
  CK(hipMalloc(&idx, n * 4));
  CK(hipMalloc(&x, 8 * max_slice));
  CK(hipMalloc(&out, (int64_t)cus * 64 * NT * 4));
  k_init_x<<<4096, 256>>>(x, 8 * max_slice / 4);
  CK(hipGetLastError());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int64_t slices[] = {int64_t(16) << 10, int64_t(3) << 20, int64_t(64) << 20};
  const char* names[] = {"stream", "gather", "both"};
  for (int64_t sl : slices) {
    const uint32_t mask = (uint32_t)(sl / 4);  // elements per slice (the index range)
    k_init_idx<<<8192, 256>>>(idx, n, mask);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    for (int mode = 0; mode < 3; ++mode) {
      if (mode == 0 && sl != slices[1]) continue;  // the stream does not depend on the slice
      for (int occ : {8, 16, 32}) {  // blocks per CU (grid = occ x CUs, a multiple of 8)
        const int grid = occ * cus / 8 * 8;
        auto launch = [&] {
          if (mode == 0) k_bench<0><<<grid, NT>>>(idx, x, tiles_per_slot, sl / 4, mask, out);
          else if (mode == 1) k_bench<1><<<grid, NT>>>(idx, x, tiles_per_slot, sl / 4, mask, out);
          else k_bench<2><<<grid, NT>>>(idx, x, tiles_per_slot, sl / 4, mask, out);
        };
        launch();
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        const int reps = 5;
        CK(hipEventRecord(a));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= reps;
        const double greq = n / (ms * 1e-3) / 1e9;
        const double bytes = (mode != 1 ? 4.0 * n : 0.0) + (mode != 0 ? 4.0 * n : 0.0);
        std::printf("%-7s slice %6lld KiB  blocks/CU %2d  %8.3f ms  %7.1f G elements/s  %7.1f GB/s (index + gather bytes)\n",
                    names[mode], (long long)(sl >> 10), occ, ms, greq, bytes / (ms * 1e-3) / 1e9);
        std::fflush(stdout);
      }
    }
  }
  CK(hipFree(idx));
  CK(hipFree(x));
  CK(hipFree(out));
  return 0;
}
