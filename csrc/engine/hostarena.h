// Pinned host arena for the out-of-core host tier (hostarena.cpp).
//
// The spool's host tier, drained pieces and host copies of device columns are
// pinned host memory. From PyTorch's caching host allocator, the first of
// them pin fresh pages inside the job that first spools (~0.8 s at RMAT-18),
// and blocks cached by earlier jobs of other sizes (an 8 GiB text input, say)
// are not reused. The arena is one segment pinned once, when the process
// chooses (reserve(): at start-up, next to the HBM pool), and carved
// best-fit with coalescing frees; a request that does not fit falls back to
// the caching host allocator.
#pragma once
#include <ATen/ATen.h>

#include <cstdint>

namespace mrh {
namespace hostarena {
// pin `bytes` (rounded up to 2 MiB) now, if no arena exists yet; returns the
// milliseconds it took (0 when one exists or bytes <= 0; -1 when the memory
// could not be pinned: the process goes on without an arena)
double reserve(int64_t bytes);
struct Stats {
  int64_t reserved = 0, in_use = 0, peak = 0, hits = 0, misses = 0;
};
Stats stats();
// a pinned CPU tensor (contiguous, `dtype`, `sizes`): from the arena when it
// fits, else from the caching host allocator
at::Tensor pinned_empty(at::IntArrayRef sizes, at::ScalarType dtype);
}  // namespace hostarena
}  // namespace mrh
