// Host <-> device byte counters: every copy the engine makes between pinned /
// pageable / memory-mapped host memory and HBM through its copy helpers
// (kv_to, the out-of-core chunk loads and result drains, spool drains, the
// exchange's host sink) adds its bytes here, so an op's PCIe traffic can be
// read off as the difference of two snapshots (tri_find_mr stages: bytes x
// crossings against the PCIe floor).
#pragma once
#include <ATen/ATen.h>

#include <cstdint>

namespace mrh {

struct XferCount {
  int64_t h2d = 0, d2h = 0;
};
XferCount xfer_count();
// count t's bytes if a copy of t to dst crosses between host and device
void note_xfer(const at::Tensor& t, at::Device dst);
void note_xfer_bytes(bool to_device, int64_t bytes);

}  // namespace mrh
