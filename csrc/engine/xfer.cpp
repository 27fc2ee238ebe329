#include "xfer.h"

#include <atomic>

namespace mrh {

namespace {
std::atomic<int64_t> g_h2d{0}, g_d2h{0};
}

XferCount xfer_count() { return {g_h2d.load(std::memory_order_relaxed), g_d2h.load(std::memory_order_relaxed)}; }

void note_xfer_bytes(bool to_device, int64_t bytes) {
  if (bytes <= 0) return;
  (to_device ? g_h2d : g_d2h).fetch_add(bytes, std::memory_order_relaxed);
}

void note_xfer(const at::Tensor& t, at::Device dst) {
  if (!t.defined() || t.device().is_cuda() == dst.is_cuda()) return;
  note_xfer_bytes(dst.is_cuda(), (int64_t)t.numel() * (int64_t)t.element_size());
}

}  // namespace mrh
