// Out-of-core convert / sort / builtin reduce (ooc.cpp): the KV or KMV lives
// in pinned host memory and HBM holds one budget-sized piece at a time.
#pragma once
#include <string>

#include "kv.h"

namespace mrh {

struct OocStats {
  int64_t parts = 0;         // partitions (convert) / range buckets (sort)
  int64_t chunks = 0;        // budget-sized pieces streamed through HBM
  int64_t bytes_staged = 0;  // bytes moved host -> HBM in the partition pass
};

// does an op whose HBM working set is `factor` x `bytes` exceed the budget?
bool needs_ooc(int64_t bytes, int64_t budget, double factor);
// results are host-resident (pinned); inputs may be on the host or the device
KMV ooc_convert(const KV& kv, int64_t budget, at::Device dev, OocStats* st = nullptr);
KV ooc_sort(const KV& kv, int flag, bool by_value, int64_t budget, at::Device dev, OocStats* st = nullptr);
KV ooc_reduce_builtin(const KMV& kmv, const std::string& op, const std::string& dtype, int64_t budget, at::Device dev,
                      OocStats* st = nullptr);

}  // namespace mrh
