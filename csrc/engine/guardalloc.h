// Device bounds-check mode (SURVEY.md §5 "Race detection / sanitizers":
// "HIP device-side bounds-check mode (guarded arena writes + canaries)").
//
// GPU AddressSanitizer is not available for gfx950 here, so out-of-bounds
// device writes are caught the way a guarded arena does it: with MRH_GUARD=1
// every HBM allocation of the process goes through a guarded allocator that
// is plugged into ATen in place of the caching allocator
// (torch::cuda::CUDAPluggableAllocator). Each block is
//     [ front canary | user bytes | back canary (+ slack to 256 B) ]
// with both canaries (4 KiB each) filled with a fixed byte pattern and the
// user bytes poisoned (0xA5, so reads of uninitialised memory show up as
// garbage instead of stale zeros). Canaries are verified when a block is
// freed and for every live block at the end of each MapReduce op (the op's
// name is recorded with the first corruption), so a kernel that writes past
// either end of any engine tensor is reported with the op that did it.
//
// Cost: every allocation is a hipMalloc and every free a device sync — a
// diagnostic mode, like MRH_SYNC (serialize) and MRH_CHECK (invariants).
// The allocator must be installed before the process's first HBM allocation:
// the Python package installs it at import, native programs when their first
// Comm / MapReduce is created.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace mrh {
namespace guard {

// MRH_GUARD set to a non-zero value
bool alloc_guard_enabled();
// install the guarded allocator if MRH_GUARD is set (idempotent); returns
// whether it is active. Throws if HBM was already allocated through ATen.
bool install_alloc_guard();
bool alloc_guard_active();

struct GuardReport {
  uint64_t ptr = 0;
  int64_t size = 0;
  int64_t front_bad = 0, back_bad = 0;  // corrupted canary bytes
  std::string alloc_op, found_op;       // op live when allocated / when the corruption was found
};
// check every live block now (device-synchronising); corruptions found are
// added to the report list and printed to stderr
int check_all_blocks(const char* op);
// every corruption found so far in this process
std::vector<GuardReport> guard_reports();
// the op currently running on this thread (recorded with each allocation)
void set_current_op(const char* op);
const char* current_op();
int64_t guarded_blocks_live();

}  // namespace guard
}  // namespace mrh
