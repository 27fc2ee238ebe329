// Failure detection, fault injection and invariant checking for the native
// engine (SURVEY.md §5 "Failure detection / fault injection", "Race detection").
//
// The reference has none of this: Error::all/one print and MPI_Abort
// (src/error.cpp:33-57), fread/fwrite failures are warnings, and the only
// resilience is aggregate's receive-overflow scale-back (src/mapreduce.cpp:
// 498-513). Here:
//
//  * bounded waits: every collective runs with a timeout (MRH_COMM_TIMEOUT
//    seconds, default 600) — the RCCL process group's watchdog and the
//    rendezvous store both honour it — so a dead peer surfaces as an error on
//    the surviving ranks instead of a hang;
//  * HBM exhaustion: the heavy device ops (convert, aggregate, sorts, builtin
//    reduces, clone) run under oom_retry(): on a HIP out-of-memory error every
//    OTHER live MapReduce object on the device is spilled to pinned host DRAM,
//    the caching allocator releases its free blocks, and the op is retried
//    once. Spilled objects come back to HBM on their next op;
//  * fault injection (tests): MRH_FAULT="kind:op:rank[:nth]" fires at the
//    nth (default 1st) entry of MapReduce op `op` on rank `rank` (-1 = every
//    rank): kind "abort" ends the process (exit status 3, no cleanup, like a
//    crashed rank), "throw" raises an error, "oom" raises a HIP OOM inside the
//    op's oom_retry (exercising the spill-and-retry path), "hip" makes the
//    checked HIP call at site `op` (hip_check) fail with hipErrorUnknown;
//  * checked HIP calls: every HIP call on a data path goes through
//    hip_check(call, site, rank) — a failed copy, event or stream wait is an
//    exception (which poisons the job's communicator on the way out), never a
//    silently ignored status and garbage output;
//  * check mode: MRH_CHECK=1 validates the KV/KMV invariants (offset arrays
//    monotone and consistent with the arenas, segment array covering every
//    value, widths) after every op, naming the op that broke them.
#pragma once
#include <c10/util/Exception.h>
#include <hip/hip_runtime.h>

#include <functional>
#include <string>

#include "kv.h"

namespace mrh {

class MapReduce;

namespace guard {

// seconds every collective may block before it is declared failed
int comm_timeout_seconds();

// fault injection hook at op entry ("abort" / "throw" kinds)
void fault_point(const char* op, int rank);
// throws (naming `site` and the rank) unless e == hipSuccess; an armed
// MRH_FAULT=hip:site:rank turns a success into hipErrorUnknown
void hip_check(hipError_t e, const char* site, int rank);
// true if an injected OOM is due for this op on this rank (consumed)
bool fault_oom(const char* op, int rank);

bool check_enabled();
// throws std::runtime_error naming `op` if an invariant does not hold
void check_kv(const KV& kv, const char* op);
void check_kmv(const KMV& kmv, const char* op);

// op trace (MRH_TRACE=path): one JSON line per MapReduce op to path.<rank>
// {"op","instance","depth","t0","ms","kv","kmv","bytes","sent","recv"}; device
// work is synchronised at op boundaries while tracing (diagnostic mode)
bool trace_enabled();
void trace_op(int rank, const char* op, int instance, int depth, double t0, double ms, int64_t nkv, int64_t nkmv,
              int64_t bytes, int64_t sent, int64_t recv);

// live MapReduce objects (for spill-on-OOM)
void register_mr(MapReduce* mr);
void unregister_mr(MapReduce* mr);
// spill every live MR except `keep` that holds device data on `dev`;
// returns how many were spilled
int spill_others(const MapReduce* keep, at::Device dev);

}  // namespace guard

// run f(); on HIP OOM spill the other MapReduce objects and retry once
template <typename F>
auto oom_retry(MapReduce* self, at::Device dev, int rank, const char* op, F&& f) -> decltype(f()) {
  try {
    if (guard::fault_oom(op, rank))
      TORCH_CHECK_WITH(OutOfMemoryError, false, "HIP out of memory (injected by MRH_FAULT in ", op, ")");
    return f();
  } catch (const c10::OutOfMemoryError&) {
    guard::spill_others(self, dev);
    return f();
  }
}

}  // namespace mrh
