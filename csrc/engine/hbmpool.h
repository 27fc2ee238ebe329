// HBM page pool: the engine's own device allocator (SURVEY.md §7.2 "page pool
// (mem_request...) -> HbmPool"), the MI355X-side counterpart of the
// reference's page pool (src/mapreduce.cpp:3318-3547: memsize pages, capped by
// maxpage, freed per op with freepage, hi-water stats).
//
// When installed (MRH_HBM_POOL=1 before the first device allocation, or
// gpu_mapreduce_amd.hbm_pool.install()), every device allocation of the
// process — engine arenas, kernel scratch, ATen temporaries — comes from a
// per-device stream-ordered HIP memory pool (hipMallocFromPoolAsync /
// hipFreeAsync) instead of the ATen caching allocator:
//  * stream order: a block freed on stream s is reusable by later work on s
//    at once; blocks used on other streams (record_stream) are freed only
//    behind an event of each of those streams;
//  * hard cap: bytes in use never exceed the cap; an allocation past it fails
//    with a c10::OutOfMemoryError naming the cap ("Cannot allocate page"), the
//    reference's behaviour when maxpage pages are taken. MapReduce ops with a
//    page budget B (maxpage x memsize, or hbm_budget) run under a cap of
//    (bytes in use at op entry) + 2B (output plus working set) + 16 MiB of
//    kernel scratch;
//  * size classes: 512-byte granules to 4 KiB, then 8 classes per power of
//    two; a freed block stays cached for later requests of its class on its
//    stream (no HIP call on that path), or serves another stream's request of
//    that class behind an event, until trim(); more than 1 GiB (and a quarter
//    of the bytes in use) cached goes back to the HIP pool before it grows;
//  * faults: an event query or stream wait of the pool that fails marks the
//    device's pool faulted — the block in question is never reused and every
//    later allocation throws (MRH_FAULT=hip:pool:<rank> injects it), so the
//    op fails and poisons its communicator instead of handing out memory a
//    faulted stream may still write;
//  * big blocks (>= 256 MiB): cut best-fit (2 MiB granules) from hipMalloc'd
//    segments of >= 2 GiB and coalesced with their free neighbours when
//    freed, so the memory held at a job's peak serves any later mix of
//    sizes; every free records an event on each stream that used the block
//    and the next user waits for them. A new segment first hands back the
//    fully free ones when the pool holds over 1.5x the bytes in use;
//  * freepage: trim() returns the pool's cached free memory to the driver;
//  * stats: bytes in use, hi-water mark, reserved bytes, counts.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace mrh::hbm {

struct PoolStats {
  int64_t in_use = 0;    // bytes of live allocations (512-byte granules)
  int64_t peak = 0;      // hi-water mark of in_use since the last reset_peak
  int64_t reserved = 0;  // bytes held from the driver (HIP pool + big-block segments)
  int64_t reserved_peak = 0;  // hi-water mark of reserved (sampled at every growth)
  int64_t cap = 0;       // hard cap on in_use (0: none)
  int64_t allocs = 0, frees = 0, failures = 0;
  int64_t cached = 0;              // bytes of freed blocks held in the caches and the segments' free ranges
  int64_t cross_stream_reuse = 0;  // allocations served from another stream's cache behind an event
  bool faulted = false;            // an event / stream wait of the pool failed: no allocation is served
  int64_t grows = 0;               // allocations the caches could not serve (hipMallocFromPoolAsync)
  double grow_ms = 0;              // host time spent in those calls (a large fresh block maps pages)
  int64_t releases = 0;            // times every cached block went back to the HIP pool
  int64_t oom_retries = 0;         // HIP out-of-memory answers retried after a release + trim
};

// make the pool the process's device allocator; false (and no change) if the
// current allocator has already been initialised by a device allocation
bool install();
// install() unless MRH_HBM_POOL=0 — what Comm construction does on a GPU
// (native programs, C API); false when it did not install
bool install_default();
bool installed();
PoolStats stats(int device);
void reset_peak(int device);
// restart the reserved hi-water mark from what is reserved now
void reset_reserved_peak(int device);
// set the hard cap on bytes in use (0 = none); returns the previous cap
int64_t set_cap(int device, int64_t cap);
// release cached free memory of the pool down to keep_bytes
void trim(int device, int64_t keep_bytes);
// a stream is about to be destroyed: its cached blocks go back to the HIP
// pool, and live or pending blocks that name it (allocated or used on it) are
// re-homed to the null stream, so no later allocation or free records an
// event on, or waits with, a dead stream (the caller has synchronised it).
// Every engine-owned stream calls this before hipStreamDestroy
void forget_stream(hipStream_t s);
// the same without waiting for the stream (an aborted communicator's stream):
// its cached blocks are leaked, not freed
void forget_stream_nosync(hipStream_t s);

// RAII: a MapReduce op's cap (in use at entry + extra bytes) while it runs;
// concurrent ops' caps combine (the tightest is in force)
class OpCap {
 public:
  OpCap(int device, int64_t extra);
  ~OpCap();
  OpCap(const OpCap&) = delete;
  OpCap& operator=(const OpCap&) = delete;

 private:
  int dev_ = -1;
  int64_t prev_ = 0;  // this op's cap
  bool on_ = false;
};

}  // namespace mrh::hbm
