// Device functors: the engine's first callback tier (callbacks
// tier 1) — user map / reduce functions written as HIP device code, compiled
// at run time for the GPU (hiprtc, gfx950) into the engine's two-pass emit
// kernels and run over device-resident KV / KMV columns. No ATen tensor
// program and no host round trip: one thread per pair (map) or per key
// (reduce), the emitted records sized by a count pass, placed by exclusive
// scans and written by a second pass (devfn.cpp).
//
// User code defines one of
//   __device__ void mr_map(mrd::Bytes key, mrd::Bytes value, long long index, mrd::Emit& out);
//   __device__ void mr_reduce(mrd::Bytes key, mrd::Values values, mrd::Emit& out);
// and emits with out.emit(kptr, kbytes, vptr, vbytes) or out.emit(k, v) for
// trivially copyable k, v. It must be a pure function of its arguments (it
// runs twice: count, then write). The prelude (kDevicePrelude in devfn.cpp)
// documents mrd::Bytes / mrd::Values / mrd::Emit.
#pragma once
#include <string>
#include <utility>

#include "kv.h"

namespace mrh {
namespace devfn {
// map: pairs [a, b) of kv (b < 0: to the end; on the GPU) through mr_map;
// index = the pair's index in kv
KV map_pairs(const KV& kv, const std::string& code, at::Device dev, int64_t a = 0, int64_t b = -1);
// map over n tasks (no input): mr_map(empty, empty, task, out)
KV map_tasks(int64_t first, int64_t n, const std::string& code, at::Device dev);
// reduce: every key of m through mr_reduce
KV reduce_groups(const KMV& m, const std::string& code, at::Device dev);
// compile only (syntax / type errors come back with the compiler log);
// returns the code object size in bytes. Works without a GPU.
int64_t compile_check(const std::string& code, bool reduce);
// sort-key functor: `__device__ unsigned long long mr_sortkey(mrd::Bytes b)`
// maps each key (or value) to a 64-bit key whose unsigned order is the wanted
// order (a comparator expressed as a key extraction); returns (keys [n],
// row index [n] int32) for the engine's stable radix sort
std::pair<at::Tensor, at::Tensor> sort_keys_of(const at::Tensor& data, const at::Tensor& off, int w, int64_t n,
                                               const std::string& code, at::Device dev);
int64_t compile_check_sortkey(const std::string& code);
// the full source handed to the compiler (prelude + code + kernels)
std::string full_source(const std::string& code, bool reduce);
}  // namespace devfn
}  // namespace mrh
