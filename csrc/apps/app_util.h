// Shared bits of the native app programs (csrc/apps): launch/teardown and
// small file helpers.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>

#include "engine/comm.h"

namespace mrh::apps {

inline void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    std::fprintf(stderr, "ERROR: %s: %s\n", what, hipGetErrorString(e));
    std::exit(1);
  }
}

inline int64_t file_size(const std::string& p) {
  FILE* f = std::fopen(p.c_str(), "rb");
  if (!f) return -1;
  std::fseek(f, 0, SEEK_END);
  const int64_t n = std::ftell(f);
  std::fclose(f);
  return n;
}

// End the job: every rank checks in with the rendezvous server (Comm::shutdown)
// and a GPU process leaves through _Exit, before the ROCm libraries' own static
// teardown (the same policy as the C API, csrc/capi/cmapreduce.cpp).
[[noreturn]] inline void finish(const CommPtr& comm, int rc) {
  std::fflush(nullptr);
  if (rc != 0) comm->poison("exited with status " + std::to_string(rc));
  else comm->shutdown();
  if (comm->device().is_cuda()) {
    hipDeviceSynchronize();
    std::_Exit(rc);
  }
  std::exit(rc);
}

}  // namespace mrh::apps
