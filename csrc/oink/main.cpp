// oink executable (reference oink/main.cpp:19-28): one process per GPU,
// launched like any torchrun job (RANK / WORLD_SIZE / LOCAL_RANK /
// MASTER_ADDR / MASTER_PORT); world size 1 needs no environment.
//   oink [-in file] [-var name v ...] [-partition NxM ...] [-screen f|none] [-log f|none] [-echo style]
#include <cstdio>
#include <exception>

#include "oink.h"

namespace mrh {
std::shared_ptr<Comm> capi_world();
}

int main(int argc, char** argv) {
  try {
    mrh::oink::Args a(argv + 1, argv + argc);
    return mrh::oink::main_args(mrh::capi_world(), a);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "ERROR: %s\n", e.what());
    // peers must see a failure, not an orderly exit (the exit handler's
    // shutdown handshake is skipped on a poisoned communicator)
    mrh::capi_world()->poison(e.what());
    return 1;
  }
}
