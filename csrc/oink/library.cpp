// C library interface to OINK (see library.h). Errors print and abort, like
// the reference's Error::all / Error::one.
#include "library.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>

#include "oink.h"

namespace mrh {
std::shared_ptr<Comm> capi_world();  // cmapreduce.cpp: the job communicator
}

namespace {
using mrh::oink::Oink;

template <typename F>
auto guard(F&& f) -> decltype(f()) {
  try {
    return f();
  } catch (const std::exception& e) {
    std::fprintf(stderr, "ERROR: %s\n", e.what());
    std::fflush(stderr);
    std::exit(1);
  }
}

// argv of the reference's command line: -partition / -var / -screen / -log / -echo
Oink* make(int argc, char** argv) {
  mrh::oink::Args parts, vars_flat;
  std::vector<std::pair<std::string, mrh::oink::Args>> vars;
  std::string logfile = "log.oink", echo;
  bool screen = true;
  for (int i = 0; i < argc;) {
    std::string a = argv[i];
    if ((a == "-partition" || a == "-p")) {
      int j = i + 1;
      while (j < argc && argv[j][0] != '-') parts.push_back(argv[j++]);
      i = j;
    } else if ((a == "-var" || a == "-v") && i + 2 < argc) {
      int j = i + 2;
      mrh::oink::Args v;
      while (j < argc && argv[j][0] != '-') v.push_back(argv[j++]);
      vars.push_back({argv[i + 1], v});
      i = j;
    } else if ((a == "-log" || a == "-l") && i + 1 < argc) {
      logfile = argv[i + 1];
      i += 2;
    } else if ((a == "-screen" || a == "-sc") && i + 1 < argc) {
      screen = std::string(argv[i + 1]) != "none";
      i += 2;
    } else if ((a == "-echo" || a == "-e") && i + 1 < argc) {
      echo = argv[i + 1];
      i += 2;
    } else {
      throw mrh::oink::Error("Invalid command-line argument " + a);
    }
  }
  Oink::Sink sink;
  if (screen)
    sink = [](const std::string& s) {
      std::fputs(s.c_str(), stdout);
      std::fflush(stdout);
    };
  return new Oink(mrh::capi_world(), parts, sink, logfile, vars, echo);
}
}  // namespace

extern "C" {

void oink_open(int argc, char** argv, void* communicator, void** ptr) {
  *ptr = guard([&]() -> void* {
    if (communicator && communicator != mrh::capi_world().get())
      throw mrh::oink::Error("oink_open: unknown communicator handle");
    return make(argc, argv);
  });
}

void oink_open_no_mpi(int argc, char** argv, void** ptr) {
  *ptr = guard([&]() -> void* { return make(argc, argv); });
}

void oink_close(void* ptr) {
  guard([&]() {
    delete static_cast<Oink*>(ptr);
    return 0;
  });
}

void oink_file(void* ptr, char* str) {
  guard([&]() {
    static_cast<Oink*>(ptr)->file(str ? str : "");
    return 0;
  });
}

char* oink_command(void* ptr, char* str) {
  return guard([&]() -> char* {
    std::string c = static_cast<Oink*>(ptr)->one(str ? str : "");
    return c.empty() ? nullptr : strdup(c.c_str());
  });
}

void oink_free(void* ptr) { std::free(ptr); }
}
