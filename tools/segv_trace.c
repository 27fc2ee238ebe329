/* LD_PRELOAD-free crash reporter for native test programs: link this file
 * in and a SIGSEGV/SIGABRT prints a symbolised backtrace to stderr. */
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

static void on_fatal(int sig) {
  void *frames[64];
  int n = backtrace(frames, 64);
  fprintf(stderr, "fatal signal %d, backtrace:\n", sig);
  backtrace_symbols_fd(frames, n, 2);
  _exit(128 + sig);
}

__attribute__((constructor)) static void install(void) {
  signal(SIGSEGV, on_fatal);
  signal(SIGABRT, on_fatal);
  signal(SIGBUS, on_fatal);
}
