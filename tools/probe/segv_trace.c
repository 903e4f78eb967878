/* Probe helper: loaded with ctypes by tools/probe/*.py, prints the native
 * backtrace of a SIGSEGV / SIGABRT (shared objects + offsets; resolve with
 * addr2line -f -e <lib> <offset>) and re-raises.  Diagnostics only. */
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static void on_fault(int sig) {
  void* frames[64];
  const int n = backtrace(frames, 64);
  const char* msg = "\n[segv_trace] native backtrace:\n";
  (void)!write(2, msg, strlen(msg));
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

__attribute__((constructor)) static void install(void) {
  signal(SIGSEGV, on_fault);
  signal(SIGABRT, on_fault);
}

/* again, after the runtimes loaded by then installed handlers of their own */
void segv_trace_reinstall(void) { install(); }

int segv_trace_installed(void) { return 1; }
