// Native fatal-signal tracer (host C++, C ABI): on SIGABRT / SIGSEGV / SIGBUS it writes the
// faulting thread's id, name and glibc backtrace to stderr, then hands the signal to the
// previously installed handler (Python's faulthandler, which prints the Python stack).
//
// Why: an abort raised inside HIP / RCCL / a c10d watchdog thread only shows Python frames
// (often of another thread), which does not say which native call aborted.  Enabled by
// tests/conftest.py under CSA_FATAL_TRACE=1 and by the job worker for its ranks.
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <sys/prctl.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cstdio>

namespace {

struct sigaction g_prev[32];

void put(const char* s) {
  ssize_t r = write(2, s, strlen(s));
  (void)r;
}

void on_fatal(int sig, siginfo_t* info, void* ctx) {
  char buf[160];
  char name[17] = {0};
  prctl(PR_GET_NAME, name, 0, 0, 0);
  snprintf(buf, sizeof buf, "\n[csa-fatal] signal %d in thread %ld (%s)\n", sig, (long)syscall(SYS_gettid), name);
  put(buf);
  void* frames[64];
  const int n = backtrace(frames, 64);
  backtrace_symbols_fd(frames, n, 2);
  put("[csa-fatal] end of native backtrace\n");
  struct sigaction& p = g_prev[sig];
  if (p.sa_flags & SA_SIGINFO) {
    if (p.sa_sigaction) p.sa_sigaction(sig, info, ctx);
  } else if (p.sa_handler != SIG_DFL && p.sa_handler != SIG_IGN && p.sa_handler) {
    p.sa_handler(sig);
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

}  // namespace

extern "C" __attribute__((visibility("default"))) int csa_install_fatal_trace() {
  void* warm[2];
  backtrace(warm, 2);            // load libgcc's unwinder now, not inside the handler
  const int sigs[] = {SIGABRT, SIGSEGV, SIGBUS};
  int already = 1;
  for (int s : sigs) {
    struct sigaction cur;
    if (sigaction(s, nullptr, &cur) == 0 && (cur.sa_flags & SA_SIGINFO) && cur.sa_sigaction == on_fatal) continue;
    already = 0;                 // (re-)install in front of whatever a library put there since
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = on_fatal;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    if (sigaction(s, &sa, &g_prev[s]) != 0) return -1;
  }
  return already;
}
