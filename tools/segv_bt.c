// Host-side crash diagnostics: a SIGSEGV / SIGABRT handler that prints the native call stack
// (glibc backtrace) to stderr, then re-raises with the default action.  Loaded with ctypes by
// tools/diag_capture.py before anything touches the GPU; no GPU code here.
//   gcc -O1 -g -shared -fPIC tools/segv_bt.c -o tools/segv_bt.so
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static void handler(int sig) {
  void* frames[96];
  const int n = backtrace(frames, 96);
  static const char head[] = "\n[segv_bt] native stack:\n";
  (void)!write(2, head, sizeof(head) - 1);
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

int segv_bt_install(void) {
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_handler = handler;
  sigemptyset(&sa.sa_mask);
  sa.sa_flags = SA_RESETHAND;
  return sigaction(SIGSEGV, &sa, 0) | sigaction(SIGABRT, &sa, 0);
}
