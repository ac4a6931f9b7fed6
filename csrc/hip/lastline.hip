// A last line for a process that dies in an optional phase.
//
// bench.py prints ONE JSON line, and only after its optional post-headline
// phase (the ZeRO-1 collectives A/B, bench/flagship.py collectives_ab) has
// run, because the A/B's result goes into that line.  That phase drives the
// copy-engine pulls over IPC-mapped peer memory; if it kills the process (a
// GPU memory fault aborts inside the HIP runtime, a peer's death makes the
// elastic agent send SIGTERM), the headline measured before it must not be
// lost with it.  Rank 0 arms a pre-rendered copy of the line (its A/B field
// saying which signal ended the run); on a fatal signal the handler writes it
// with write(2) -- the only async-signal-safe way out -- and leaves with
// _exit(code).  Other ranks arm an empty line: they only leave.
//
// Host-only code; no device code in this file.
#include <signal.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <atomic>
#include <mutex>

namespace {

constexpr int kSignals[] = {SIGSEGV, SIGBUS, SIGABRT, SIGFPE, SIGILL, SIGTERM};
constexpr int kNumSignals = sizeof(kSignals) / sizeof(kSignals[0]);

char* g_text = nullptr;  // owned; replaced only while disarmed
long g_len = 0;
long g_signo_at = -1;    // two characters overwritten with the signal number
int g_code = 0;
std::atomic<int> g_fired{0};
bool g_armed = false;
struct sigaction g_prev[kNumSignals];
std::mutex g_mu;  // arm / disarm from several threads (the bench's watchdog and main thread)

void write_all(int fd, const char* p, long n) {
  while (n > 0) {
    ssize_t w = write(fd, p, static_cast<size_t>(n));
    if (w <= 0) return;
    p += w;
    n -= w;
  }
}

void on_signal(int sig) {
  if (g_fired.exchange(1) != 0) _exit(g_code);  // a second signal during the write: just leave
  if (g_len > 0) {
    if (g_signo_at >= 0 && g_signo_at + 1 < g_len) {
      g_text[g_signo_at] = static_cast<char>('0' + (sig / 10) % 10);
      g_text[g_signo_at + 1] = static_cast<char>('0' + sig % 10);
    }
    write_all(1, g_text, g_len);
  }
  static const char msg[] = "[lastline] fatal signal in an optional phase; leaving with the armed status\n";
  write_all(2, msg, sizeof(msg) - 1);
  _exit(g_code);
}

void restore() {
  if (!g_armed) return;
  for (int i = 0; i < kNumSignals; ++i) sigaction(kSignals[i], &g_prev[i], nullptr);
  g_armed = false;
}

}  // namespace

extern "C" {

// Arm (or re-arm) the handler: `text` (len bytes, newline included by the
// caller; len 0 = write nothing) is written to stdout on SIGSEGV / SIGBUS /
// SIGABRT / SIGFPE / SIGILL / SIGTERM, then the process exits with `code`.
// signo_at >= 0: offset of two placeholder characters that receive the
// signal number.  Returns 0, or -1 if a handler could not be installed.
int toa_lastline_arm(const char* text, long len, long signo_at, int code) {
  std::lock_guard<std::mutex> lock(g_mu);
  restore();  // never swap the buffer under an installed handler
  free(g_text);
  g_text = nullptr;
  g_len = 0;
  if (len > 0) {
    g_text = static_cast<char*>(malloc(static_cast<size_t>(len)));
    if (g_text == nullptr) return -1;
    memcpy(g_text, text, static_cast<size_t>(len));
    g_len = len;
  }
  g_signo_at = signo_at;
  g_code = code;
  g_fired.store(0);
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_handler = on_signal;
  sigfillset(&sa.sa_mask);  // no other handled signal interleaves with the write
  for (int i = 0; i < kNumSignals; ++i) {
    if (sigaction(kSignals[i], &sa, &g_prev[i]) != 0) {
      for (int j = 0; j < i; ++j) sigaction(kSignals[j], &g_prev[j], nullptr);
      return -1;
    }
  }
  g_armed = true;
  return 0;
}

// Put back the handlers that were installed before toa_lastline_arm.
int toa_lastline_disarm() {
  std::lock_guard<std::mutex> lock(g_mu);
  restore();
  return 0;
}

}  // extern "C"
