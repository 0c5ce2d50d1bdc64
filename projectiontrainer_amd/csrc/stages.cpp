// Per-stage device timers (SURVEY §5 tracing row: "per-stage HIP event timers behind an env flag"; the reference
// itself has none beyond tqdm).  Off by default; PTK_STAGE_TIMERS=1 or ptk_stage_timers_enable(1) turns them on.
//
// A stage is a [begin, end) span of one stream, bracketed by two HIP events: the model entry points mark their
// pieces (siglip.fwd, gemma.fwd.attn, gemma.lm_head_ce, gemma.bwd.mlp, ...) and the host code marks its own
// (ptk_stage_begin / ptk_stage_end: vision, projector, optimizer).  Spans nest per thread.  Nothing synchronises
// until ptk_stage_timers_read, which waits for the recorded spans, adds their times per name and hands the
// events back to a pool.  Spans begun while the stream is being captured into a HIP graph record nothing.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/ptk.h"
#include "ptk_internal.h"

namespace ptk {
namespace {

struct Span {
  std::string name;
  hipEvent_t e0 = nullptr, e1 = nullptr;
};
struct Total {
  std::string name;
  double ms = 0;
  long count = 0;
};

std::mutex g_mu;
std::atomic<bool> g_on{[] {
  const char* e = getenv("PTK_STAGE_TIMERS");
  return e && *e && strcmp(e, "0") != 0;
}()};   // read and written from any thread
std::vector<hipEvent_t> g_pool;   // events ready for reuse
std::vector<Span> g_closed;        // recorded, not yet read
std::vector<Total> g_totals;       // first-seen order
thread_local std::vector<Span> g_open;

hipEvent_t take_event() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  return hipEventCreate(&e) == hipSuccess ? e : nullptr;
}

bool capturing(hipStream_t st) {
  hipStreamCaptureStatus s = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(st, &s) == hipSuccess && s != hipStreamCaptureStatusNone;
}

}  // namespace

bool stage_timers_on() { return g_on.load(std::memory_order_relaxed); }

void stage_begin(const char* name, hipStream_t st) {
  Span s;
  s.name = name ? name : "?";
  if (!capturing(st)) {
    std::lock_guard<std::mutex> lk(g_mu);
    s.e0 = take_event();
    s.e1 = take_event();
  }
  if (s.e0) (void)hipEventRecord(s.e0, st);
  g_open.push_back(std::move(s));
}

int stage_end(hipStream_t st) {
  if (g_open.empty()) return set_error("stage_end: no open stage on this thread");
  Span s = std::move(g_open.back());
  g_open.pop_back();
  std::lock_guard<std::mutex> lk(g_mu);
  if (!s.e0 || !s.e1) {
    if (s.e0) g_pool.push_back(s.e0);
    if (s.e1) g_pool.push_back(s.e1);
    return 0;
  }
  (void)hipEventRecord(s.e1, st);
  g_closed.push_back(std::move(s));
  return 0;
}

}  // namespace ptk

using namespace ptk;

extern "C" {

int ptk_stage_timers_enable(int on) {
  g_on.store(on != 0, std::memory_order_relaxed);
  return 0;
}

int ptk_stage_begin(const char* name, void* stream) {
  if (stage_timers_on()) stage_begin(name, (hipStream_t)stream);
  else g_open.push_back(Span{});   // keeps begin / end paired across an enable in between
  return 0;
}

int ptk_stage_end(void* stream) {
  if (!g_open.empty() && !g_open.back().e0 && g_open.back().name.empty()) {
    g_open.pop_back();
    return 0;
  }
  return stage_end((hipStream_t)stream);
}

// "name\tms\tcount\n" per stage, in first-seen order.  Returns the length of the full report (which may exceed
// cap - 1: call again with a larger buffer), or -1 with ptk_last_error set.  reset != 0 clears the totals after
// the report is written.
int64_t ptk_stage_timers_read(char* buf, size_t cap, int reset) {
  std::lock_guard<std::mutex> lk(g_mu);
  for (size_t k = 0; k < g_closed.size(); ++k) {
    const Span& s = g_closed[k];
    float ms = 0;
    if (hipEventSynchronize(s.e1) != hipSuccess || hipEventElapsedTime(&ms, s.e0, s.e1) != hipSuccess) {
      // the spans already added and the failing one are dropped (its events destroyed, not pooled), so the next
      // read starts after it instead of failing on it again
      const std::string nm = s.name;
      (void)hipEventDestroy(s.e0);
      (void)hipEventDestroy(s.e1);
      g_closed.erase(g_closed.begin(), g_closed.begin() + k + 1);
      return set_error("stage timers: the events of %s failed", nm.c_str()), -1;
    }
    size_t i = 0;
    while (i < g_totals.size() && g_totals[i].name != s.name) ++i;
    if (i == g_totals.size()) g_totals.push_back(Total{s.name, 0, 0});
    g_totals[i].ms += ms;
    g_totals[i].count += 1;
    g_pool.push_back(s.e0);
    g_pool.push_back(s.e1);
  }
  g_closed.clear();
  std::string out;
  char line[256];
  for (const Total& t : g_totals) {
    snprintf(line, sizeof line, "%s\t%.6f\t%ld\n", t.name.c_str(), t.ms, t.count);
    out += line;
  }
  if (buf && cap) {
    const size_t n = out.size() < cap - 1 ? out.size() : cap - 1;
    memcpy(buf, out.data(), n);
    buf[n] = 0;
  }
  if (reset) g_totals.clear();
  return (int64_t)out.size();
}

}  // extern "C"
