// nc_prof.cpp — opt-in per-kernel timers (nc_profile_enable / nc_profile_read /
// nc_profile_read_span).  bench.py uses them to time the step's kernels on the streams
// they run on, so its roofline numbers come from the same launches rocprofv3 sees.
//
// Two measurements per profiled launch:
//  * HIP events recorded around the launch on its stream (mode 1 only).  They include
//    any time the kernel waits behind other streams' work after the start event;
//  * the kernel's execution span, recorded by the kernel itself (nc_device.h
//    Span / span_record: min wave start .. max wave end on the 100 MHz wall clock) —
//    what rocprofv3 --kernel-trace reports as the kernel's duration.  No host work per
//    launch beyond handing the kernel its slot, so mode 2 (spans only) is cheap enough to
//    stay on during a timed region.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "nc_engine.h"
#include "nc_span.h"

namespace nc {

struct KernelTimers {
  struct Slot {
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
    size_t used = 0;
    std::vector<int> spans;     // span slots of this tag's launches since the last read
  };
  std::map<std::string, Slot> slots;
  // event pairs created when timing is enabled, handed to the first launches of each tag: a
  // timed region then records events without creating them (hipEventCreate is host work in
  // the region the events measure)
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pool;
  bool events = true;
  bool roof_only = false;   // mode 3: events only around the roofline kernels
  bool marks = false;       // mode 5: marker spans around the small entry points (MarkSpan)
  unsigned long long* span_buf = nullptr;   // [kSpanCap][kSpanLines][kSpanStride]: (start, end, pad)
  int span_used = 0;
  double clock_khz = 100000.0;
  ~KernelTimers() {
    for (auto& kv : slots)
      for (auto& p : kv.second.ev) {
        (void)hipEventDestroy(p.first);
        (void)hipEventDestroy(p.second);
      }
    for (auto& p : pool) {
      (void)hipEventDestroy(p.first);
      (void)hipEventDestroy(p.second);
    }
    if (span_buf) (void)hipFree(span_buf);
  }
};

constexpr size_t kSpanLaunchU64 = (size_t)kSpanLines * kSpanStride;

static void span_reset(KernelTimers& t) {
  std::vector<unsigned long long> h((size_t)kSpanCap * kSpanLaunchU64, 0ull);
  for (size_t i = 0; i < h.size(); i += kSpanStride) h[i] = ~0ull;
  (void)hipMemcpy(t.span_buf, h.data(), h.size() * sizeof(unsigned long long), hipMemcpyHostToDevice);
  t.span_used = 0;
}

KTimer::KTimer(Context& ctx, const char* tag, hipStream_t st) : ctx_(ctx), tag_(tag), st_(st) {
  if (!ctx_.timers) return;
  KernelTimers& t = *ctx_.timers;
  auto& slot = t.slots[tag_];
  if (t.span_buf && t.span_used < kSpanCap) {
    slot.spans.push_back(t.span_used);
    span_ = t.span_buf + (size_t)t.span_used++ * kSpanLaunchU64;
  }
  if (!t.events) return;
  if (t.roof_only && std::strcmp(tag_, "stft_mel") && std::strcmp(tag_, "cqt_low") && std::strcmp(tag_, "cqt_high") &&
      std::strcmp(tag_, "window_tg"))
    return;
  if (slot.used == slot.ev.size()) {
    if (!t.pool.empty()) {
      slot.ev.push_back(t.pool.back());
      t.pool.pop_back();
    } else {
      hipEvent_t a = nullptr, b = nullptr;
      if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return;
      slot.ev.emplace_back(a, b);
    }
  }
  auto& p = slot.ev[slot.used++];
  (void)hipEventRecord(p.first, st_);
  stop_ = p.second;
}

KTimer::~KTimer() {
  if (stop_) (void)hipEventRecord(static_cast<hipEvent_t>(stop_), st_);
}

MarkSpan::MarkSpan(Context& ctx, const char* tag, hipStream_t st) : st_(st) {
  KernelTimers* t = ctx.timers;
  if (!t || !t->marks || !t->span_buf || t->span_used >= kSpanCap) return;
  t->slots[tag].spans.push_back(t->span_used);
  span_ = t->span_buf + (size_t)t->span_used++ * kSpanLaunchU64;
  (void)launch_span_mark(span_, 0, st_);
}

MarkSpan::~MarkSpan() {
  if (span_) (void)launch_span_mark(span_, 1, st_);
}

void free_timers(Context& ctx) {
  delete ctx.timers;
  ctx.timers = nullptr;
}

}  // namespace nc

namespace nc {

// mode 0: off; 1: events + spans; 2: spans only; 3: events around the roofline kernels + spans;
// 4: events around the roofline kernels, no spans; 5: spans, plus marker spans around the small
// entry points (MarkSpan: timeline diagnosis only, the markers are launches of their own)
void profile_enable(Context& ctx, int mode) {
  free_timers(ctx);
  if (!mode) return;
  auto* t = new KernelTimers();
  t->events = mode == 1 || mode == 3 || mode == 4;
  t->roof_only = mode == 3 || mode == 4;
  t->marks = mode == 5;
  if (t->events) {
    constexpr int kPoolPairs = 1024;   // a 10-step bench region launches ~500 timed kernels
    t->pool.reserve(kPoolPairs);
    for (int i = 0; i < kPoolPairs; ++i) {
      hipEvent_t a = nullptr, b = nullptr;
      if (hipEventCreate(&a) != hipSuccess) break;
      if (hipEventCreate(&b) != hipSuccess) {
        (void)hipEventDestroy(a);
        break;
      }
      t->pool.emplace_back(a, b);
    }
  }
  // mode 4 records no spans: every workgroup's clock read and span atomics cost the step ~3 %
  if (mode != 4 && hipMalloc(&t->span_buf, sizeof(unsigned long long) * kSpanCap * kSpanLaunchU64) != hipSuccess)
    t->span_buf = nullptr;
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx.device) == hipSuccess && khz > 0)
    t->clock_khz = khz;
  if (t->span_buf) span_reset(*t);
  ctx.timers = t;
}

int profile_read(Context& ctx, const char* tag, double* total_ms, int* launches) {
  *total_ms = 0.0;
  *launches = 0;
  if (!ctx.timers) return 0;
  auto it = ctx.timers->slots.find(tag);
  if (it == ctx.timers->slots.end()) return 0;
  auto& slot = it->second;
  double tot = 0.0;
  for (size_t i = 0; i < slot.used; ++i) {
    if (hipEventSynchronize(slot.ev[i].second) != hipSuccess) {
      set_error("nc_profile_read: event synchronize failed");
      return -1;
    }
    float ms = 0.0f;
    if (hipEventElapsedTime(&ms, slot.ev[i].first, slot.ev[i].second) != hipSuccess) {
      set_error("nc_profile_read: elapsed time failed");
      return -1;
    }
    tot += ms;
  }
  *total_ms = tot;
  *launches = (int)slot.used;
  slot.used = 0;
  return 0;
}

// Summed execution spans of `tag`'s launches since the last span read.  Waits for the
// device; the span buffer is recycled once no tag has unread spans.
int profile_read_span(Context& ctx, const char* tag, double* total_ms, int* launches) {
  *total_ms = 0.0;
  *launches = 0;
  KernelTimers* t = ctx.timers;
  if (!t || !t->span_buf) return 0;
  auto it = t->slots.find(tag);
  if (it == t->slots.end() || it->second.spans.empty()) return 0;
  if (hipDeviceSynchronize() != hipSuccess) {
    set_error("nc_profile_read_span: device synchronize failed");
    return -1;
  }
  std::vector<unsigned long long> h((size_t)t->span_used * kSpanLaunchU64);
  if (t->span_used && hipMemcpy(h.data(), t->span_buf, h.size() * sizeof(unsigned long long),
                                hipMemcpyDeviceToHost) != hipSuccess) {
    set_error("nc_profile_read_span: copy failed");
    return -1;
  }
  double tot = 0.0;
  int n = 0;
  for (int s : it->second.spans) {
    unsigned long long a = ~0ull, b = 0ull;
    for (int l = 0; l < kSpanLines; ++l) {
      const unsigned long long* p = h.data() + (size_t)s * kSpanLaunchU64 + (size_t)l * kSpanStride;
      a = std::min(a, p[0]);
      b = std::max(b, p[1]);
    }
    if (b >= a && a != ~0ull) {          // launches with no work (empty grids) record nothing
      tot += (double)(b - a) / t->clock_khz;
      ++n;
    }
  }
  it->second.spans.clear();
  *total_ms = tot;
  *launches = n;
  bool any = false;
  for (auto& kv : t->slots) any |= !kv.second.spans.empty();
  if (!any) span_reset(*t);
  return 0;
}

// Device occupancy over every span recorded since the last reset, all tags together: the
// union of the launches' execution spans (busy) and first start .. last end (extent).  Only
// the timed (tagged) kernels record spans -- every large one; the small ones (bootstraps,
// plans, tails, gathers), torch's fills and the copies do not, so busy is a lower bound and
// 1 - busy / extent an upper bound of the idle fraction.  Clears every tag's spans.
int profile_read_busy(Context& ctx, double* busy_ms, double* extent_ms, int* launches) {
  *busy_ms = *extent_ms = 0.0;
  *launches = 0;
  KernelTimers* t = ctx.timers;
  if (!t || !t->span_buf) return 0;
  if (hipDeviceSynchronize() != hipSuccess) {
    set_error("nc_profile_read_busy: device synchronize failed");
    return -1;
  }
  std::vector<unsigned long long> h((size_t)t->span_used * kSpanLaunchU64);
  if (t->span_used && hipMemcpy(h.data(), t->span_buf, h.size() * sizeof(unsigned long long),
                                hipMemcpyDeviceToHost) != hipSuccess) {
    set_error("nc_profile_read_busy: copy failed");
    return -1;
  }
  std::vector<std::pair<unsigned long long, unsigned long long>> iv;
  for (int s = 0; s < t->span_used; ++s) {
    unsigned long long a = ~0ull, b = 0ull;
    for (int l = 0; l < kSpanLines; ++l) {
      const unsigned long long* p = h.data() + (size_t)s * kSpanLaunchU64 + (size_t)l * kSpanStride;
      a = std::min(a, p[0]);
      b = std::max(b, p[1]);
    }
    if (b >= a && a != ~0ull) iv.emplace_back(a, b);
  }
  std::sort(iv.begin(), iv.end());
  unsigned long long busy = 0, cur_a = 0, cur_b = 0;
  bool open = false;
  for (auto& p : iv) {
    if (!open || p.first > cur_b) {
      if (open) busy += cur_b - cur_a;
      cur_a = p.first;
      cur_b = p.second;
      open = true;
    } else {
      cur_b = std::max(cur_b, p.second);
    }
  }
  if (open) busy += cur_b - cur_a;
  if (!iv.empty()) {
    unsigned long long last = 0;
    for (auto& p : iv) last = std::max(last, p.second);
    *extent_ms = (double)(last - iv.front().first) / t->clock_khz;
  }
  *busy_ms = (double)busy / t->clock_khz;
  *launches = (int)iv.size();
  for (auto& kv : t->slots) kv.second.spans.clear();
  span_reset(*t);
  return 0;
}

// Every span since the last reset with its tag, in launch order (start, end relative to the
// earliest start).  Clears every tag's spans, as profile_read_busy.
int profile_dump_spans(Context& ctx, char* tags, int tags_cap, int* tag_index, double* start_ms, double* end_ms,
                       int cap, int* n) {
  *n = 0;
  tags[0] = '\0';
  KernelTimers* t = ctx.timers;
  if (!t || !t->span_buf) return 0;
  if (hipDeviceSynchronize() != hipSuccess) {
    set_error("nc_profile_dump_spans: device synchronize failed");
    return -1;
  }
  std::vector<unsigned long long> h((size_t)t->span_used * kSpanLaunchU64);
  if (t->span_used && hipMemcpy(h.data(), t->span_buf, h.size() * sizeof(unsigned long long),
                                hipMemcpyDeviceToHost) != hipSuccess) {
    set_error("nc_profile_dump_spans: copy failed");
    return -1;
  }
  std::vector<int> owner((size_t)t->span_used, -1);
  std::string names;
  int ti = 0;
  for (auto& kv : t->slots) {
    for (int sidx : kv.second.spans) owner[(size_t)sidx] = ti;
    names += kv.first;
    names += '\n';
    ++ti;
  }
  if ((int)names.size() + 1 > tags_cap) {
    set_error("nc_profile_dump_spans: tag buffer too small");
    return -1;
  }
  std::memcpy(tags, names.c_str(), names.size() + 1);
  unsigned long long t0 = ~0ull;
  std::vector<std::pair<unsigned long long, unsigned long long>> se((size_t)t->span_used, {0ull, 0ull});
  for (int sidx = 0; sidx < t->span_used; ++sidx) {
    unsigned long long a = ~0ull, b = 0ull;
    for (int l = 0; l < kSpanLines; ++l) {
      const unsigned long long* p = h.data() + (size_t)sidx * kSpanLaunchU64 + (size_t)l * kSpanStride;
      a = std::min(a, p[0]);
      b = std::max(b, p[1]);
    }
    se[(size_t)sidx] = {a, b};
    if (b >= a && a != ~0ull) t0 = std::min(t0, a);
  }
  int m = 0;
  for (int sidx = 0; sidx < t->span_used && m < cap; ++sidx) {
    const auto [a, b] = se[(size_t)sidx];
    if (!(b >= a && a != ~0ull) || owner[(size_t)sidx] < 0) continue;
    tag_index[m] = owner[(size_t)sidx];
    start_ms[m] = (double)(a - t0) / t->clock_khz;
    end_ms[m] = (double)(b - t0) / t->clock_khz;
    ++m;
  }
  *n = m;
  for (auto& kv : t->slots) kv.second.spans.clear();
  span_reset(*t);
  return 0;
}

}  // namespace nc
