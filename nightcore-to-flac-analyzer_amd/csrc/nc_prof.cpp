// nc_prof.cpp — opt-in per-kernel HIP-event timers (nc_profile_enable / nc_profile_read).
// bench.py uses them to time the dominant kernel of the step on the stream it runs on,
// so its roofline numbers come from the same launches rocprofv3 sees.
#include <hip/hip_runtime.h>

#include <map>
#include <string>
#include <utility>
#include <vector>

#include "nc_engine.h"

namespace nc {

struct KernelTimers {
  struct Slot {
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
    size_t used = 0;
  };
  std::map<std::string, Slot> slots;
  ~KernelTimers() {
    for (auto& kv : slots)
      for (auto& p : kv.second.ev) {
        (void)hipEventDestroy(p.first);
        (void)hipEventDestroy(p.second);
      }
  }
};

KTimer::KTimer(Context& ctx, const char* tag, hipStream_t st) : ctx_(ctx), tag_(tag), st_(st) {
  if (!ctx_.timers) return;
  auto& slot = ctx_.timers->slots[tag_];
  if (slot.used == slot.ev.size()) {
    hipEvent_t a = nullptr, b = nullptr;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return;
    slot.ev.emplace_back(a, b);
  }
  auto& p = slot.ev[slot.used++];
  (void)hipEventRecord(p.first, st_);
  stop_ = p.second;
}

KTimer::~KTimer() {
  if (stop_) (void)hipEventRecord(static_cast<hipEvent_t>(stop_), st_);
}

void free_timers(Context& ctx) {
  delete ctx.timers;
  ctx.timers = nullptr;
}

}  // namespace nc

namespace nc {

void profile_enable(Context& ctx, bool on) {
  free_timers(ctx);
  if (on) ctx.timers = new KernelTimers();
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

}  // namespace nc
