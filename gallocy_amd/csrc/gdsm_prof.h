// Optional per-kernel HIP-event timing for the launchers (internal).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <vector>

#include "gdsm.h"

namespace gdsm {

struct Prof {
  static constexpr int kStages = GDSM_PROF_STAGES;
  bool on = false;
  hipStream_t stream = nullptr;
  struct Mark { int stage; hipEvent_t a, b; };
  std::vector<Mark> pending;
  std::vector<hipEvent_t> pool;
  double ms[kStages] = {};
  uint64_t launches[kStages] = {};
  int open_stage = -1;
  hipEvent_t open_ev = nullptr;

  hipEvent_t take() {
    if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
  }
  void begin(int stage, hipStream_t s) {
    if (!on) return;
    open_stage = stage;
    open_ev = take();
    if (open_ev) (void)hipEventRecord(open_ev, s);
  }
  void end(hipStream_t s) {
    if (!on || open_stage < 0) return;
    hipEvent_t e = take();
    if (e && open_ev) {
      (void)hipEventRecord(e, s);
      pending.push_back({open_stage, open_ev, e});
    }
    open_stage = -1;
  }
  // An event recorded on s now (nullptr when off); span() pairs two of them into a stage.
  hipEvent_t mark(hipStream_t s) {
    if (!on) return nullptr;
    hipEvent_t e = take();
    if (e) (void)hipEventRecord(e, s);
    return e;
  }
  void span(int stage, hipEvent_t a, hipEvent_t b) {
    if (a && b) pending.push_back({stage, a, b});
    else {
      if (a) pool.push_back(a);
      if (b) pool.push_back(b);
    }
  }
  // Caller synchronised the stream.
  void resolve() {
    for (auto& m : pending) {
      float t = 0.f;
      if (hipEventElapsedTime(&t, m.a, m.b) == hipSuccess) {
        ms[m.stage] += t;
        launches[m.stage] += 1;
      }
      pool.push_back(m.a);
      pool.push_back(m.b);
    }
    pending.clear();
  }
  void clear() {
    for (int i = 0; i < kStages; ++i) { ms[i] = 0; launches[i] = 0; }
  }
  ~Prof() {
    for (auto& m : pending) { (void)hipEventDestroy(m.a); (void)hipEventDestroy(m.b); }
    for (auto e : pool) (void)hipEventDestroy(e);
  }
};

// RAII bracket around one kernel launch.
struct ProfScope {
  Prof* p;
  hipStream_t s;
  ProfScope(Prof* p_, int stage, hipStream_t s_) : p(p_), s(s_) { if (p) p->begin(stage, s); }
  ~ProfScope() { if (p) p->end(s); }
};

}  // namespace gdsm
