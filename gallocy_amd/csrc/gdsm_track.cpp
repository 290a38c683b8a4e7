// Host write-fault capture: the step before the GPU diff.
//
// The reference describes, but never implements, protecting shared pages and taking a fault on
// access so that the page's contents can be negotiated and copied (resources/NUTSHELL.md:52-69,
// resources/IMPLEMENTATION.md:246-249: "a SIGSEGV signal is raised in the thread that caused
// the fault"); its only mprotect use is the thread-stack guard pages
// (gallocy/threads.cpp:53-58). This file is that missing piece for the twin/diff protocol:
//
//   gdsm_track_begin   protects a page-aligned host region PROT_READ and installs a SIGSEGV
//                      handler (SA_SIGINFO, chained to whatever handler was there before);
//   first write to a page (in any thread): the handler copies the page to the tracker's twin
//                      buffer, appends its id to the dirty list, makes it writable and
//                      returns, so the faulting store retries and succeeds; later writes to the
//                      page run at full speed until the next interval;
//   gdsm_track_dirty   the sorted ids of the pages written in this interval;
//   gdsm_track_diff    (gdsm_capi.cpp) packs those pages' twin and current contents, uploads
//                      them and runs the GPU run diff (SPEC §3) on them;
//   gdsm_track_rearm   re-protects the dirty pages and starts the next interval (a release
//                      point: no thread may write the region meanwhile).
//
// Per page state (atomic u8): 0 clean and protected, 1 being captured, 2 dirty and writable.
// Concurrent first writes to one page: one thread captures, the others wait for state 2.
// The handler only does memcpy, mprotect and atomics. Only write faults are claimed (x86-64:
// the page-fault error code's W bit); any other fault, e.g. an instruction fetch from a tracked
// PROT_READ page, goes to the previous handler. gdsm_track_end unpublishes the tracker and then
// waits until no handler is in flight (g_inflight) before freeing it, so a handler that loaded
// the tracker just before never touches freed memory.
#include <errno.h>
#include <signal.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sched.h>
#include <sys/mman.h>
#include <ucontext.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <new>

#include "gdsm.h"
#include "gdsm_track.h"

struct gdsm_tracker {
  uint8_t* base = nullptr;
  uint64_t n_pages = 0;
  uint8_t* twin = nullptr;              // n_pages x 4 KiB (mmap'd, only dirty pages written)
  std::atomic<uint8_t>* state = nullptr;
  uint32_t* dirty = nullptr;            // append-only list of the interval's dirty page ids
  std::atomic<uint64_t> n_dirty{0};
  std::atomic<uint64_t> faults{0};      // write faults taken (all intervals)
};

namespace {

constexpr int kMaxTrackers = 64;
std::atomic<gdsm_tracker*> g_trackers[kMaxTrackers];
std::atomic<int> g_inflight{0};  // SIGSEGV handlers currently inside the tracker scan
std::mutex g_install_mu;
struct sigaction g_prev;
bool g_installed = false;

bool capture(gdsm_tracker* t, uintptr_t addr) {
  const uintptr_t lo = reinterpret_cast<uintptr_t>(t->base);
  if (addr < lo || addr >= lo + t->n_pages * GDSM_PAGE_SZ) return false;
  const uint64_t p = (addr - lo) / GDSM_PAGE_SZ;
  uint8_t expect = 0;
  if (t->state[p].compare_exchange_strong(expect, 1, std::memory_order_acq_rel)) {
    uint8_t* page = t->base + p * GDSM_PAGE_SZ;
    memcpy(t->twin + p * GDSM_PAGE_SZ, page, GDSM_PAGE_SZ);  // readable: PROT_READ
    t->dirty[t->n_dirty.fetch_add(1, std::memory_order_relaxed)] = (uint32_t)p;
    t->faults.fetch_add(1, std::memory_order_relaxed);
    mprotect(page, GDSM_PAGE_SZ, PROT_READ | PROT_WRITE);
    t->state[p].store(2, std::memory_order_release);
  } else {
    while (t->state[p].load(std::memory_order_acquire) == 1) {
    }
  }
  return true;
}

// True when the fault was a data write (only those are the tracker's: tracked pages are
// always readable).
bool is_write_fault(void* uctx) {
#if defined(__x86_64__)
  const ucontext_t* uc = static_cast<const ucontext_t*>(uctx);
  return (uc->uc_mcontext.gregs[REG_ERR] & 0x2) != 0;
#else
  (void)uctx;
  return true;
#endif
}

void on_segv(int sig, siginfo_t* si, void* uctx) {
  const uintptr_t addr = reinterpret_cast<uintptr_t>(si->si_addr);
  if (is_write_fault(uctx)) {
    g_inflight.fetch_add(1, std::memory_order_seq_cst);
    bool mine = false;
    for (int i = 0; i < kMaxTrackers && !mine; ++i) {
      gdsm_tracker* t = g_trackers[i].load(std::memory_order_seq_cst);
      mine = t && capture(t, addr);
    }
    g_inflight.fetch_sub(1, std::memory_order_seq_cst);
    if (mine) return;
  }
  // Not ours: hand the fault to the handler that was installed before us.
  if (g_prev.sa_flags & SA_SIGINFO) {
    if (g_prev.sa_sigaction) {
      g_prev.sa_sigaction(sig, si, uctx);
      return;
    }
  } else if (g_prev.sa_handler != SIG_DFL && g_prev.sa_handler != SIG_IGN) {
    g_prev.sa_handler(sig);
    return;
  }
  // Default action: restore it and return; the faulting access repeats and terminates.
  struct sigaction dfl;
  memset(&dfl, 0, sizeof(dfl));
  dfl.sa_handler = SIG_DFL;
  sigemptyset(&dfl.sa_mask);
  sigaction(SIGSEGV, &dfl, nullptr);
}

int install() {
  std::lock_guard<std::mutex> lk(g_install_mu);
  if (g_installed) return 0;
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = on_segv;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  if (sigaction(SIGSEGV, &sa, &g_prev) != 0) return -errno;
  g_installed = true;
  return 0;
}

void* map_anon(uint64_t bytes) {
  void* p = mmap(nullptr, bytes ? bytes : GDSM_PAGE_SZ, PROT_READ | PROT_WRITE,
                 MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  return p == MAP_FAILED ? nullptr : p;
}

void destroy(gdsm_tracker* t) {
  if (!t) return;
  if (t->twin) munmap(t->twin, t->n_pages * GDSM_PAGE_SZ);
  if (t->dirty) munmap(t->dirty, t->n_pages * sizeof(uint32_t));
  if (t->state) munmap(static_cast<void*>(t->state), t->n_pages);
  delete t;
}

}  // namespace

extern "C" {

int gdsm_track_begin(gdsm_tracker** out, void* base, uint64_t n_pages) {
  if (!out || !base || n_pages == 0 || n_pages > 0xFFFFFFFFull) return -EINVAL;
  if (reinterpret_cast<uintptr_t>(base) % GDSM_PAGE_SZ) return -EINVAL;
  int rc = install();
  if (rc) return rc;
  gdsm_tracker* t = new (std::nothrow) gdsm_tracker;
  if (!t) return -ENOMEM;
  t->base = static_cast<uint8_t*>(base);
  t->n_pages = n_pages;
  t->twin = static_cast<uint8_t*>(map_anon(n_pages * GDSM_PAGE_SZ));
  t->dirty = static_cast<uint32_t*>(map_anon(n_pages * sizeof(uint32_t)));
  void* st = map_anon(n_pages);  // zero-filled: every page starts clean
  t->state = static_cast<std::atomic<uint8_t>*>(st);
  if (!t->twin || !t->dirty || !st) {
    destroy(t);
    return -ENOMEM;
  }
  int slot = -1;
  for (int i = 0; i < kMaxTrackers && slot < 0; ++i) {
    gdsm_tracker* none = nullptr;
    if (g_trackers[i].compare_exchange_strong(none, t)) slot = i;
  }
  if (slot < 0) {
    destroy(t);
    return -ENOMEM;
  }
  if (mprotect(base, n_pages * GDSM_PAGE_SZ, PROT_READ) != 0) {
    rc = -errno;
    g_trackers[slot].store(nullptr);
    destroy(t);
    return rc;
  }
  *out = t;
  return 0;
}

int gdsm_track_dirty(gdsm_tracker* t, uint32_t* ids, uint64_t cap, uint64_t* n_out) {
  if (!t || !n_out) return -EINVAL;
  const uint64_t n = t->n_dirty.load(std::memory_order_acquire);
  *n_out = n;
  if (!ids) return 0;
  if (cap < n) return -ENOSPC;
  memcpy(ids, t->dirty, n * sizeof(uint32_t));
  std::sort(ids, ids + n);
  return 0;
}

int gdsm_track_twin(gdsm_tracker* t, const void** twin) {
  if (!t || !twin) return -EINVAL;
  *twin = t->twin;
  return 0;
}

int gdsm_track_faults(gdsm_tracker* t, uint64_t* faults) {
  if (!t || !faults) return -EINVAL;
  *faults = t->faults.load(std::memory_order_relaxed);
  return 0;
}

int gdsm_track_rearm(gdsm_tracker* t) {
  if (!t) return -EINVAL;
  const uint64_t n = t->n_dirty.load(std::memory_order_acquire);
  std::sort(t->dirty, t->dirty + n);
  // re-protect maximal runs of consecutive dirty pages with one mprotect each
  for (uint64_t i = 0; i < n;) {
    uint64_t j = i + 1;
    while (j < n && t->dirty[j] == t->dirty[j - 1] + 1) ++j;
    if (mprotect(t->base + (uint64_t)t->dirty[i] * GDSM_PAGE_SZ, (j - i) * GDSM_PAGE_SZ,
                 PROT_READ) != 0)
      return -errno;
    for (uint64_t k = i; k < j; ++k) t->state[t->dirty[k]].store(0, std::memory_order_release);
    i = j;
  }
  t->n_dirty.store(0, std::memory_order_release);
  return 0;
}

int gdsm_track_end(gdsm_tracker* t) {
  if (!t) return -EINVAL;
  for (int i = 0; i < kMaxTrackers; ++i) {
    gdsm_tracker* self = t;
    g_trackers[i].compare_exchange_strong(self, nullptr, std::memory_order_seq_cst);
  }
  // Quiesce: a handler that loaded `t` before it was unpublished incremented g_inflight first
  // (both seq_cst), so it is seen here; wait for it to leave before freeing the tracker.
  while (g_inflight.load(std::memory_order_seq_cst) != 0) sched_yield();
  const int rc = mprotect(t->base, t->n_pages * GDSM_PAGE_SZ, PROT_READ | PROT_WRITE) ? -errno : 0;
  destroy(t);
  return rc;
}

}  // extern "C"

namespace gdsm {

int track_pack(gdsm_tracker* t, uint8_t* twin_dst, uint8_t* cur_dst, uint32_t* ids_dst,
               uint64_t cap, uint64_t* n_out) {
  if (!t || !n_out) return -EINVAL;
  uint64_t n = 0;
  int rc = gdsm_track_dirty(t, ids_dst, cap, &n);
  if (rc) return rc;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t p = ids_dst[i];
    memcpy(twin_dst + i * GDSM_PAGE_SZ, t->twin + p * GDSM_PAGE_SZ, GDSM_PAGE_SZ);
    memcpy(cur_dst + i * GDSM_PAGE_SZ, t->base + p * GDSM_PAGE_SZ, GDSM_PAGE_SZ);
  }
  *n_out = n;
  return 0;
}

}  // namespace gdsm
