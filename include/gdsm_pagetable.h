/*
 * gdsm_pagetable.h — the page-table heap layer gallocy reserved but never wrote, on libgdsm.
 *
 * gallocy composes its allocators from HL heap layers (gallocy/include/gallocy/heaplayers/;
 * the application stack is LockedHeap<StdlibHeap<FirstFitHeap<SizeHeap<ZoneHeap<
 * SourceMmapHeap<PURPOSE_APPLICATION_HEAP>>>>>>, heaplayers/application.h:20-29). Its
 * PageTableHeap<Super> (heaplayers/pagetableheap.h:12-29) is a stub that only logs, and it is
 * instantiated nowhere. This header is that layer with the DSM protocol behind it
 * (resources/NUTSHELL.md:52-69: protect, fault, copy the latest contents, update page tables):
 *
 *   - placed directly above the source heap, the first allocation puts the whole zone
 *     (kZoneBytes from the first address the source hands out) under write-fault tracking
 *     (gdsm_track_begin): every page the program, or the layers above, first writes in an
 *     interval is twinned by the SIGSEGV handler and listed as dirty;
 *   - release(): the interval's dirty pages are diffed on the GPU against their twins
 *     (gdsm_track_diff, SPEC §3 run records) and the zone is re-armed for the next interval;
 *   - apply_at_home(): the home side applies a release to its REPLICA arena (gdsm_apply);
 *   - malloc / free / getSize / __reset forward to Super exactly like the reference layer.
 *
 * Header-only C++14 over the C ABI of include/gdsm.h; nothing here is GPU code.
 */
#ifndef GDSM_PAGETABLE_H_
#define GDSM_PAGETABLE_H_

#include <errno.h>
#include <stddef.h>
#include <stdint.h>

#include "gdsm.h"

namespace gdsm_hl {

template <class Super, size_t kZoneBytes>
class PageTableHeap : public Super {
  static_assert(kZoneBytes % GDSM_PAGE_SZ == 0, "the zone is a whole number of pages");

 public:
  static constexpr uint64_t kZonePages = kZoneBytes / GDSM_PAGE_SZ;

  inline void* malloc(size_t sz) {
    void* ptr = Super::malloc(sz);
    if (ptr && !tracker_ && !error_) attach(ptr);
    return ptr;
  }
  inline void free(void* ptr) { Super::free(ptr); }
  inline size_t getSize(void* ptr) { return Super::getSize(ptr); }
  inline void __reset() {
    detach();
    Super::__reset();
  }
  ~PageTableHeap() { detach(); }

  // ---- the DSM side
  /* Zone base (page-aligned) once the first allocation attached it, else NULL. */
  void* zone() const { return base_; }
  /* 0, or the negative errno with which tracking the zone failed. */
  int error() const { return error_; }
  /* Pages written since the last release (count only). */
  int dirty_count(uint64_t* n) const {
    if (!tracker_) return -EINVAL;
    return gdsm_track_dirty(tracker_, nullptr, 0, n);
  }
  /* Release point: diffs this interval's dirty pages on ctx's GPU into `out` (one record per
   * dirty page, ascending page index; ids_dev receives the indices, >= dirty_count entries) and
   * starts the next interval. No thread may write the zone during the call. */
  int release(gdsm_ctx* ctx, gdsm_runs* out, uint32_t* ids_dev, uint64_t* n_out) {
    if (!tracker_) return -EINVAL;
    int rc = gdsm_track_diff(ctx, tracker_, out, ids_dev, n_out);
    if (rc) return rc;
    return gdsm_track_rearm(tracker_);
  }
  /* Home side: applies a release (pages `ids_dev`, n = in->n) to the REPLICA arena of ctx, whose
   * page i mirrors zone page i. Asynchronous; gdsm_sync reports a malformed stream. */
  static int apply_at_home(gdsm_ctx* ctx, const uint32_t* ids_dev, const gdsm_runs* in) {
    return gdsm_apply(ctx, GDSM_REPLICA, ids_dev, in);
  }
  /* The write-fault tracker of the zone (include/gdsm.h gdsm_track_*), NULL before attach. */
  gdsm_tracker* tracker() const { return tracker_; }

 private:
  void attach(void* first) {
    // SourceMmapHeap hands out its zone from the mmap base (heaplayers/source.h:18-38).
    const uintptr_t b = reinterpret_cast<uintptr_t>(first) & ~(uintptr_t)(GDSM_PAGE_SZ - 1);
    base_ = reinterpret_cast<void*>(b);
    error_ = gdsm_track_begin(&tracker_, base_, kZonePages);
    if (error_) tracker_ = nullptr;
  }
  void detach() {
    if (tracker_) (void)gdsm_track_end(tracker_);
    tracker_ = nullptr;
    base_ = nullptr;
    error_ = 0;
  }

  gdsm_tracker* tracker_ = nullptr;
  void* base_ = nullptr;
  int error_ = 0;
};

}  // namespace gdsm_hl

#endif /* GDSM_PAGETABLE_H_ */
