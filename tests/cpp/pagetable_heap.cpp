// TEST DRIVER (tests/test_pagetable_heap.py, tests/test_gpu_pagetable_heap.py): gdsm_hl::PageTableHeap
// (include/gdsm_pagetable.h) inside a gallocy-style heap-layer stack,
//   SizeHeap<PageTableHeap<BumpSource, 1 MiB>>
// shaped like gallocy's SizeHeap (16-B size header, heaplayers/sizeheap.h:26-47) over
// SourceMmapHeap (one mmap'd zone handed out by a bump pointer, heaplayers/source.h:15-66).
//   pagetable_heap cpu  -> the write-fault side only (no GPU): the pages the program and the
//                          SizeHeap headers write are exactly the dirty list, the twins hold the
//                          contents before the interval, release points re-arm the zone.
//   pagetable_heap gpu  -> two release intervals diffed on the GPU (gdsm_track_diff) and applied
//                          at a home REPLICA (gdsm_apply); the replica equals the zone each time.
// Prints "ok <checks>" and exits 0, or names the failed check and exits 1.
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#include <set>
#include <vector>

#include "gdsm.h"
#include "gdsm_pagetable.h"

static int g_checks = 0;
#define CHECK(c)                                                              \
  do {                                                                        \
    ++g_checks;                                                               \
    if (!(c)) {                                                               \
      fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c);          \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

constexpr size_t kZone = 1 << 20;  // 256 pages

struct BumpSource {  // SourceMmapHeap's shape: one zone, bump allocation, free is a no-op
  void* malloc(size_t sz) {
    if (!zone_) {
      void* z = mmap(nullptr, kZone, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
      if (z == MAP_FAILED) return nullptr;
      zone_ = static_cast<char*>(z);
      next_ = zone_;
    }
    sz = (sz + 15) & ~(size_t)15;
    if (next_ + sz > zone_ + kZone) return nullptr;
    void* p = next_;
    next_ += sz;
    return p;
  }
  void free(void*) {}
  size_t getSize(void*) { return 0; }
  void __reset() {
    if (zone_) munmap(zone_, kZone);
    zone_ = next_ = nullptr;
  }
  char* zone_ = nullptr;
  char* next_ = nullptr;
};

template <class Super>
struct SizeHeap : Super {  // 16-B header holding the size, like gallocy's SizeHeap
  void* malloc(size_t sz) {
    char* p = static_cast<char*>(Super::malloc(sz + 16));
    if (!p) return nullptr;
    *reinterpret_cast<size_t*>(p) = sz;
    return p + 16;
  }
  void free(void* p) { Super::free(static_cast<char*>(p) - 16); }
  size_t getSize(void* p) { return *reinterpret_cast<size_t*>(static_cast<char*>(p) - 16); }
};

typedef SizeHeap<gdsm_hl::PageTableHeap<BumpSource, kZone>> Heap;

static std::set<uint64_t> pages_of(const char* zone, const char* p, size_t n) {
  std::set<uint64_t> s;
  for (size_t i = 0; i < n; i += 1) s.insert((uint64_t)(p + i - zone) / GDSM_PAGE_SZ);
  return s;
}

static std::vector<uint32_t> dirty(Heap& h) {
  uint64_t n = 0;
  CHECK(gdsm_track_dirty(h.tracker(), nullptr, 0, &n) == 0);
  std::vector<uint32_t> ids(n ? n : 1);
  CHECK(gdsm_track_dirty(h.tracker(), ids.data(), ids.size(), &n) == 0);
  ids.resize(n);
  return ids;
}

int main(int argc, char** argv) {
  const bool gpu = argc > 1 && !strcmp(argv[1], "gpu");
  Heap heap;
  std::vector<char*> objs;
  std::set<uint64_t> want;
  // interval 1: allocations (headers) + writes spread over the zone
  char* z = nullptr;
  for (int i = 0; i < 40; ++i) {
    const size_t sz = 100 + 1000 * (i % 7);
    char* p = static_cast<char*>(heap.malloc(sz));
    CHECK(p != nullptr);
    if (!z) {
      z = static_cast<char*>(heap.zone());
      CHECK(z != nullptr && heap.error() == 0);
      CHECK(((uintptr_t)z & (GDSM_PAGE_SZ - 1)) == 0);
    }
    for (uint64_t pg : pages_of(z, p - 16, 16)) want.insert(pg);  // the SizeHeap header
    if (i % 3 == 0) {
      memset(p, 0x40 + i, sz);
      for (uint64_t pg : pages_of(z, p, sz)) want.insert(pg);
    }
    objs.push_back(p);
  }
  CHECK(heap.getSize(objs[5]) == 100 + 1000 * 5);
  std::vector<uint32_t> d = dirty(heap);
  CHECK(std::set<uint64_t>(d.begin(), d.end()) == want);
  const char* twin = nullptr;
  CHECK(gdsm_track_twin(heap.tracker(), reinterpret_cast<const void**>(&twin)) == 0);
  for (uint32_t pg : d)  // the zone was fresh (zero) before the interval
    for (size_t b = 0; b < GDSM_PAGE_SZ; ++b) CHECK(twin[pg * GDSM_PAGE_SZ + b] == 0);

  gdsm_ctx* ctx = nullptr;
  gdsm_runs runs;
  uint32_t* ids_dev = nullptr;
  std::vector<char> replica(kZone, 0);
  if (gpu) {
    CHECK(gdsm_init(&ctx, 0, heap.kZonePages, GDSM_WANT_REPLICA) == 0);
    CHECK(gdsm_upload(ctx, GDSM_REPLICA, 0, heap.kZonePages, replica.data()) == 0);
    CHECK(gdsm_runs_alloc(ctx, heap.kZonePages, 0, &runs) == 0);
    CHECK(gdsm_dev_alloc(ctx, 4 * heap.kZonePages, reinterpret_cast<void**>(&ids_dev)) == 0);
  }
  for (int interval = 0; interval < 2; ++interval) {
    if (gpu) {
      uint64_t n = 0;
      CHECK(heap.release(ctx, &runs, ids_dev, &n) == 0);
      CHECK(n == want.size());
      CHECK(Heap::apply_at_home(ctx, ids_dev, &runs) == 0);
      CHECK(gdsm_sync(ctx) == 0);
      CHECK(gdsm_download(ctx, GDSM_REPLICA, 0, heap.kZonePages, replica.data()) == 0);
      CHECK(memcmp(replica.data(), z, kZone) == 0);
    } else {
      CHECK(gdsm_track_rearm(heap.tracker()) == 0);
    }
    uint64_t n = 99;
    CHECK(heap.dirty_count(&n) == 0 && n == 0);  // a release point re-arms the zone
    if (interval == 0) {  // interval 2: rewrite a few objects, free one, allocate more
      want.clear();
      for (int i = 1; i < 40; i += 9) {
        char* p = objs[i];
        p[7] ^= 0x5A;
        for (uint64_t pg : pages_of(z, p + 7, 1)) want.insert(pg);
      }
      heap.free(objs[2]);
      char* q = static_cast<char*>(heap.malloc(5000));
      CHECK(q != nullptr);
      memset(q, 0x11, 5000);
      for (uint64_t pg : pages_of(z, q - 16, 5016)) want.insert(pg);
      d = dirty(heap);
      CHECK(std::set<uint64_t>(d.begin(), d.end()) == want);
    }
  }
  if (gpu) {
    CHECK(gdsm_runs_free(ctx, &runs) == 0);
    CHECK(gdsm_fini(ctx) == 0);
  }
  heap.__reset();
  printf("ok %d\n", g_checks);
  return 0;
}
