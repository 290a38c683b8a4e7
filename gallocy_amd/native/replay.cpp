// Config 5's round loop (BASELINE configs[4], the test_mmult trace) in C++ over the public C ABI
// (include/gdsm.h): the host side a C++ DSM runtime would run, as the reference's own runtime is
// C++ (gallocy/ heap + DSM layers). gallocy_amd/replay.py builds the plan on the device (events
// per round, page lists, row-copy descriptors) and calls this once for every round, so what is
// timed is the library's calls, not Python's per-call overhead. Per round, exactly the calls the
// Python round issues (replay.MmultReplay.round): the coherence batch on the page-table context,
// the round's row writes as one batched copy, and the release (or, retwin = 0, round 4's twin +
// gdsm_diff_apply_ids). Bench driver, not part of libgdsm.
#include <stdint.h>

#include <thread>

#include "gdsm.h"

extern "C" int gdsm_replay_mmult(gdsm_ctx* data, gdsm_ctx* pt, uint32_t r0, uint32_t r1,
                                 const uint64_t* events, const int64_t* ev_off, uint64_t* totals,
                                 const uint32_t* ids, const uint32_t* home, const int64_t* id_off,
                                 const uint64_t* desc, const int64_t* desc_off, gdsm_runs* runs,
                                 int retwin) {
  if (!data || !pt || !ev_off || !id_off || !desc_off || !runs) return -22;
  for (uint32_t r = r0; r < r1; ++r) {
    int rc = gdsm_coherence_batch_async(pt, events + ev_off[r], (uint64_t)(ev_off[r + 1] - ev_off[r]),
                                        totals + 10ull * r);
    if (rc) return rc;
    const uint64_t a = (uint64_t)id_off[r], n = (uint64_t)(id_off[r + 1] - id_off[r]);
    if (!retwin && (rc = gdsm_twin(data, ids + a, n))) return rc;
    rc = gdsm_memcpy_batch(data, desc + 3ull * (uint64_t)desc_off[r],
                           (uint64_t)(desc_off[r + 1] - desc_off[r]));
    if (rc) return rc;
    rc = retwin ? gdsm_release(data, ids + a, n, runs, GDSM_REPLICA, home + a, GDSM_RELEASE_RETWIN)
                : gdsm_diff_apply_ids(data, ids + a, n, runs, GDSM_REPLICA, home + a);
    if (rc) return rc;
  }
  return 0;
}

// The same rounds issued by two host threads, one per context (a context is driven by one thread
// at a time; the two streams never wait for each other within a round): the page-table thread
// issues every round's coherence batch, the page-data thread every round's row writes and release.
extern "C" int gdsm_replay_mmult_threads(gdsm_ctx* data, gdsm_ctx* pt, uint32_t r0, uint32_t r1,
                                         const uint64_t* events, const int64_t* ev_off,
                                         uint64_t* totals, const uint32_t* ids,
                                         const uint32_t* home, const int64_t* id_off,
                                         const uint64_t* desc, const int64_t* desc_off,
                                         gdsm_runs* runs, int retwin) {
  if (!data || !pt || !ev_off || !id_off || !desc_off || !runs) return -22;
  int rc_pt = 0;
  std::thread table([&] {
    for (uint32_t r = r0; r < r1 && !rc_pt; ++r)
      rc_pt = gdsm_coherence_batch_async(pt, events + ev_off[r],
                                         (uint64_t)(ev_off[r + 1] - ev_off[r]), totals + 10ull * r);
  });
  int rc = 0;
  for (uint32_t r = r0; r < r1 && !rc; ++r) {
    const uint64_t a = (uint64_t)id_off[r], n = (uint64_t)(id_off[r + 1] - id_off[r]);
    if (!retwin && (rc = gdsm_twin(data, ids + a, n))) break;
    rc = gdsm_memcpy_batch(data, desc + 3ull * (uint64_t)desc_off[r],
                           (uint64_t)(desc_off[r + 1] - desc_off[r]));
    if (rc) break;
    rc = retwin ? gdsm_release(data, ids + a, n, runs, GDSM_REPLICA, home + a, GDSM_RELEASE_RETWIN)
                : gdsm_diff_apply_ids(data, ids + a, n, runs, GDSM_REPLICA, home + a);
  }
  table.join();
  return rc ? rc : rc_pt;
}
