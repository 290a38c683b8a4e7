// Host-side launchers for the gdsm kernels (internal; the public ABI is include/gdsm.h).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include "gdsm_prof.h"

namespace gdsm {

// Workspace of one diff of n list entries (ticket counter + one look-back granule per unit).
uint64_t diff_workspace_bytes(uint64_t n);
// Kernel variant knobs (see gdsm_tune); returns -1 for an unknown key.
int tune(const char* key, int64_t value);
int coh_tune(const char* key, int64_t value);

hipError_t launch_gen_pages(uint8_t* twin, uint8_t* cur, uint8_t* replica, uint64_t n,
                            uint64_t first_global, uint64_t stride, uint64_t seed, int mode,
                            uint32_t ppm, hipStream_t s);
hipError_t launch_twin(uint8_t* twin, const uint8_t* cur, const uint32_t* ids, uint64_t n,
                       hipStream_t s, Prof* prof = nullptr);
// Full diff of n pages in one pass: rec_off[n+1], data[cap]. With `target`, the runs are also
// applied to target (same page ids) by the same kernel.
hipError_t launch_diff(const uint8_t* twin, const uint8_t* cur, const uint32_t* ids, uint64_t n,
                       uint64_t* rec_off, uint8_t* data, uint64_t cap, uint8_t* ws,
                       uint64_t ws_bytes, hipStream_t s, Prof* prof = nullptr,
                       uint8_t* target = nullptr);
hipError_t launch_apply(uint8_t* target, const uint32_t* ids, uint64_t n,
                        const uint64_t* rec_off, const uint8_t* data, uint32_t* err,
                        hipStream_t s, Prof* prof = nullptr);
// A received fixed-budget stream: zeroes rec_off (nothing applied) and err |= 4 unless
// rec_off[0] == 0 and rec_off[n] <= cap.
hipError_t launch_guard_stream(uint64_t* rec_off, uint64_t n, uint64_t cap, uint32_t* err,
                               hipStream_t s);
// Caller page-id lists at the context level: safe[i] = ids[i] if < n_pages, else n_pages (the
// arenas' guard page), and err |= 8 when any id was out of range.
hipError_t launch_check_ids(const uint32_t* ids, uint64_t n, uint64_t n_pages, uint32_t* safe,
                            uint32_t* err, hipStream_t s);

// Coherence (SPEC §5).
uint64_t coh_workspace_bytes(uint64_t n_events);
// Page table: one u64 per page, state | faults << 32.
hipError_t launch_coh_init(uint64_t* pt, uint64_t n_pages, uint32_t n_nodes, hipStream_t s);
// Events naming a page >= n_pages or a node >= n_nodes reject the batch (err |= 2).
hipError_t launch_coherence(uint64_t* pt, uint64_t n_pages, uint32_t n_nodes,
                            const uint64_t* events, uint64_t n_events, uint64_t* totals,
                            uint8_t* ws, uint64_t ws_bytes, uint32_t* err, hipStream_t s,
                            Prof* prof = nullptr);
hipError_t launch_gen_events(uint64_t* events, const uint64_t* offsets, uint64_t first_page,
                             uint64_t n, uint64_t seed, uint32_t n_nodes, uint32_t write_pct,
                             hipStream_t s);

// GPU NW alignment (legacy diff()): workspace per pair and the fill + trace launches.
uint64_t nw_pair_ws_bytes(uint32_t max_len);
hipError_t launch_nw(const uint8_t* a, const uint64_t* a_off, const uint8_t* b,
                     const uint64_t* b_off, uint64_t n, uint32_t max_len, uint8_t* out1,
                     uint8_t* out2, uint64_t* out_len, uint8_t* ws, uint64_t ws_bytes,
                     uint32_t* err, hipStream_t s, Prof* prof = nullptr);

// Diff wire format (SPEC §7).
uint64_t wire_frame_bytes(uint64_t n, uint64_t data_bytes);
hipError_t launch_wire_sum(const uint8_t* frame, uint64_t F, uint64_t* sum, hipStream_t s);
// dst[i] = i for i < n (identity page-id lists on the device).
hipError_t launch_iota(uint32_t* dst, uint64_t n, hipStream_t s);
hipError_t launch_b64_encode(const uint8_t* frame, uint64_t F, uint8_t* text, hipStream_t s);
hipError_t launch_b64_decode(const uint8_t* text, uint64_t T, uint32_t pad, uint8_t* frame,
                             uint64_t F, uint32_t* err, hipStream_t s);
hipError_t launch_wire_check(const uint32_t* ids, const uint64_t* rec_off, uint64_t n,
                             uint64_t D, uint64_t n_pages, uint32_t* err, hipStream_t s);

}  // namespace gdsm
