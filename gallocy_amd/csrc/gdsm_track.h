// Internal: the write-fault tracker's packing step used by gdsm_track_diff (gdsm_capi.cpp).
#pragma once
#include <stdint.h>

#include "gdsm.h"

namespace gdsm {

// Sorted dirty ids into ids_dst (cap entries), and the twin / current contents of those pages
// packed in id order into twin_dst / cur_dst (n x 4 KiB each).
int track_pack(gdsm_tracker* t, uint8_t* twin_dst, uint8_t* cur_dst, uint32_t* ids_dst,
               uint64_t cap, uint64_t* n_out);

}  // namespace gdsm
