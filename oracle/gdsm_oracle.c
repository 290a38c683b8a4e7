/*
 * gdsm oracle — TEST INFRASTRUCTURE ONLY (see gdsm_oracle.h for the pinning statement).
 * Plain C99, single thread. Built by oracle/Makefile into oracle/liboracle.so.
 */
#include "gdsm_oracle.h"

#include <stdlib.h>
#include <string.h>

uint64_t or_mix64(uint64_t z) {
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBull;
  z ^= z >> 31;
  return z;
}

uint64_t or_hash3(uint64_t s, uint64_t a, uint64_t b) {
  return or_mix64(or_mix64(s ^ (a * 0x9E3779B97F4A7C15ull)) + b * 0xC2B2AE3D27D4EB4Full +
                  0x165667B19E3779F9ull);
}

/* ---------------------------------------------------------------- synthetic pages (SPEC §6) */
void or_gen_pages(uint8_t* twin, uint8_t* cur, uint8_t* replica, uint64_t first_page,
                  uint64_t stride, uint64_t n, uint64_t seed, int mode, uint32_t ppm) {
  uint64_t tw[512], cw[512];
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t p = first_page + i * stride;
    for (uint64_t w = 0; w < 512; ++w) {
      const uint64_t v = or_hash3(seed ^ 0xDA7Aull, p, w);
      int changed;
      if (mode == 0)
        changed = (or_hash3(seed ^ 0x5E1EC7EDull, p, w) % 1000000ull) < ppm;
      else
        changed = (or_hash3(seed ^ 0xC1057E12ull, p, w >> 3) % 1000000ull) < ppm;
      uint64_t x = 0;
      if (changed) {
        x = or_hash3(seed ^ 0x0F11E5ull, p, w);
        if (x == 0) x = 1;
      }
      tw[w] = v;
      cw[w] = v ^ x;
    }
    if (twin) memcpy(twin + i * OR_PAGE_SZ, tw, OR_PAGE_SZ);
    if (cur) memcpy(cur + i * OR_PAGE_SZ, cw, OR_PAGE_SZ);
    if (replica) memcpy(replica + i * OR_PAGE_SZ, tw, OR_PAGE_SZ);
  }
}

/* ---------------------------------------------------------------- run diff (SPEC §3) */
typedef struct { uint16_t off, len; } or_run;

static uint32_t page_runs(const uint8_t* t, const uint8_t* c, or_run* runs, uint32_t* payload) {
  const uint64_t* tw = (const uint64_t*)t;
  const uint64_t* cw = (const uint64_t*)c;
  uint32_t nr = 0, pay = 0, start = 0;
  int in_run = 0;
  for (uint32_t w = 0; w < 512; ++w) {
    const uint64_t x = tw[w] ^ cw[w];
    if (x == 0) {
      if (in_run) {
        runs[nr].off = (uint16_t)start;
        runs[nr].len = (uint16_t)(w * 8 - start);
        pay += runs[nr].len;
        ++nr;
        in_run = 0;
      }
      continue;
    }
    for (uint32_t b = 0; b < 8; ++b) {
      const int d = ((x >> (8 * b)) & 0xff) != 0;
      const uint32_t pos = w * 8 + b;
      if (d && !in_run) {
        start = pos;
        in_run = 1;
      } else if (!d && in_run) {
        runs[nr].off = (uint16_t)start;
        runs[nr].len = (uint16_t)(pos - start);
        pay += runs[nr].len;
        ++nr;
        in_run = 0;
      }
    }
  }
  if (in_run) {
    runs[nr].off = (uint16_t)start;
    runs[nr].len = (uint16_t)(OR_PAGE_SZ - start);
    pay += runs[nr].len;
    ++nr;
  }
  *payload = pay;
  return nr;
}

uint64_t or_diff_pages(const uint8_t* twin, const uint8_t* cur, const uint32_t* ids,
                       uint64_t n, uint64_t* rec_off, uint8_t* data, uint64_t cap) {
  or_run runs[2048];
  uint64_t off = 0;
  rec_off[0] = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t p = ids ? ids[i] : i;
    const uint8_t* t = twin + p * OR_PAGE_SZ;
    const uint8_t* c = cur + p * OR_PAGE_SZ;
    uint32_t pay = 0;
    const uint32_t nr = page_runs(t, c, runs, &pay);
    uint64_t sz = 0;
    if (nr) {
      sz = 4 + 4ull * nr + ((pay + 3u) & ~3u);
      if (off + sz <= cap) {
        uint8_t* r = data + off;
        memcpy(r, &nr, 4);
        uint8_t* pl = r + 4 + 4ull * nr;
        for (uint32_t k = 0; k < nr; ++k) {
          const uint32_t h = (uint32_t)runs[k].off | ((uint32_t)runs[k].len << 16);
          memcpy(r + 4 + 4ull * k, &h, 4);
          memcpy(pl, c + runs[k].off, runs[k].len);
          pl += runs[k].len;
        }
        while ((uint64_t)(pl - r) < sz) *pl++ = 0;
      }
    }
    off += sz;
    rec_off[i + 1] = off;
  }
  return off;
}

/* ---------------------------------------------------------------- apply (SPEC §4) */
int or_apply(uint8_t* target, const uint32_t* ids, uint64_t n, const uint64_t* rec_off,
             const uint8_t* data) {
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t sz = rec_off[i + 1] - rec_off[i];
    if (sz == 0) continue;
    const uint8_t* r = data + rec_off[i];
    uint32_t nr;
    memcpy(&nr, r, 4);
    if (nr == 0 || nr > 2048 || sz < 4 + 4ull * nr) return -22;
    const uint64_t p = ids ? ids[i] : i;
    uint8_t* dst = target + p * OR_PAGE_SZ;
    const uint8_t* pl = r + 4 + 4ull * nr;
    uint32_t end = 0, pay = 0;
    for (uint32_t k = 0; k < nr; ++k) {
      uint32_t h;
      memcpy(&h, r + 4 + 4ull * k, 4);
      const uint32_t o = h & 0xffffu, l = h >> 16;
      if (l == 0 || o + l > OR_PAGE_SZ || (k && o < end)) return -22;
      end = o + l;
      pay += l;
    }
    if (sz != 4 + 4ull * nr + ((pay + 3u) & ~3u)) return -22;
    for (uint32_t k = 0; k < nr; ++k) {
      uint32_t h;
      memcpy(&h, r + 4 + 4ull * k, 4);
      const uint32_t o = h & 0xffffu, l = h >> 16;
      memcpy(dst + o, pl, l);
      pl += l;
    }
  }
  return 0;
}

void or_twin(uint8_t* twin, const uint8_t* cur, const uint32_t* ids, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t p = ids ? ids[i] : i;
    memcpy(twin + p * OR_PAGE_SZ, cur + p * OR_PAGE_SZ, OR_PAGE_SZ);
  }
}

/* ---------------------------------------------------------------- NW (reference diff()) */
/* Restates gallocy/utils/diff.cpp:73-167:
 *  - rows y over mem1 (n1+1), columns x over mem2 (n2+1)              diff.cpp:77-78
 *  - borders: M[0][x] = -x (traceback left), M[y][0] = -y (up)         diff.cpp:91-102
 *  - diag = M[y-1][x-1] + (mem1[y-1] == mem2[x-1]); the ternary
 *    `Cost::MATCH ? a == b : Cost::MISMATCH` always takes the (a==b)
 *    arm, so a mismatch scores 0, never -2                             diff.cpp:107-108
 *  - left/up = neighbour - 1; tie-break diag > left > up               diff.cpp:109-121
 *  - traceback from (n1,n2) to (0,0), gaps written as '-'              diff.cpp:125-158  */
int or_nw_diff(const char* m1, size_t n1, const char* m2, size_t n2, char* out1, char* out2,
               size_t* out_len) {
  const size_t R = n1 + 1, C = n2 + 1;
  int32_t* prev = (int32_t*)malloc(C * sizeof(int32_t));
  int32_t* row = (int32_t*)malloc(C * sizeof(int32_t));
  uint8_t* dir = (uint8_t*)malloc(R * C); /* 0 none, 1 diag, 2 left, 3 up */
  if (!prev || !row || !dir) {
    free(prev); free(row); free(dir);
    return -12;
  }
  for (size_t x = 0; x < C; ++x) {
    prev[x] = -(int32_t)x;
    dir[x] = x ? 2 : 0;
  }
  for (size_t y = 1; y < R; ++y) {
    row[0] = -(int32_t)y;
    dir[y * C] = 3;
    for (size_t x = 1; x < C; ++x) {
      const int32_t dg = prev[x - 1] + (m1[y - 1] == m2[x - 1] ? 1 : 0);
      const int32_t lf = row[x - 1] - 1;
      const int32_t up = prev[x] - 1;
      int32_t mx = dg;
      if (lf > mx) mx = lf;
      if (up > mx) mx = up;
      dir[y * C + x] = (dg == mx) ? 1 : (lf == mx) ? 2 : 3;
      row[x] = mx;
    }
    int32_t* t = prev; prev = row; row = t;
  }
  size_t L = 0;
  for (size_t y = n1, x = n2; y || x; ++L) {
    const uint8_t d = dir[y * C + x];
    if (d == 1) { --y; --x; } else if (d == 2) { --x; } else { --y; }
  }
  size_t k = L;
  out1[L] = 0;
  out2[L] = 0;
  for (size_t y = n1, x = n2; y || x;) {
    const uint8_t d = dir[y * C + x];
    --k;
    if (d == 1) { out1[k] = m1[y - 1]; out2[k] = m2[x - 1]; --y; --x; }
    else if (d == 2) { out1[k] = '-'; out2[k] = m2[x - 1]; --x; }
    else { out1[k] = m1[y - 1]; out2[k] = '-'; --y; }
  }
  *out_len = L;
  free(prev); free(row); free(dir);
  return 0;
}

/* ---------------------------------------------------------------- coherence (SPEC §5) */
void or_coh_init(uint32_t* state, uint32_t* faults, uint64_t n_pages, uint32_t n_nodes) {
  const uint64_t per = (n_pages + n_nodes - 1) / n_nodes;
  for (uint64_t p = 0; p < n_pages; ++p) {
    const uint32_t home = (uint32_t)(p / per);
    state[p] = (1u << home) | (home << 8) | (2u << 16);
    faults[p] = 0;
  }
}

int or_coherence(uint32_t* state, uint32_t* faults, uint64_t n_pages, uint32_t n_nodes,
                 const uint64_t* events, uint64_t n_events, uint64_t* totals) {
  for (int k = 0; k < 10; ++k) totals[k] = 0;
  uint64_t last_page = 0;
  for (uint64_t i = 0; i < n_events; ++i) {
    const uint64_t e = events[i];
    const uint64_t p = e >> 4;
    const uint32_t node = (uint32_t)((e >> 1) & 7u);
    const int wr = (int)(e & 1u);
    if (p >= n_pages || (i && p < last_page) || node >= n_nodes) return -22;
    last_page = p;
    uint32_t s = state[p];
    uint32_t cs = s & 0xffu, owner = (s >> 8) & 0xffu, st = (s >> 16) & 3u, dirty = (s >> 18) & 1u;
    const uint32_t bit = 1u << node;
    if (!wr) {
      if (!(cs & bit)) {
        faults[p]++;
        totals[2 + node]++;
        cs |= bit;
        if (st == 2) st = 1;
      }
    } else {
      dirty = 1;
      if (!(st == 2 && owner == node)) {
        faults[p]++;
        totals[2 + node]++;
        totals[0] += (uint64_t)__builtin_popcount(cs & ~bit);
        totals[1] += (owner != node);
      }
      owner = node;
      cs = bit;
      st = 2;
    }
    state[p] = cs | (owner << 8) | (st << 16) | (dirty << 18);
  }
  return 0;
}

void or_gen_events(uint64_t* events, const uint64_t* offsets, uint64_t first_page, uint64_t n,
                   uint64_t seed, uint32_t n_nodes, uint32_t write_pct) {
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t p = first_page + i;
    for (uint64_t j = 0, c = offsets[i + 1] - offsets[i]; j < c; ++j) {
      const uint64_t node = or_hash3(seed ^ 0x40DEull, p, j) % n_nodes;
      const uint64_t rw = (or_hash3(seed ^ 0x3217Eull, p, j) % 100u) < write_pct;
      events[offsets[i] + j] = (p << 4) | (node << 1) | rw;
    }
  }
}
