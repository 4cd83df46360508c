// pqg_fused.hip — K3 + K4 fused: the level decode and, for the small 4-byte
// dictionary pages (the C2 shape), the dictionary decode of the same page in
// the same wave.
//
// k_page_levels (pqg_levels.hip) decodes levels (VALU-bound: the speculative
// header parse and the run chain) and k_dict_walk / k_dict_walk_g decode the
// index streams (memory-bound: index bytes in, 4 bytes per value out).  As
// separate launches their times add.  Here one wave does both for a page, so
// on every CU some waves decode levels while others stream values, and the
// two overlap.
//
// The catch is the output position: a page's values go to value_offset =
// notNull of every earlier page of its chunk (readPageData appends,
// chunk_reader.go:380-402), which k_nn_scan computes only after every page's
// levels.  Here each page publishes its notNull as soon as its levels are
// decoded and finds its offset by a decoupled look-back over the chunk's
// earlier pages:
//   lb[p] = AGG | notNull          after p's levels,
//           INCL | offset+notNull   once p knows its own offset,
//           BLOCKED                 when p's notNull is not known here (a
//                                   level run handed to k_level_long).
// A page sums the AGG words of its predecessors, nearest first, until an
// INCL word (or the chunk's first page).  Pages are pulled from ONE queue
// head in list order, so every page a wave waits for was pulled earlier by a
// running wave, which publishes its AGG word without waiting for anything:
// the look-back always ends.  (The spin is bounded anyway: a page that gives
// up is left to k_dict_walk, which decodes it after k_nn_scan.)
//
// Pages this kernel decodes carry kPageFused: k_dict_plan gives them no work
// item.  Everything else (other pages' values, the notNull scan, capacity
// checks) is unchanged; k_nn_scan recomputes the same value offsets.
#include <hip/hip_runtime.h>

#include "pqg_common.h"
#include "pqg_device.h"
#include "pqg_hybrid.h"
#include "pqg_idxwalk.h"
#include "pqg_levdec.h"

namespace pqg {

constexpr uint64_t kLbAgg = 1ull << 62, kLbIncl = 2ull << 62, kLbBlocked = 3ull << 62;
constexpr uint64_t kLbValue = (1ull << 62) - 1;
constexpr int kLbSpins = 1 << 16;  // look-back polls before a page gives up (left to k_dict_walk)

__device__ __forceinline__ uint64_t lb_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A 4-byte dictionary page this kernel does not decode: the dictionary stage
// (k_dict_plan, k_dict4 / k_dict_walk) runs for it.
__device__ __forceinline__ void leave_to_dict_stage(const int* total) {
  int* present = const_cast<int*>(total) + kModePresentOff;
  if (present[1] == 0) present[1] = 1;
}

// The exclusive notNull prefix of page `pidx` over the chunk's pages
// [base, pidx): -1 when a predecessor is BLOCKED or the spin budget runs out.
// Wave-parallel: 64 predecessors per poll, nearest first.
__device__ __forceinline__ int64_t look_back(const uint64_t* lb, int64_t base, int64_t pidx) {
  const int lane = lane_id();
  int64_t acc = 0;
  int64_t k = pidx - 1;  // nearest predecessor not yet summed
  int spins = 0;
  while (k >= base) {
    const int64_t q = k - lane;
    const uint64_t v = q >= base ? lb_load(lb + q) : kLbIncl;  // before the chunk: an INCL of 0
    const uint64_t flag = v & ~kLbValue;
    const uint64_t done = __ballot(flag == kLbIncl || flag == kLbBlocked);
    const uint64_t notyet = __ballot(flag == 0);
    const int f = done ? __ffsll((long long)done) - 1 : 64;  // nearest INCL / BLOCKED (64: none in this poll)
    const uint64_t before = f >= 64 ? ~0ull : ((1ull << f) - 1);
    if (notyet & before) {  // a nearer page has not published yet: poll again
      if (++spins > kLbSpins) return -1;
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    // lanes < f hold AGG words; lane f the INCL (or BLOCKED) word
    const int64_t mine = (int64_t)(v & kLbValue);
    const int64_t part = wave_sum(lane < f ? mine : 0);
    acc += part;
    if (f < 64) {
      const uint64_t vf = (uint64_t)__builtin_amdgcn_readlane((int)(uint32_t)v, f) |
                          (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), f) << 32;
      if ((vf & ~kLbValue) == kLbBlocked) return -1;
      return acc + (int64_t)(vf & kLbValue);
    }
    k -= 64;
  }
  return acc;  // reached the chunk's first page
}

// One wave per page of the list, pulled in list order from ONE queue head
// (queue[0]).  Levels exactly as k_page_levels; then, for a small 4-byte
// dictionary page, the look-back and the index walk (IdxWalk, global
// dictionary gathers: the wave's LDS is the level window or the walk ring).
#ifndef PQG_FUSED_WPE
#define PQG_FUSED_WPE 3
#endif
__global__ void __launch_bounds__(64, PQG_FUSED_WPE) k_page_fused(JobDev* jobs, PageDev* pages, const int* list, const int* total,
                                                   int* queue, uint8_t* scratch, HStream* streams, uint8_t* def_arena,
                                                   uint8_t* rep_arena, LongLev* longs, int long_cap, LevPiece* pieces,
                                                   int piece_cap, uint8_t* value_arena, uint64_t* lb) {
  __shared__ __attribute__((aligned(16))) union {
    LevShared lev;
    WalkShared walk;
  } sh;
  const int lane = lane_id();
  const LongTables lt{longs, pieces, const_cast<int*>(total), long_cap, piece_cap};
  for (;;) {
    int t = 0;
    if (lane == 0) t = atomicAdd(queue, 1);  // one head: pages in list order (see the look-back)
    t = __builtin_amdgcn_readfirstlane(t);
    if (t >= *total) return;
    const int pidx = __builtin_amdgcn_readfirstlane(list[t]);
    const PageDev pg = pages[pidx];
    if (lane == 0) {
      pages[pidx].hs_rep = pages[pidx].hs_def = pages[pidx].hs_val = -1;
      pages[pidx].vmode = -1;
    }
    int64_t nn = 0;
    int de = kOK;
    bool deferred = false, fusable = false;
    int w = 0;                // index bit width
    gcu8 vals = nullptr;      // the index stream
    int64_t vals_n = 0;
    const bool is_data = pg.read_status == kOK && (pg.page_type == 0 || pg.page_type == 3);
    const JobDev& job = jobs[is_data ? pg.job : 0];  // wave-uniform: scalar loads
    const bool job_ok = is_data && job.status != kCAPACITY;
    if (job_ok) {
      const PageStreams ps = page_setup(job, pg, pidx, pages, streams, total, scratch, lane == 0, true);
      if (ps.e == kOK) {
        const int64_t n = pg.num_values;
        // ---- readValues (page_v1.go:27-55): rep levels, then def levels
        if (n > 0) {
          if (job.max_rep > 0) {
            if (ps.rep_n < 0) de = kLEVELS;
            else {
              uint32_t unused;
              bool dfr = false;
              de = level_stream(ps.rep, ps.rep_n, bits_len((uint32_t)job.max_rep), (uint32_t)n,
                                gmut(rep_arena) + job.slot_base + pg.slot_offset, 0x100u, sh.lev, &unused, lt, pidx, &dfr);
              deferred |= dfr;
            }
          }
          if (de == kOK) {
            if (job.max_def > 0) {
              if (ps.def_n < 0) de = kLEVELS;
              else {
                uint32_t c;
                bool dfr = false;
                de = level_stream(ps.def, ps.def_n, bits_len((uint32_t)job.max_def), (uint32_t)n,
                                  gmut(def_arena) + job.slot_base + pg.slot_offset, (uint32_t)job.max_def, sh.lev, &c,
                                  lt, pidx, &dfr);
                deferred |= dfr;
                nn = c;
              }
            } else {
              nn = n;
            }
          }
        }
        if (lane == 0) {
          pages[pidx].not_null = de == kOK ? (int32_t)nn : 0;
          if (de != kOK) pages[pidx].decode_status = de;
        }
        if (de != kOK) nn = 0;
        // a small 4-byte dictionary page with a valid bit width and keys to decode
        // (the page's fields from page_setup's registers: this wave's own stores
        // of the page record are not read back)
        if (de == kOK && !deferred && nn > 0 && ps.vmode == 1 && pg.num_values <= kSplitMin && ps.val_n >= 2) {
          w = (int)ps.val[0];
          fusable = w >= 1 && w <= 32;
          vals = ps.val + 1;
          vals_n = ps.val_n - 1;
        }
        if (ps.vmode == 1 && !fusable && lane == 0) leave_to_dict_stage(total);
      }
    }
    // ---- publish this page's notNull (every page of the list, data or not)
    const int64_t base = job_ok ? job.page_base : (int64_t)pidx;
    if (lane == 0) lb_store(lb + pidx, deferred ? kLbBlocked : (kLbAgg | (uint64_t)nn));
    if (!fusable) continue;
    // ---- the output position, then the keys
    const int64_t off = look_back(lb, base, pidx);
    if (off < 0) {  // left to k_dict_walk (after k_nn_scan)
      if (lane == 0) leave_to_dict_stage(total);
      continue;
    }
    if (lane == 0) lb_store(lb + pidx, kLbIncl | (uint64_t)(off + nn));
    if ((off + nn) * 4 > job.value_cap) {  // the arena is short: k_nn_scan reports it, the host grows it
      if (lane == 0) leave_to_dict_stage(total);
      continue;
    }
    const uint32_t dcount = job.dict_data ? (uint32_t)job.dict_count : 0u;
    PQG_G uint32_t* out = (PQG_G uint32_t*)(gmut(value_arena) + job.value_base) + off;
    const PQG_G uint32_t* dsafe = (const PQG_G uint32_t*)(job.dict_data ? gconst(job.dict_data) : (gcu8)out);
    IdxWalk<GlobalDict, false> iw{vals, (uint32_t)vals_n, w, (uint32_t)nn, out, dcount, GlobalDict{dsafe}, &sh.walk,
                           (uint32_t)((uintptr_t)vals & (kIWin - 1))};
    iw.run();
    const int64_t bad = wave_min((int64_t)iw.bad);
    const int vs = bad < nn ? kDICT_INDEX : (iw.produced < (uint32_t)nn ? iw.serr : kOK);
    if (lane == 0) {
      pages[pidx].flags = pg.flags | kPageFused;
      if (vs != kOK) pages[pidx].decode_status = vs;
    }
  }
}

}  // namespace pqg
