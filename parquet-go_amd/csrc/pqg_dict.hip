// pqg_dict.hip — K4 hot path: data pages of 4-byte dictionary columns
// (RLE_DICTIONARY indices → int32 / float values, the C2 shape).
//
// dictDecoder.decodeValues (type_dict.go:39-59): dst[i] = values[key] for the
// page's notNull keys, "dict: invalid index" at the first key >= len(values);
// keys come from the hybrid stream (hybridDecoder.next, hybrid_decoder.go:82-166)
// whose runs k_hybrid_walk has tabled (RunEnt / BlockDesc, pqg_hybrid.h).
//
// k_values<1> (pqg_values.hip) paid two memory round trips per 1024 values:
// the run/payload loads of the next block group, then the dictionary gathers,
// and the wait for the gathers also waited for the previous group's stores
// (vmcnt retires in issue order).  Here:
//   * a workgroup of kDWaves waves takes kDWaves consecutive pages of the page
//     list per queue item (one atomic per workgroup); the first page's
//     dictionary, if it has at most kDictLdsEntries entries, is copied into LDS
//     once and kept while later items belong to the same chunk, so those gathers
//     are ds_read_b32 (C2: b <= 12);
//   * each wave stages a *piece* of its page — up to kPBlocks blocks, kPRuns
//     runs and kPPay payload bytes — with one round of loads (descriptors are
//     read into lanes, then every run and payload granule of the piece is
//     loaded before the first LDS write), then decodes the piece's blocks
//     from LDS with no global load in between;
//   * larger dictionaries are gathered from global memory, software-pipelined
//     across block pairs: the gathers of pair k + 1 are issued before the
//     stores of pair k, so no wait for a gather includes stores issued after it.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "pqg_common.h"
#include "pqg_device.h"
#include "pqg_hybrid.h"

namespace pqg {

// inclusive prefix max over the wave (DPP row_shr 1/2/4/8, row_bcast 15/31)
__device__ __forceinline__ uint32_t ldpp_incl_max_u32(uint32_t x) {
  uint32_t t;
#define PQG_MAX_STEP(ctrl, rm, bc)                                         \
  t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, ctrl, rm, 0xf, bc); \
  x = t > x ? t : x;
  PQG_MAX_STEP(0x111, 0xf, true) PQG_MAX_STEP(0x112, 0xf, true) PQG_MAX_STEP(0x114, 0xf, true)
  PQG_MAX_STEP(0x118, 0xf, true) PQG_MAX_STEP(0x142, 0xa, false) PQG_MAX_STEP(0x143, 0xc, false)
#undef PQG_MAX_STEP
  return x;
}

// Output stores: non-temporal (streaming), so that the output stream does not
// evict the dictionary's L2 lines (b = 20: 4 MiB, the size of one XCD's L2).
#ifndef PQG_DICT_NT
#define PQG_DICT_NT PQG_NT_OUT
#endif
#ifndef PQG_DICT_NT_IN
#define PQG_DICT_NT_IN 1  // the index-stream stage loads non-temporal too (r04: C2 3.22 -> 3.14-3.18 ms; 0: temporal)
#endif
__device__ __forceinline__ void dict_store(PQG_G uint32_t* p, uint32_t v) {
#if PQG_DICT_NT
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}

// Dictionary entries in LDS or in global memory.  Keys >= count read entry 0;
// the caller records the first such index (the page then fails with "dict:
// invalid index", and its values are never used).
struct LdsDict {
  static constexpr bool kGlobal = false;
  const PQG_L uint32_t* d;
  __device__ __forceinline__ uint32_t operator()(uint32_t k) const { return d[k]; }
};
struct GlobalDict {
  static constexpr bool kGlobal = true;
  const PQG_G uint32_t* d;
  __device__ __forceinline__ uint32_t operator()(uint32_t k) const { return d[k]; }
};
// A dictionary whose first n entries are in LDS and the rest in global memory
// (k_dict4_big).  Both loads are issued for every lane (a load under a branch
// is waited for inside it); lanes served by LDS all read global entry 0, one
// request per wave, so only the keys past the prefix cost L2 requests.
struct PrefixDict {
  static constexpr bool kGlobal = true;
  const PQG_L uint32_t* l;
  const PQG_G uint32_t* g;
  uint32_t n;
  __device__ __forceinline__ uint32_t operator()(uint32_t k) const {
    const bool in = k < n;
    const uint32_t gv = g[in ? 0u : k];
    const uint32_t lv = l[in ? k : 0u];
    return in ? lv : gv;
  }
};

#ifndef PQG_DICT_PPAY
#define PQG_DICT_PPAY 4096
#endif
#ifndef PQG_DICT_WAVES
#define PQG_DICT_WAVES 4
#endif
#ifndef PQG_DICT_WPE
#define PQG_DICT_WPE 2
#endif
constexpr int kDWaves = PQG_DICT_WAVES; // waves per workgroup = pages per queue item
constexpr int kDictLdsEntries = 4096;   // dictionaries gathered from LDS (16 KiB)
constexpr int kPBlocks = 63;            // blocks per piece (lane 63's descriptor bounds the last one)
#ifndef PQG_DICT_PRUNS
#define PQG_DICT_PRUNS 128
#endif
constexpr int kPRuns = PQG_DICT_PRUNS;   // run entries per piece (a multiple of 128)
constexpr int kPPay = PQG_DICT_PPAY;    // payload bytes per piece
constexpr int kPG = kPPay / 1024;       // payload granules per lane
constexpr int kPRunGr = kPRuns / 128;   // run-table granules per lane

struct PieceShared {
  RunEnt runs[kPRunGr * 128];       // from the 16-byte granule holding the piece's first run
  uint32_t stage[kPG * 256 + 4];    // payload window from a 16-byte aligned address (+ a dword past it)
  uint8_t rmap[kHBlock];            // run starting at each value of a multi-run block
  uint8_t ridx[kHBlock];            // run of each value of a multi-run block
};
// LDS of a dictionary workgroup.  kMode 0: run-table pages with a dictionary
// of <= kDictLdsEntries entries, or none (k_dict4); 3: run-table pages with a
// larger dictionary, its first kBigLdsEntries entries in LDS (k_dict4_big, one
// 8-wave workgroup per CU).
constexpr int kBigWaves = 8;
constexpr int kBigLdsEntries = 26624;  // 104 KiB: with 8 waves' page stages, one workgroup per CU
template <int kMode>
constexpr int dict_waves() { return kMode == 3 ? kBigWaves : kDWaves; }
template <int kMode>
struct DictShared {
  uint32_t dict[kMode == 3 ? kBigLdsEntries : kDictLdsEntries];
  PieceShared w[dict_waves<kMode>()];
  const uint8_t* dict_ptr;          // the dictionary being staged (set by a wave that holds its VRec)
  int dict_cnt;
  int item;
  int wjob[dict_waves<kMode>()];    // job of each wave's page (-1: none, or done)
  int dict_job;                     // job whose dictionary `dict` holds (-1: none)
};

#ifdef PQG_PROFILE
int prof_read_dict(unsigned long long* out) {
  unsigned long long z[64] = {0};
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pqg_prof), sizeof(z)) != hipSuccess) return -1;
  hipMemcpyToSymbol(HIP_SYMBOL(pqg_prof), z, sizeof(z));
  return 0;
}
#endif

// Per-wave phase accumulators of diagnostic builds (-DPQG_PROFILE), flushed
// with one atomic per slot when the wave exits (per-event atomics on one word
// would serialise the waves and distort what they measure).
struct DProf {
#ifdef PQG_PROFILE
  uint64_t a[16] = {0};
  __device__ __forceinline__ void add(int k, uint64_t x) { a[k] += x; }
  __device__ __forceinline__ void flush() {
    if (lane_id() == 0)
      for (int k = 0; k < 16; k++)
        if (a[k]) atomicAdd(&pqg_prof[k], (unsigned long long)a[k]);
  }
#else
  __device__ __forceinline__ void add(int, uint64_t) {}
  __device__ __forceinline__ void flush() {}
#endif
};
#ifdef PQG_PROFILE
#define PQG_DT(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#else
#define PQG_DT(v) const uint64_t v = 0
#endif

// One block of a piece, wave-uniform fields (read from lanes of the descriptor registers).
struct PBlock {
  uint32_t v0, v1;   // values [v0, v1)
  uint32_t rl, nr;   // first run: piece-local run index; runs in the block
  bool on;
};

// Keys of block B (lane L: values L + 64 q, q < 8: the LDS reads of the run
// marks are conflict-free, and each store instruction writes 64 consecutive
// values, 256 contiguous bytes), looked up and stored to out[value - B.v0]
// (out: the block's first value).  `bad`: first value index with key >= dcount.
template <class Dict>
__device__ __forceinline__ void block_out(PieceShared& ps, const PBlock& B, uint32_t mask, int w, int64_t plo8,
                                          int lane, PQG_G uint32_t* out, uint32_t dcount, const Dict& dict,
                                          int64_t& bad) {
  const uint32_t nv = B.v1 - B.v0;  // <= kHBlock
  uint32_t key[8];
  if (B.nr == 1) {
    const RunEnt e = ps.runs[B.rl];
    const uint32_t st = (uint32_t)__builtin_amdgcn_readfirstlane(e.start), src = (uint32_t)__builtin_amdgcn_readfirstlane(e.src);
    if (!(st & kRunBP)) {
      // one RLE run: one lookup
      const uint32_t x = dict(src < dcount ? src : 0u);
      if (src >= dcount) bad = (int64_t)B.v0 < bad ? (int64_t)B.v0 : bad;
#pragma unroll
      for (int q = 0; q < 8; q++)
        if ((uint32_t)(lane + 64 * q) < nv) dict_store(out + lane + 64 * q, x);
      return;
    }
    const uint32_t rb0 = (uint32_t)((int64_t)src * 8 - plo8) + (B.v0 + (uint32_t)lane - (st & ~kRunBP)) * (uint32_t)w;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint32_t rb = rb0 + (uint32_t)(64 * q * w);
      const uint32_t d = rb >> 5;
      key[q] = __builtin_amdgcn_alignbit(ps.stage[d + 1], ps.stage[d], rb & 31) & mask;
    }
  } else {
    // run of each value: marks at run starts, a prefix max over lane's 8
    // consecutive values and across lanes, into ridx
    __builtin_amdgcn_wave_barrier();
    *(PQG_L u32x2_t*)(lds_ptr(ps.rmap) + 8 * lane) = u32x2_t{0u, 0u};
    __builtin_amdgcn_wave_barrier();
    if (lane > 0 && (uint32_t)lane < B.nr) ps.rmap[(ps.runs[B.rl + lane].start & ~kRunBP) - B.v0] = (uint8_t)lane;
    __builtin_amdgcn_wave_barrier();
    const u32x2_t mk = *(const PQG_L u32x2_t*)(lds_ptr(ps.rmap) + 8 * lane);
    uint32_t idx[8], run_max = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint32_t m = ((q < 4 ? mk.x : mk.y) >> (8 * (q & 3))) & 0xff;
      run_max = m > run_max ? m : run_max;
      idx[q] = run_max;
    }
    uint32_t before = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ldpp_incl_max_u32(run_max), 0x138, 0xf, 0xf, false);
    uint32_t r4[2] = {0u, 0u};
#pragma unroll
    for (int q = 0; q < 8; q++) r4[q >> 2] |= (idx[q] > before ? idx[q] : before) << (8 * (q & 3));
    *(PQG_L u32x2_t*)(lds_ptr(ps.ridx) + 8 * lane) = u32x2_t{r4[0], r4[1]};
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint32_t j = (uint32_t)(lane + 64 * q);
      const RunEnt e = ps.runs[B.rl + ps.ridx[j]];
      const uint32_t rb = (uint32_t)((int64_t)e.src * 8 - plo8) + (B.v0 + j - (e.start & ~kRunBP)) * (uint32_t)w;
      const uint32_t d = rb >> 5;
      const uint32_t bits = __builtin_amdgcn_alignbit(ps.stage[d + 1], ps.stage[d], rb & 31) & mask;
      key[q] = (e.start & kRunBP) ? bits : e.src;
    }
  }
  // every lookup of the block issued before the first store
  uint32_t mx = 0;
#pragma unroll
  for (int q = 0; q < 8; q++) mx = (uint32_t)(lane + 64 * q) < nv && key[q] > mx ? key[q] : mx;
  if (__ballot(mx >= dcount)) {
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint32_t j = (uint32_t)(lane + 64 * q);
      if (j < nv && key[q] >= dcount) bad = (int64_t)(B.v0 + j) < bad ? (int64_t)(B.v0 + j) : bad;
      key[q] = key[q] < dcount ? key[q] : 0u;
    }
  }
  uint32_t val[8];
#pragma unroll
  for (int q = 0; q < 8; q++) val[q] = dict((uint32_t)(lane + 64 * q) < nv ? key[q] : 0u);
#pragma unroll
  for (int q = 0; q < 8; q++)
    if ((uint32_t)(lane + 64 * q) < nv) dict_store(out + lane + 64 * q, val[q]);
}

// Decode one page (or a part of a big page): keys piece by piece, looked up
// in `dict`, stored straight to `out` (the first block's value 0).  A piece is one round of independent loads: the descriptors of blocks
// kb .. kb + 63, kPRuns run entries from the run of block kb, and a kPPay-byte
// payload window from `pos` (at or before the next payload byte the page
// needs: blocks consume the stream in order, and a block's payload starts at
// most one byte before the previous block's ends).  The piece is the leading
// blocks whose runs and payload lie inside what was staged.
template <class Dict>
__device__ __forceinline__ int64_t dict_page(PieceShared& ps, const gcu8 sp, const int64_t n, const int w,
                                             const PQG_G RunEnt* runs, const PQG_G BlockDesc* blks, const int nb_all,
                                             const uint32_t end_all, gu8 out, uint32_t dcount, const Dict& dict,
                                             DProf& pf) {
  const int lane = lane_id();
  const uint32_t mask = w == 32 ? 0xffffffffu : ((1u << w) - 1);
  int64_t bad = INT64_MAX;
  if (end_all == 0) return bad;
  const uintptr_t pa = (uintptr_t)sp;
  if (nb_all <= 0) return bad;
  int kb = 0;
  // a part of a big page starts at any block: its first run and payload byte
  const uint4 d0 = ldg16((uintptr_t)blks);
  uint32_t rcur = d0.y;                 // first run of block kb
  int64_t pos = (d0.w & 0xffffu) ? (int64_t)d0.z : 0;  // stream offset of the payload window (before alignment)
  const uint32_t vfirst = d0.x;         // the first block's value 0: out[0]
  PQG_G uint32_t* const out32 = (PQG_G uint32_t*)out;
  while (kb < nb_all) {
    PQG_DT(ta);
    // ---- one round of loads: descriptors, run entries, payload window
    // (unconditional: a lane past the last block reads the last one, then
    // takes the empty descriptor; a load under a branch is waited for inside it)
    uint4 q = ldg16((uintptr_t)(blks + (kb + lane < nb_all ? kb + lane : nb_all - 1)));
    const uintptr_t ra = (uintptr_t)(runs + rcur);
    const uintptr_t ra_al = ra & ~(uintptr_t)15;
    const int rskew = (int)((ra - ra_al) >> 3);  // 0 or 1 entry before rcur
    uint4 rg[kPRunGr];
#pragma unroll
    for (int k = 0; k < kPRunGr; k++) rg[k] = ldg16(ra_al + 16 * (uintptr_t)(lane + 64 * k));
    const int64_t plo = pos - (int64_t)((pa + (uintptr_t)pos) & 15);  // 16-byte aligned address
    uint4 pg[kPG];
#pragma unroll
    for (int k = 0; k < kPG; k++) {  // unconditional loads (see dbp_restage): zeroed when stored
      const int64_t at = plo + 16 * (int64_t)(lane + 64 * k);
#if PQG_DICT_NT_IN
      pg[k] = ldg16_nt(at < n ? (uintptr_t)(sp + at) : (pa & ~(uintptr_t)15));  // index bytes: read once
#else
      pg[k] = ldg16(at < n ? (uintptr_t)(sp + at) : (pa & ~(uintptr_t)15));
#endif
    }
#pragma unroll
    for (int k = 0; k < kPRunGr; k++) sts16(lds_ptr(ps.runs) + 2 * (lane + 64 * k), rg[k]);
#pragma unroll
    for (int k = 0; k < kPG; k++) {
      const int64_t at = plo + 16 * (int64_t)(lane + 64 * k);
      sts16(lds_ptr(ps.stage) + 4 * (lane + 64 * k), mask_tail(pg[k], at, n));
    }
    if (kb + lane >= nb_all) q = make_uint4(0xffffffffu, 0u, 0u, 0u);
    const uint32_t v0 = q.x, r0 = q.y, lo = q.z, nbytes = q.w & 0xffffu, nr = q.w >> 16;
    __builtin_amdgcn_wave_barrier();
    PQG_DT(tb);
    pf.add(0, tb - ta);
    pf.add(4, 1);
    // ---- the piece: leading blocks whose runs and payload were staged
    const bool need = v0 < end_all;
    const bool hasp = need && nbytes > 0;
    const int64_t stage_end = plo + 16 * (int64_t)(64 * kPG);
    const uint32_t run_room = (uint32_t)(kPRunGr * 128 - rskew);
    const bool fits = lane < kPBlocks && need && r0 >= rcur && (r0 + nr - rcur) <= run_room &&
                      (!hasp || ((int64_t)lo >= plo && (int64_t)lo + nbytes <= stage_end));
    const uint64_t fm = __ballot(fits);
    const int m = (int)__builtin_ctzll(~fm);  // fm bit 63 is never set
    if (m == 0) {
      if (!__builtin_amdgcn_readfirstlane((int)need)) break;  // block kb starts at or past count
      // the window missed block kb's payload: restage at it (never twice in a row)
      pos = (int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)lo);
      continue;
    }
    const int64_t plo8 = plo * 8;
    // ---- blocks of the piece
    for (int k = 0; k < m; k++) {
      PQG_DT(tp0);
      PBlock B;
      B.on = true;
      B.v0 = (uint32_t)__builtin_amdgcn_readlane((int)v0, k);
      const uint32_t nx = (uint32_t)__builtin_amdgcn_readlane((int)v0, k + 1);
      B.v1 = nx < end_all ? nx : end_all;
      B.rl = (uint32_t)__builtin_amdgcn_readlane((int)r0, k) - rcur + (uint32_t)rskew;
      B.nr = (uint32_t)__builtin_amdgcn_readlane((int)nr, k);
      block_out(ps, B, mask, w, plo8, lane, out32 + (B.v0 - vfirst), dcount, dict, bad);
      PQG_DT(tp2);
      pf.add(11, tp2 - tp0);
    }
    __builtin_amdgcn_wave_barrier();
    PQG_DT(tc);
    pf.add(1, tc - tb);
    pf.add(5, (uint64_t)m);
    // ---- the next piece: block kb + m (lane m's descriptor)
    const uint32_t hi = hasp ? lo + nbytes : 0u;
    const uint32_t phi = (uint32_t)__builtin_amdgcn_readlane((int)ldpp_incl_max_u32(hi), m - 1);
    kb += m;
    rcur = (uint32_t)__builtin_amdgcn_readlane((int)r0, m);
    const uint64_t nxp = __ballot(lane >= m && hasp);
    if (nxp) pos = (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)lo, __builtin_ctzll(nxp));
    else if (phi > 0) pos = (int64_t)phi - 1;
  }
  return bad;
}

// a run-table page for k_dict4_big: a dictionary past the small LDS size of
// which the LDS prefix holds at least a third (C2 b = 16: 0.39 -> 0.31 ms;
// b = 20's 1 M entries gain nothing from 2.5 % and lose the occupancy, 0.55 ->
// 0.65 ms, so they stay with k_dict4's global gathers)
__device__ __forceinline__ bool big_dict(const VRec& r) {
  return r.dict && r.dcount > kDictLdsEntries && r.dcount <= 3 * kBigLdsEntries;
}

// Read phase of every 4-byte dictionary page in the list, and its VRec at the
// page's list position (valuesDecoder.init type_dict.go:22-37: the bit-width
// byte, > 32 is an error).
// One VRec per work item (a page's part, k_part_plan): a part of a big page is
// its blocks [b0, next part's b0) and values [v0, next part's v0).
__global__ void __launch_bounds__(256) k_dict_plan(JobDev* jobs, PageDev* pages, const PartRec* parts, const int* total,
                                                   uint8_t* value_arena, const HStream* streams, const RunEnt* runs,
                                                   const BlockDesc* blks, VRec* recs) {
  if (total[kModePresentOff + 1] == 0) return;
  const int nt = min(total[kCtrItems], total[kCtrPartsCap]);
  for (int t = blockIdx.x * 256 + threadIdx.x; t < nt; t += gridDim.x * 256) {
    VRec r;
    memset(&r, 0, sizeof(r));
    r.job = -1;
    const PartRec pr = parts[t];
    const int pidx = pr.pidx;
    r.pidx = pidx;
    PageDev& P = pages[pidx];
    if (pr.vmode == 1 && P.read_status == kOK && (P.page_type == 0 || P.page_type == 3) && P.vmode == 1) {
      const JobDev& J = jobs[P.job];
      if (J.status != kCAPACITY) {
        int re = kOK, dw = 0;
        if (P.val_n < 1) re = kEOF;
        else {
          dw = P.val[0];
          if (dw > 32) re = kBIT_WIDTH;
        }
        if (re != kOK) P.read_status = re;
        else if (P.decode_status == kOK && P.not_null > 0) {
          r.job = P.job;
          r.out = value_arena + J.value_base + P.value_offset * 4;
          r.dict = J.dict_data;
          r.dcount = J.dict_data ? (int32_t)J.dict_count : 0;
          r.nn = P.not_null;
          r.w = dw;
          if (dw > 0) {
            const HStream& S = streams[P.hs_val];
            const bool last = pr.p + 1 >= pr.np;
            const int b1 = last ? S.n_blocks : parts[t + 1].b0;
            r.p = S.p;
            r.n = (int32_t)S.n;
            r.runs = runs + S.run_base;
            r.blks = blks + S.blk_base + pr.b0;
            r.n_blocks = b1 - pr.b0;
            r.count = S.produced < r.nn ? S.produced : r.nn;
            if (!last && (int32_t)parts[t + 1].v0 < r.count) r.count = (int32_t)parts[t + 1].v0;
            r.out = value_arena + J.value_base + (P.value_offset + pr.v0) * 4;
            r.produced = S.produced;
            r.serr = (S.status != kOK && S.produced < r.nn) ? S.status : kOK;
            if (big_dict(r)) const_cast<int*>(total)[kModePresentOff + kPresentBigDict] = 1;
          }
        }
      }
    }
    recs[t] = r;
  }
}

// Mode 1 pages (4-byte dictionary columns): the C2 path, kDWaves * 64 threads
// per workgroup taking kDWaves consecutive work items.  kMode (DictShared):
// 0 = k_dict4, 3 = k_dict4_big.  Separate kernels, so each is compiled for
// its own register and LDS budget.
__device__ __forceinline__ void dict_fill0(const VRec& r, int lane, int& de) {
  // a zero-width decoder yields key 0 forever, reading nothing (hybrid_decoder.go:84-86)
  if (r.dcount < 1) de = kDICT_INDEX;
  else {
    const uint32_t d0 = *(const PQG_G uint32_t*)gconst(r.dict);
    for (int64_t i = lane; i < r.nn; i += 64) ((PQG_G uint32_t*)gmut(r.out))[i] = d0;
  }
}

template <int kMode>
__device__ __forceinline__ void dict_items(PageDev* pages, const int* total, int* queue, const VRec* recs,
                                           int big = 0) {
  __shared__ __attribute__((aligned(16))) DictShared<kMode> sh;
  constexpr int kDWaves = dict_waves<kMode>();  // this kernel's waves per workgroup (= pages per item)
  const int lane = lane_id(), wid = (int)(threadIdx.x >> 6);
  if (total[kModePresentOff + 1] == 0) return;  // no page of this stage
  if (kMode == 3 && total[kModePresentOff + kPresentBigDict] == 0) return;
  if (threadIdx.x == 0) sh.dict_job = -1;
  const int nt = min(total[kCtrItems], total[kCtrPartsCap]);  // work items: pages' parts (k_part_plan)
  DProf pf;
  for (;;) {
    PQG_DT(t0);
    if (threadIdx.x == 0) sh.item = queue_pull(queue);
    __syncthreads();
    const int t = __builtin_amdgcn_readfirstlane(sh.item) * kDWaves + wid;
    const int t_first = t - wid;
    if (t_first >= nt) break;  // workgroup-uniform
    // ---- this wave's page (wave-uniform: scalar loads)
    VRec r;
    r.job = -1;
    if (t < nt) r = recs[t];
    // a zero-width page (key 0 for every value, no run table) stays with
    // k_dict4 whatever its dictionary's size: k_dict_plan raises the big-dict
    // stage flag only for pages with index streams
    const int own = kMode == 0 ? (r.n_blocks >= 0 && !(big && r.w > 0 && big_dict(r)))
                               : (r.n_blocks >= 0 && r.w > 0 && big_dict(r));
    if (!own) r.job = -1;  // another kernel's page
    PQG_DT(t1);
    pf.add(2, t1 - t0);
    {
    // ---- the dictionaries of the item's pages into LDS, one job
    // at a time (an item holds pages of at most kDWaves jobs); the pages of
    // the job in LDS decode, then the next job's
    if (lane == 0) sh.wjob[wid] = r.job;
    __syncthreads();
    for (;;) {
      int want = -1;
#pragma unroll
      for (int k = 0; k < kDWaves; k++)
        if (want < 0) want = sh.wjob[k];
      want = __builtin_amdgcn_readfirstlane(want);
      if (want < 0) break;  // workgroup-uniform
      if (want != sh.dict_job) {
        // every wave of the item with this job holds its dictionary pointer; take the first's
        int src_w = 0;
#pragma unroll
        for (int k = kDWaves - 1; k >= 0; k--)
          if (sh.wjob[k] == want) src_w = k;
        if (wid == src_w && lane == 0) {
          sh.dict_ptr = r.dict;
          sh.dict_cnt = r.dcount;
        }
        __syncthreads();
        const int64_t dc = sh.dict_ptr ? sh.dict_cnt : 0;
        if constexpr (kMode == 3) {
          // the dictionary's first kBigLdsEntries entries, in rounds of 8 loads per thread
          const PQG_G uint32_t* src = (const PQG_G uint32_t*)gconst(sh.dict_ptr);
          const int m = (int)(dc < kBigLdsEntries ? dc : kBigLdsEntries);
          for (int b0 = 0; b0 < m; b0 += 8 * kDWaves * 64) {
            uint32_t rr[8];
#pragma unroll
            for (int k = 0; k < 8; k++) {
              const int i = b0 + (int)threadIdx.x + k * kDWaves * 64;
              rr[k] = src[i < m ? i : 0];
            }
#pragma unroll
            for (int k = 0; k < 8; k++) {
              const int i = b0 + (int)threadIdx.x + k * kDWaves * 64;
              if (i < m) sh.dict[i] = rr[k];
            }
          }
          __syncthreads();
          if (threadIdx.x == 0) sh.dict_job = want;
        } else if (dc > 0 && dc <= kDictLdsEntries) {
          const PQG_G uint32_t* src = (const PQG_G uint32_t*)gconst(sh.dict_ptr);
          uint32_t rr[kDictLdsEntries / (kDWaves * 64)];
#pragma unroll
          for (int k = 0; k < kDictLdsEntries / (kDWaves * 64); k++) {
            const int i = (int)threadIdx.x + k * kDWaves * 64;
            rr[k] = src[i < dc ? i : 0];  // unconditional (a load under a branch is waited for inside it)
          }
#pragma unroll
          for (int k = 0; k < kDictLdsEntries / (kDWaves * 64); k++) {
            const int i = (int)threadIdx.x + k * kDWaves * 64;
            if (i < dc) sh.dict[i] = rr[k];
          }
          __syncthreads();
          if (threadIdx.x == 0) sh.dict_job = want;
        } else if (threadIdx.x == 0) {
          sh.dict_job = -1;
        }
        pf.add(8, 1);
        __syncthreads();
      }
      const bool lds = sh.dict_job == want;
      PQG_DT(t2);
      pf.add(3, t2 - t1);
      if (r.job == want) {
        int de = kOK;
        if (r.w == 0) {
          dict_fill0(r, lane, de);
        } else if constexpr (kMode == 3) {
          PieceShared& ps = sh.w[wid];
          const PQG_G uint32_t* dg = (const PQG_G uint32_t*)gconst(r.dict);
          const uint32_t nl = (uint32_t)(r.dcount < kBigLdsEntries ? r.dcount : kBigLdsEntries);
          int64_t bad = dict_page(ps, gconst(r.p), r.n, r.w, gconst(r.runs), gconst(r.blks), r.n_blocks,
                                  (uint32_t)r.count, gmut(r.out), (uint32_t)r.dcount,
                                  PrefixDict{lds_ptr(sh.dict), dg, lds ? nl : 0u}, pf);
          bad = wave_min(bad);
          if (bad < r.nn && (r.serr == kOK || bad < r.produced)) de = kDICT_INDEX;
          else de = r.serr;
        } else if constexpr (kMode == 0) {
          const gcu8 sp = gconst(r.p);
          const PQG_G RunEnt* rt = gconst(r.runs);
          const PQG_G BlockDesc* bt = gconst(r.blks);
          PieceShared& ps = sh.w[wid];
          int64_t bad;
          if (lds) {
            bad = dict_page(ps, sp, r.n, r.w, rt, bt, r.n_blocks, (uint32_t)r.count, gmut(r.out), (uint32_t)r.dcount,
                            LdsDict{lds_ptr(sh.dict)}, pf);
            pf.add(7, 1);
          } else {
            const PQG_G uint32_t* dsafe = (const PQG_G uint32_t*)(r.dict ? gconst(r.dict) : gconst(r.out));
            bad = dict_page(ps, sp, r.n, r.w, rt, bt, r.n_blocks, (uint32_t)r.count, gmut(r.out), (uint32_t)r.dcount,
                            GlobalDict{dsafe}, pf);
          }
          bad = wave_min(bad);
          if (bad < r.nn && (r.serr == kOK || bad < r.produced)) de = kDICT_INDEX;
          else de = r.serr;
        }
        // parts of a page: kDICT_INDEX wins
        if (lane == 0 && de != kOK) atomicMin(&pages[r.pidx].decode_status, de);
        if (lane == 0) sh.wjob[wid] = -1;
        r.job = -2;  // done
      }
      __syncthreads();
      PQG_DT(t3);
      pf.add(6, 1);
      pf.add(9, t3 - t2);
    }
    }
  }
  pf.add(10, 1);
  pf.flush();
}

// big: k_dict4_big runs too and takes the pages with larger dictionaries
__global__ void __attribute__((amdgpu_flat_work_group_size(1, kDWaves * 64), amdgpu_waves_per_eu(PQG_DICT_WPE)))
k_dict4(PageDev* pages, const int* total, int* queue, const VRec* recs, int big) {
  dict_items<0>(pages, total, queue, recs, big);
}
__global__ void __attribute__((amdgpu_flat_work_group_size(1, kBigWaves * 64), amdgpu_waves_per_eu(2)))
k_dict4_big(PageDev* pages, const int* total, int* queue, const VRec* recs) {
  dict_items<3>(pages, total, queue, recs, 1);
}

}  // namespace pqg
