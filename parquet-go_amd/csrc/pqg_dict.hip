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
// In-kernel walk of a small page's index stream (no run tables, see
// IdxWalk below): a ring window over the stream, the run marks / run index
// of a batch's values, the batch's run entries and the chain flags.
constexpr int kIWin = 4096;   // ring bytes; stream byte at absolute address a sits at (a & (kIWin - 1))
constexpr int kINeed = 3072;  // window bytes a step wants at and after its first header (the ring streams
                              // in 1 KiB quarters: a quarter is replaced once the step has left it)
constexpr int kIPos = 64;     // header positions parsed per step (one per lane)
constexpr int kISpan = 512;   // values per batch (8 per lane)
struct WalkShared {
  uint32_t win[kIWin / 4];
  uint8_t tm[kISpan];   // 1 + run position at each run's first value; then the run of every value
  u32x2_t te[kIPos];    // per run position: {first value | bit 31 bit-packed, BP: payload bit in the ring; RLE: value}
  uint8_t cflag[kIPos];
};
// LDS of a dictionary workgroup.  kMode 0: run-table pages (k_dict4); 1:
// walked pages with a dictionary of <= kDictLdsEntries entries (k_dict_walk);
// 2: walked pages gathering from global memory (k_dict_walk_g: no LDS
// dictionary, so more workgroups fit a CU).
template <int kMode>
struct DictShared {
  uint32_t dict[kMode == 2 ? 1 : kDictLdsEntries];
  typename std::conditional<kMode == 0, PieceShared, WalkShared>::type w[kDWaves];
  const uint8_t* dict_ptr;          // the dictionary being staged (set by a wave that holds its VRec)
  int dict_cnt;
  int item;
  int wjob[kDWaves];                // job of each wave's page (-1: none, or done)
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

// One block of a piece, wave-uniform fields (read from lanes of the descriptor registers).
struct PBlock {
  uint32_t v0, v1;   // values [v0, v1)
  uint32_t rl, nr;   // first run: piece-local run index; runs in the block
  bool on;
};

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

// ---- Small pages: the index stream walked here, wave-parallel ----------------
// hybridDecoder.next (hybrid_decoder.go:82-166) over a page's keys without the
// run tables of k_hybrid_walk (which skips these streams), the way the level
// decoder of pqg_levels.hip walks level streams, for widths 1..32 and with the
// dictionary lookups as its sink.  Per step:
//   1. every lane parses a run header speculatively at pos + lane (uvarint
//      header, RLE value or bit-packed extent, its errors);
//   2. unless run 0's successor lies beyond the step's positions, the chain
//      from run 0 by pointer doubling (chain_marks64);
//   3. a saturating DPP prefix sum of the chain runs' counts gives each run its
//      first value; the runs the page's keys need, up to kISpan values and
//      with their payload inside the window, form the batch; errors are
//      checked lane-parallel, in stream order;
//   4. keys: a one-run batch directly (RLE: one lookup; bit-packed: w-bit
//      fields of the ring), several runs through run marks at their first
//      values and a prefix max; the keys of values lane + 64 q are looked up
//      and stored (each store instruction writes 256 contiguous bytes).
// A run longer than a batch goes in pieces.  Errors as k_hybrid_walk: header
// EOF / > MaxInt32 / uint64 overflow, empty runs, RLE values wider than w,
// short bit-packed reads (the last needed group must start inside the
// stream; bytes past it read as zero, Q5); then dictDecoder.decodeValues
// (type_dict.go:39-59): a key >= the dictionary size fails the page unless
// a stream error comes before it.
struct IRun {
  uint32_t cnt;   // values the header declares (saturated)
  uint32_t next;  // stream offset of the next header (saturated)
  uint32_t pay;   // BP: stream offset of the payload; RLE: the value
  int err;        // header / RLE value error (kOK: none)
  bool bp;
  bool cplx;      // header longer than 4 bytes: parsed serially
};

__device__ __forceinline__ uint32_t dpp_incl_add_sat(uint32_t x) {
  // saturating 64-lane inclusive sum (row_shr 1/2/4/8, row_bcast 15/31)
  uint32_t t;
#define PQG_SAT_STEP(ctrl, rm, bc)                                         \
  t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, ctrl, rm, 0xf, bc); \
  x = x + t < x ? 0xffffffffu : x + t;
  PQG_SAT_STEP(0x111, 0xf, true) PQG_SAT_STEP(0x112, 0xf, true) PQG_SAT_STEP(0x114, 0xf, true)
  PQG_SAT_STEP(0x118, 0xf, true) PQG_SAT_STEP(0x142, 0xa, false) PQG_SAT_STEP(0x143, 0xc, false)
#undef PQG_SAT_STEP
  return x;
}

// The chain 0 -> next(0) -> ... among 64 speculative positions (next: the
// successor of position `lane`, 64 when it leaves the positions or the item
// there fails) as a mask, by pointer doubling: J_k = next^(2^k) by
// ds_bpermute, then the marks {next^m(0) : m < 32} in five scatter rounds
// through 64 LDS flag bytes F.  Items are >= 2 positions long: <= 32 of them.
__device__ __forceinline__ uint64_t chain_marks64(int next, PQG_L uint8_t* F) {
  const int lane = lane_id();
  uint32_t j[5];
  j[0] = (uint32_t)next;
#pragma unroll
  for (int k = 1; k < 5; k++) {
    const uint32_t q = j[k - 1];
    const uint32_t a = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((q & 63) * 4), (int)q);
    j[k] = q < 64 ? a : 64u;
  }
  F[lane] = lane == 0 ? 1 : 0;
  uint64_t cm = 1;
#pragma unroll
  for (int k = 4; k >= 0; k--) {
    if (((cm >> lane) & 1) && j[k] < 64u) F[j[k]] = 1;
    __builtin_amdgcn_wave_barrier();
    cm = __ballot(F[lane] != 0);
  }
  return cm;
}

template <class Dict>
struct IdxWalk {
  gcu8 p;
  uint32_t n;       // stream bytes
  int w;            // 1..32
  uint32_t count;   // keys wanted (the page's notNull)
  PQG_G uint32_t* out;
  uint32_t dcount;
  Dict dict;
  WalkShared* sh;
  uint32_t wb;                // ring offset of stream byte 0
  int32_t wlo = 0, whi = 0;   // stream offsets [wlo, whi) in the ring (none yet)
  uint32_t bad = 0xffffffffu; // first value whose key is >= dcount
  int serr = kOK;             // stream error met after `produced` keys
  uint32_t produced = 0;
  // the quarter after the window, loaded ahead (one granule per lane)
  uint4 pf = make_uint4(0, 0, 0, 0);
  int32_t pf_at = INT32_MIN;
  // global dictionaries: the previous batch's gathered values, stored after
  // this batch's gathers are issued (vmcnt retires in issue order: a wait for
  // gathers never includes stores issued after them)
  uint32_t pv[8];
  uint32_t pbase = 0, ptot = 0;

  __device__ __forceinline__ uint32_t vmask() const { return w >= 32 ? 0xffffffffu : ((1u << w) - 1); }
  __device__ __forceinline__ bool in_win(uint32_t x, uint32_t len) const {
    return (int64_t)x >= wlo && (int64_t)x + len <= (int64_t)whi;
  }
  __device__ __forceinline__ uint32_t ring_bit(uint32_t x) const { return ((wb + x) & (kIWin - 1)) * 8; }

  // The ring from the 16-byte granule holding stream byte `at`: every load
  // issued before the first is used (a granule holding no stream byte reads
  // the stream's first one); bytes past n are zero (Q5).
  __device__ __forceinline__ void fill(uint32_t at) {
    const int lane = lane_id();
    const uintptr_t pa = (uintptr_t)p;
    const uintptr_t a0 = (pa + at) & ~(uintptr_t)15;
    const int64_t g0 = (int64_t)(a0 - pa);  // > -16
    uint4 v[kIWin / 1024];
#pragma unroll
    for (int k = 0; k < kIWin / 1024; k++) {
      const int64_t g = g0 + 16 * (lane + 64 * k);
      v[k] = ldg16_nt(g < (int64_t)n ? a0 + 16 * (uintptr_t)(lane + 64 * k) : (pa & ~(uintptr_t)15));
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < kIWin / 1024; k++) {
      const int64_t g = g0 + 16 * (lane + 64 * k);
      const uint4 x = g < (int64_t)n ? mask_tail(v[k], g, n) : make_uint4(0, 0, 0, 0);
      const uint32_t o = (uint32_t)((a0 + 16 * (uintptr_t)(lane + 64 * k)) & (kIWin - 1));
      sts16(lds_ptr(sh->win) + (o >> 2), x);
    }
    wlo = (int32_t)g0;
    whi = (int32_t)g0 + kIWin;
    __builtin_amdgcn_wave_barrier();
    prefetch(whi);
  }
  // the 1 KiB quarter at stream offset `at` (16-byte aligned in memory), into pf
  __device__ __forceinline__ void prefetch(int32_t at) {
    const uintptr_t pa = (uintptr_t)p;
    const int64_t g = (int64_t)at + 16 * lane_id();
    pf = ldg16_nt(g < (int64_t)n ? pa + (uintptr_t)g : (pa & ~(uintptr_t)15));
    pf_at = at;
  }
  // The window covers [pos, pos + kINeed) or reaches past the stream's end
  // (the zero bytes there included): the prefetched quarter is written over
  // the quarter the steps have left, and the next one is loaded.
  __device__ __forceinline__ void ensure(uint32_t pos) {
    if (!in_win(pos, 64)) {
      fill(pos);
      return;
    }
    while ((int64_t)pos + kINeed > (int64_t)whi && (int64_t)whi < (int64_t)n + 128) {
      if (pf_at != whi) {
        fill(pos);
        return;
      }
      const int64_t g = (int64_t)whi + 16 * lane_id();
      const uint4 x = g < (int64_t)n ? mask_tail(pf, g, n) : make_uint4(0, 0, 0, 0);
      const uint32_t o = (uint32_t)(((uintptr_t)p + (uintptr_t)g) & (kIWin - 1));
      __builtin_amdgcn_wave_barrier();
      sts16(lds_ptr(sh->win) + (o >> 2), x);
      __builtin_amdgcn_wave_barrier();
      wlo += 1024;
      whi += 1024;
      prefetch(whi);
    }
  }
  // bytes [q, q + 8) of the ring as two dwords
  __device__ __forceinline__ void rd8(uint32_t q, uint32_t& lo, uint32_t& hi) const {
    constexpr uint32_t M = kIWin / 4 - 1;
    const PQG_L uint32_t* W = lds_ptr(sh->win);
    const uint32_t o = wb + q, d = o >> 2, s = (o & 3) * 8;
    const uint32_t a = W[d & M], b = W[(d + 1) & M], c = W[(d + 2) & M];
    lo = __builtin_amdgcn_alignbit(b, a, s);
    hi = __builtin_amdgcn_alignbit(c, b, s);
  }
  // w bits at ring bit `bit` (wraps)
  __device__ __forceinline__ uint32_t bits_at(uint32_t bit) const {
    constexpr uint32_t M = kIWin / 4 - 1;
    const PQG_L uint32_t* W = lds_ptr(sh->win);
    const uint32_t d = bit >> 5;
    return __builtin_amdgcn_alignbit(W[(d + 1) & M], W[d & M], bit & 31) & vmask();
  }
  __device__ __forceinline__ uint32_t byte_at(uint32_t x) {  // wave-uniform x
    if (!in_win(x, 1)) fill(x);
    return (lds_ptr((uint8_t*)sh->win))[(wb + x) & (kIWin - 1)];
  }

  // readUVariant32 + the run's first fields at stream offset q (<= 4-byte
  // headers; longer ones are `cplx`).  Bytes past n read as zero, so a header
  // running past the stream's end terminates at or past n: EOF.
  __device__ __forceinline__ IRun parse(uint32_t q) const {
    uint32_t lo, hi;
    rd8(q, lo, hi);
    IRun r;
    r.err = kOK;
    r.cplx = false;
    const uint32_t cont = ~lo & 0x80808080u;
    const uint32_t hl = cont ? (uint32_t)(__builtin_ctz(cont) >> 3) + 1 : 5u;
    uint32_t h = (lo & 0x7f) | ((lo >> 1) & 0x3f80) | ((lo >> 2) & 0x1fc000) | ((lo >> 3) & 0xfe00000);
    h &= hl >= 4 ? 0xfffffffu : ((1u << (7 * hl)) - 1);
    if (q >= n || (hl <= 4 && q + hl - 1 >= n)) r.err = kEOF;
    else if (hl > 4) r.cplx = true;
    r.bp = (h & 1) != 0;
    const uint32_t g = h >> 1;
    if (r.err == kOK && !r.cplx && g == 0) r.err = kRLE;  // empty run
    if (r.bp) {
      r.cnt = g * 8;  // g < 2^27
      r.pay = q + hl;
      const uint64_t nx = (uint64_t)q + hl + (uint64_t)g * (uint32_t)w;
      r.next = nx > 0xffffffffull ? 0xffffffffu : (uint32_t)nx;
    } else {
      r.cnt = g;
      const uint32_t rb = ((uint32_t)w + 7) >> 3;
      const uint32_t vp = q + hl;
      if (r.err == kOK && !r.cplx && (uint64_t)vp + rb > n) r.err = kEOF;  // readRLERunValue: short read
      const uint64_t x = (uint64_t)lo | (uint64_t)hi << 32;
      const uint32_t vm = rb >= 4 ? 0xffffffffu : ((1u << (8 * rb)) - 1);
      r.pay = (uint32_t)(x >> (8 * (hl < 4 ? hl : 4))) & vm;
      if (r.err == kOK && !r.cplx && w < 32 && (r.pay >> w) != 0) r.err = kRLE;  // value too large
      r.next = vp + rb;
    }
    return r;
  }
  __device__ __forceinline__ int succ(const IRun& r, uint32_t pos) const {
    if (r.err != kOK || r.cplx) return kIPos;
    const uint32_t d = r.next - pos;
    return d < (uint32_t)kIPos ? (int)d : kIPos;
  }

  // Keys of values base + lane + 64 q (q < 8, values < base + total): checked,
  // looked up and stored.  Every lookup of the batch is issued before a store;
  // with a global dictionary the batch's stores wait for the next batch.
  __device__ __forceinline__ void store8(const uint32_t (&v)[8], uint32_t base, uint32_t total) {
    const int lane = lane_id();
    PQG_G uint32_t* o = out + base;
#pragma unroll
    for (int q = 0; q < 8; q++)
      if ((uint32_t)(lane + 64 * q) < total) dict_store(o + lane + 64 * q, v[q]);
  }
  __device__ __forceinline__ void flush() {
    if (Dict::kGlobal && ptot) store8(pv, pbase, ptot);
    ptot = 0;
  }
  __device__ __forceinline__ void sink_keys(uint32_t (&key)[8], uint32_t base, uint32_t total) {
    const int lane = lane_id();
    uint32_t mx = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint32_t j = (uint32_t)(lane + 64 * q);
      key[q] = j < total ? key[q] : 0u;
      mx = key[q] > mx ? key[q] : mx;
    }
    if (__ballot(mx >= dcount)) {
#pragma unroll
      for (int q = 0; q < 8; q++) {
        const uint32_t j = (uint32_t)(lane + 64 * q);
        if (j < total && key[q] >= dcount) bad = base + j < bad ? base + j : bad;
        key[q] = key[q] < dcount ? key[q] : 0u;
      }
    }
    uint32_t val[8];
#pragma unroll
    for (int q = 0; q < 8; q++) val[q] = dict(key[q]);
    if (Dict::kGlobal) {
      flush();
#pragma unroll
      for (int q = 0; q < 8; q++) pv[q] = val[q];
      pbase = base;
      ptot = total;
    } else {
      store8(val, base, total);
    }
  }
  // one key for values [base, base + total)
  __device__ __forceinline__ void sink_rle(uint32_t k, uint32_t base, uint32_t total) {
    const int lane = lane_id();
    if (k >= dcount) bad = base < bad ? base : bad;
    const uint32_t x = dict(k < dcount ? k : 0u);
    PQG_G uint32_t* o = out + base;
    for (uint32_t j = (uint32_t)lane; j < total; j += 64) dict_store(o + j, x);
  }

  // One run of `take` keys from value `produced` on, in pieces of the window.
  __device__ __forceinline__ void long_run(bool bp, uint32_t pay, uint32_t take) {
    if (!bp) {
      sink_rle(pay, produced, take);
      return;
    }
    const int lane = lane_id();
    const uint32_t pmax = min((uint32_t)kISpan, (uint32_t)((kIWin - 32) * 8) / (uint32_t)w);
    for (uint32_t done = 0; done < take;) {
      const uint32_t piece = take - done < pmax ? take - done : pmax;
      const uint64_t b0 = (uint64_t)pay * 8 + (uint64_t)done * (uint32_t)w;
      const uint32_t byte0 = (uint32_t)(b0 >> 3);
      const uint32_t nbytes = (uint32_t)(((uint64_t)piece * (uint32_t)w + 7) >> 3) + 9;
      if (!in_win(byte0, nbytes)) fill(byte0);
      const uint32_t rbit = ring_bit(byte0) + (uint32_t)(b0 & 7);
      uint32_t key[8];
#pragma unroll
      for (int q = 0; q < 8; q++) key[q] = bits_at(rbit + (uint32_t)(lane + 64 * q) * (uint32_t)w);
      sink_keys(key, produced + done, piece);
      done += piece;
    }
  }

  // A run met alone (it does not fit a batch, or its header is > 4 bytes):
  // its take (short bit-packed reads end the stream), its keys, then pos.
  // Returns true when the stream ends here.
  __device__ __forceinline__ bool single_run(bool bp, uint32_t cnt, uint32_t pay, uint32_t nx, uint32_t& pos) {
    const uint32_t left = count - produced;
    uint32_t take = cnt < left ? cnt : left;
    int e = kOK;
    if (bp) {
      const uint64_t need = (take + 7) >> 3;
      if ((uint64_t)pay + (need - 1) * (uint32_t)w >= n) {
        const uint32_t ok = pay < n ? (n - pay + (uint32_t)w - 1) / (uint32_t)w : 0u;
        take = ok * 8;
        e = kEOF;
      }
    }
    if (take) long_run(bp, pay, take);
    produced += take;
    if (e != kOK) {
      serr = e;
      return true;
    }
    pos = nx;
    return false;
  }

  // The header at q walked byte by byte (binary.ReadUvarint + the MaxInt32
  // check, then the run's fields), and its run.  Returns true when the stream ends.
  __device__ __forceinline__ bool serial_run(uint32_t q, uint32_t& pos) {
    uint64_t v = 0;
    unsigned sft = 0;
    uint32_t hl = 0;
    int e = kOK;
    for (uint32_t i = 0;; i++) {
      if (q + i >= n) { e = kEOF; break; }
      const uint32_t b = byte_at(q + i);
      if (b < 0x80) {
        if (i > 9 || (i == 9 && b > 1)) e = kRLE;  // overflows uint64
        else {
          v |= sft < 64 ? (uint64_t)b << sft : 0;
          if (v > 0x7fffffffull) e = kRLE;  // > MaxInt32
        }
        hl = i + 1;
        break;
      }
      if (sft < 64) v |= (uint64_t)(b & 0x7f) << sft;
      sft += 7;
    }
    if (e != kOK) {
      serr = e;
      return true;
    }
    const uint32_t h = (uint32_t)v, g = h >> 1;
    if (g == 0) {
      serr = kRLE;
      return true;
    }
    if (h & 1) {
      const uint64_t nx = (uint64_t)q + hl + (uint64_t)g * (uint32_t)w;
      return single_run(true, g > 0x1fffffffu ? 0xffffffffu : g * 8, q + hl, nx > 0xffffffffull ? 0xffffffffu : (uint32_t)nx,
                        pos);
    }
    const uint32_t rb = ((uint32_t)w + 7) >> 3, vp = q + hl;
    if ((uint64_t)vp + rb > n) {
      serr = kEOF;
      return true;
    }
    uint32_t val = 0;
    for (uint32_t k = 0; k < rb; k++) val |= byte_at(vp + k) << (8 * k);
    if (w < 32 && (val >> w) != 0) {
      serr = kRLE;
      return true;
    }
    return single_run(false, g, val, vp + rb, pos);
  }

  // Keys of the chain runs in mask m (run 0 among them) from value
  // `produced` on; returns the values emitted and the next header position.
  // Per lane, the run's first value s, its take k, its next header, and its
  // key source te = {bit-packed flag, payload bit in the ring | RLE value}.
  __device__ __forceinline__ uint32_t emit(uint64_t m, uint32_t s, uint32_t k, uint32_t nx, bool bp, uint32_t info, uint32_t& nxt) {
    const int lane = lane_id();
    const int ll = 63 - __builtin_clzll(m);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)s, ll) + (uint32_t)__builtin_amdgcn_readlane((int)k, ll);
    nxt = (uint32_t)__builtin_amdgcn_readlane((int)nx, ll);
    if (total == 0) return 0;
    uint32_t key[8];
    if (m == 1) {  // run 0 alone
      const uint32_t inf = (uint32_t)__builtin_amdgcn_readfirstlane((int)info);
      if (!__builtin_amdgcn_readfirstlane((int)bp)) {
        sink_rle(inf, produced, total);
        return total;
      }
#pragma unroll
      for (int q = 0; q < 8; q++) key[q] = bits_at(inf + (uint32_t)(lane + 64 * q) * (uint32_t)w);
      sink_keys(key, produced, total);
      return total;
    }
    // several runs: run marks at their first values, then a prefix max
    PQG_L uint8_t* TM = lds_ptr(sh->tm);
    PQG_L u32x2_t* TE = lds_ptr(sh->te);
    __builtin_amdgcn_wave_barrier();
    *(PQG_L u32x2_t*)(TM + 8 * lane) = u32x2_t{0u, 0u};
    __builtin_amdgcn_wave_barrier();
    if (((m >> lane) & 1) && k > 0) {
      TE[lane] = u32x2_t{s | (bp ? 0x80000000u : 0u), info};
      TM[s] = (uint8_t)(lane + 1);
    }
    __builtin_amdgcn_wave_barrier();
    const u32x2_t mk = *(const PQG_L u32x2_t*)(TM + 8 * lane);
    uint32_t run_max = 0, ix[2] = {0u, 0u};
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint32_t mm = ((q < 4 ? mk.x : mk.y) >> (8 * (q & 3))) & 0xff;
      run_max = mm > run_max ? mm : run_max;
      ix[q >> 2] |= run_max << (8 * (q & 3));
    }
    const uint32_t before = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ldpp_incl_max_u32(run_max), 0x138, 0xf, 0xf, false);
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint32_t mm = (ix[q >> 2] >> (8 * (q & 3))) & 0xff;
      if (mm < before) ix[q >> 2] = (ix[q >> 2] & ~(0xffu << (8 * (q & 3)))) | (before << (8 * (q & 3)));
    }
    __builtin_amdgcn_wave_barrier();
    *(PQG_L u32x2_t*)(TM + 8 * lane) = u32x2_t{ix[0], ix[1]};
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint32_t j = (uint32_t)(lane + 64 * q);
      const uint32_t r = TM[j];  // >= 1 for every value of the batch
      const u32x2_t te = TE[(r - 1) & (kIPos - 1)];
      const uint32_t bits = bits_at(te.y + (j - (te.x & 0x7fffffffu)) * (uint32_t)w);
      key[q] = (te.x & 0x80000000u) ? bits : te.y;
    }
    sink_keys(key, produced, total);
    return total;
  }

  __device__ __forceinline__ void run() {
    walk();
    flush();
  }
  __device__ __forceinline__ void walk() {
    const int lane = lane_id();
    uint32_t pos = 0;
    while (produced < count) {
      if (pos >= n) {
        serr = kEOF;
        return;
      }
      ensure(pos);
      const uint32_t left = count - produced;
      // ---- 1-2. speculative headers and the chain
      const IRun r = parse(pos + (uint32_t)lane);
      const int nx = succ(r, pos);
      uint64_t cm = 1;
      if (__builtin_amdgcn_readfirstlane(nx) < kIPos) cm = chain_marks64(nx, lds_ptr(sh->cflag));
      const bool on = (cm >> lane) & 1;
      // ---- 3. first values, takes, checks
      const uint32_t c = on ? r.cnt : 0u;
      const uint32_t st = dpp_incl_add_sat(c) - c;  // values before the run (chain runs)
      int e = kOK;
      uint32_t take = 0;
      bool cut = false;
      const bool need = on && st < left;
      if (need) {
        if (r.cplx) e = kCOMPLEX;
        else if (r.err != kOK) e = r.err;
        else {
          take = r.cnt < left - st ? r.cnt : left - st;
          if (r.bp) {
            const uint64_t ng = (take + 7) >> 3;
            if ((uint64_t)r.pay + (ng - 1) * (uint32_t)w >= n) {  // short read: the groups that start in the stream
              const uint32_t ok = r.pay < n ? (n - r.pay + (uint32_t)w - 1) / (uint32_t)w : 0u;
              take = ok * 8;
              e = kEOF;  // after its `take` keys
            }
            const uint64_t pend = (uint64_t)r.pay + (((uint64_t)take * (uint32_t)w + 7) >> 3) + 8;
            cut = (int64_t)r.pay < wlo || (int64_t)pend > (int64_t)whi;
          }
          cut |= st + take > (uint32_t)kISpan;
        }
      }
      const uint64_t eb = __ballot(e != kOK), xb = __ballot(cut), nb = __ballot(need);
      const int first_err = eb ? __ffsll((long long)eb) - 1 : kIPos;
      const int first_cut = xb ? __ffsll((long long)xb) - 1 : kIPos;
      auto below = [](int lim) { return lim >= 64 ? ~0ull : ((1ull << lim) - 1); };
      const uint32_t info = r.bp ? ring_bit(r.pay) : r.pay;
      uint32_t nxt = pos;
      if (first_cut < kIPos && first_cut <= first_err) {
        if (first_cut == 0) {  // run 0 alone is longer than a batch or leaves the window
          if (single_run(__builtin_amdgcn_readfirstlane((int)r.bp) != 0, (uint32_t)__builtin_amdgcn_readfirstlane((int)r.cnt),
                         (uint32_t)__builtin_amdgcn_readfirstlane((int)r.pay),
                         (uint32_t)__builtin_amdgcn_readfirstlane((int)r.next), pos))
            return;
          continue;
        }
        produced += emit(nb & below(first_cut), st, take, r.next, r.bp, info, nxt);
        pos = nxt;
        continue;
      }
      if (first_err < kIPos) {
        const int ee = __builtin_amdgcn_readlane(e, first_err);
        if (ee == kCOMPLEX) {  // the runs before it, then its header byte by byte
          const uint64_t m = nb & below(first_err);
          if (m) produced += emit(m, st, take, r.next, r.bp, info, nxt);
          if (serial_run(pos + (uint32_t)first_err, pos)) return;
          continue;
        }
        // the runs up to the failing one (its own keys: a short bit-packed run's)
        produced += emit(nb & below(first_err + 1), st, take, r.next, r.bp, info, nxt);
        serr = ee;
        return;
      }
      produced += emit(nb, st, take, r.next, r.bp, info, nxt);
      pos = nxt;
    }
  }
};

// Read phase of every 4-byte dictionary page in the list, and its VRec at the
// page's list position (valuesDecoder.init type_dict.go:22-37: the bit-width
// byte, > 32 is an error).
// One VRec per work item (a page's part, k_part_plan): a part of a big page is
// its blocks [b0, next part's b0) and values [v0, next part's v0).
// walk_small: pages of <= kSplitMin values were not walked by k_hybrid_walk
// (dict_walk_page): k_dict_walk / k_dict_walk_g walk their streams (VRec.n_blocks < 0).
__global__ void __launch_bounds__(256) k_dict_plan(JobDev* jobs, PageDev* pages, const PartRec* parts, const int* total,
                                                   uint8_t* value_arena, const HStream* streams, const RunEnt* runs,
                                                   const BlockDesc* blks, VRec* recs, int walk_small) {
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
          if (dw > 0 && walk_small && dict_walk_page(P)) {
            const HStream& S = streams[P.hs_val];
            r.p = S.p;
            r.n = (int32_t)S.n;
            r.runs = nullptr;  // walked in k_dict_walk
            r.blks = nullptr;
            // k_dict_walk: a dictionary that fits LDS; k_dict_walk_g: any other
            r.n_blocks = (r.dict && r.dcount >= 1 && r.dcount <= kDictLdsEntries) ? -1 : -2;
            r.count = r.nn;
            r.produced = r.nn;
            r.serr = kOK;
          } else if (dw > 0) {
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
          }
        }
      }
    }
    recs[t] = r;
  }
}

// Mode 1 pages (4-byte dictionary columns): the C2 path, kDWaves * 64 threads
// per workgroup taking kDWaves consecutive work items.  kMode (DictShared):
// 0 = pages with run tables (k_dict4), 1 / 2 = small pages whose index
// streams are walked here (k_dict_walk / k_dict_walk_g, VRec.n_blocks -1 /
// -2).  Separate kernels, so each is compiled for its own register and LDS
// budget.
__device__ __forceinline__ void dict_fill0(const VRec& r, int lane, int& de) {
  // a zero-width decoder yields key 0 forever, reading nothing (hybrid_decoder.go:84-86)
  if (r.dcount < 1) de = kDICT_INDEX;
  else {
    const uint32_t d0 = *(const PQG_G uint32_t*)gconst(r.dict);
    for (int64_t i = lane; i < r.nn; i += 64) ((PQG_G uint32_t*)gmut(r.out))[i] = d0;
  }
}

template <class Dict>
__device__ __forceinline__ int walk_dict_page(VRec& r, WalkShared& ws, const Dict& dict) {
  IdxWalk<Dict> iw{gconst(r.p), (uint32_t)r.n, r.w, (uint32_t)r.nn, (PQG_G uint32_t*)gmut(r.out), (uint32_t)r.dcount,
                   dict, &ws, (uint32_t)((uintptr_t)r.p & (kIWin - 1))};
  iw.run();
  // keys are checked only among the produced ones: a bad key comes first
  const int64_t bad = wave_min((int64_t)iw.bad);
  if (bad < r.nn) return kDICT_INDEX;
  return iw.produced < (uint32_t)r.nn ? iw.serr : kOK;
}

template <int kMode>
__device__ __forceinline__ void dict_items(PageDev* pages, const int* total, int* queue, const VRec* recs) {
  __shared__ __attribute__((aligned(16))) DictShared<kMode> sh;
  const int lane = lane_id(), wid = (int)(threadIdx.x >> 6);
  if (total[kModePresentOff + 1] == 0) return;  // no page of this stage
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
    const int own = kMode == 0 ? (r.n_blocks >= 0) : kMode == 1 ? (r.n_blocks == -1) : (r.n_blocks == -2);
    if (!own) r.job = -1;  // another kernel's page
    PQG_DT(t1);
    pf.add(2, t1 - t0);
    if constexpr (kMode == 2) {
      __syncthreads();  // sh.item is read
      if (r.job < 0) continue;
      int de = kOK;
      if (r.w == 0) dict_fill0(r, lane, de);
      else {
        const PQG_G uint32_t* dsafe = (const PQG_G uint32_t*)(r.dict ? gconst(r.dict) : gconst(r.out));
        de = walk_dict_page(r, sh.w[wid], GlobalDict{dsafe});
      }
      if (lane == 0 && de != kOK) atomicMin(&pages[r.pidx].decode_status, de);
      continue;
    } else {
    // ---- kMode 0 / 1: the dictionaries of the item's pages into LDS, one job
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
        if (dc > 0 && dc <= kDictLdsEntries) {
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
        } else if constexpr (kMode == 1) {
          // k_dict_plan gives this kernel only pages whose dictionary fits LDS
          de = lds ? walk_dict_page(r, sh.w[wid], LdsDict{lds_ptr(sh.dict)}) : kCAPACITY;
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

__global__ void __attribute__((amdgpu_flat_work_group_size(1, kDWaves * 64), amdgpu_waves_per_eu(PQG_DICT_WPE)))
k_dict4(PageDev* pages, const int* total, int* queue, const VRec* recs) {
  dict_items<0>(pages, total, queue, recs);
}

#ifndef PQG_DICT_WALK_WPE
#define PQG_DICT_WALK_WPE 3
#endif
#ifndef PQG_DICT_WALKG_WPE
#define PQG_DICT_WALKG_WPE 3
#endif
__global__ void __attribute__((amdgpu_flat_work_group_size(1, kDWaves * 64), amdgpu_waves_per_eu(PQG_DICT_WALK_WPE)))
k_dict_walk(PageDev* pages, const int* total, int* queue, const VRec* recs) {
  dict_items<1>(pages, total, queue, recs);
}
__global__ void __attribute__((amdgpu_flat_work_group_size(1, kDWaves * 64), amdgpu_waves_per_eu(PQG_DICT_WALKG_WPE)))
k_dict_walk_g(PageDev* pages, const int* total, int* queue, const VRec* recs) {
  dict_items<2>(pages, total, queue, recs);
}

}  // namespace pqg
