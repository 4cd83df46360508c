// pqg_levels.hip — K3: page setup, level decode, the RLE/bit-packed hybrid
// run walk of the value streams, and the notNull scan.
//
//   K3a k_page_levels    one wave per data page: the read phase of the page
//                        (V1 initSize: page_v1.go:99-105, hybrid_decoder.go:57-67;
//                        V2 raw level bytes: page_v2.go:103-121), registration
//                        of its value stream (dictionary indices
//                        type_dict.go:22-37, RLE booleans type_boolean.go:100-120),
//                        then rep and def levels decoded straight into the level
//                        arenas (hybridDecoder.next, hybrid_decoder.go:82-166;
//                        decodePackedArray helpers.go:131-147), notNull = #(def == maxD)
//   K3b k_hybrid_walk    one LANE per value stream: the serial run-header walk
//                        writes a run table and a block index for the values
//                        kernels (pqg_hybrid.h)
//   K3d k_nn_scan        per chunk: value offsets = exclusive scan of notNull
//                        (readPageData chunk_reader.go:380-402) and the
//                        dictionary page (page_dict.go:30-64)
#include <hip/hip_runtime.h>

#include "pqg_common.h"
#include "pqg_device.h"
#include "pqg_hybrid.h"
#include "pqg_levdec.h"
#include "pqg_lev1.h"
#include <type_traits>

namespace pqg {

#ifndef PQG_LEVELS_WPE
#define PQG_LEVELS_WPE 6  // minimum waves per SIMD the register allocation must allow
#endif

#ifdef PQG_PROFILE
// host reader of this translation unit's phase counters (see pqg_debug_counters)
int prof_read_levels(unsigned long long* out) {
  unsigned long long z[64] = {0};
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pqg_prof), sizeof(z)) != hipSuccess) return -1;
  hipMemcpyToSymbol(HIP_SYMBOL(pqg_prof), z, sizeof(z));
  return 0;
}
#endif

// ---- K3b ---------------------------------------------------------------------
// One lane walks one stream.  The lane's window on its stream: 64-byte chunks
// (16-byte aligned in memory); the chunk holding `pos` and the next one sit in
// two LDS slots and the one after is prefetched into registers, so the walk
// waits on global memory about once per 64 bytes, for a load issued a chunk
// earlier.  Positions are 32-bit (a page is < 2 GiB: its sizes are thrift
// i32); the per-run path is kept short because a single wave per SIMD walks
// it with nothing to hide its latency behind.
// one lane per stream: small blocks spread the (latency-bound) lanes over
// every CU instead of one 256-lane block on each of the first few

#ifndef PQG_LANE_WIN
#define PQG_LANE_WIN 8
#endif
constexpr int kLaneWinG = PQG_LANE_WIN;  // 16-byte granules of a lane's window (128 bytes)
struct LaneWin {
  gcu8 p;
  uint32_t n;
  uint32_t base;           // stream offset of window byte 0 (16-aligned address; may precede the stream: wraps)
  PQG_L uint32_t* r;       // dword k of the window at r[64 k]
  // The window at the granule holding stream byte pos.  Every load is issued
  // unconditionally before the first is used (a granule past the stream
  // re-reads its last one, mapped): the loads of a lane then cost one wait —
  // which also waits for the lane's earlier level stores, vmcnt retiring in
  // order — instead of one per guarded load.
  __device__ __forceinline__ void fill(uint32_t pos) {
    const uint32_t mis = (uint32_t)((uintptr_t)(p + pos) & 15);
    base = pos - mis;
    const uintptr_t a0 = (uintptr_t)(p + pos) - mis;
    const uintptr_t last = ((uintptr_t)(p + n) - 1) & ~(uintptr_t)15;  // n > pos >= 0
    uint4 g[kLaneWinG];
#pragma unroll
    for (int k = 0; k < kLaneWinG; k++) {
      const uintptr_t a = a0 + 16 * k;
      g[k] = ldg16(a <= last ? a : last);
    }
#pragma unroll
    for (int k = 0; k < kLaneWinG; k++) {
      const uint4 v = mask_tail(g[k], (int64_t)pos - mis + 16 * k, n);  // bytes past n read as zero (Q5)
      r[64 * (4 * k + 0)] = v.x;
      r[64 * (4 * k + 1)] = v.y;
      r[64 * (4 * k + 2)] = v.z;
      r[64 * (4 * k + 3)] = v.w;
    }
  }
  __device__ __forceinline__ void ensure(uint32_t pos) {
    if (pos - base > 16 * kLaneWinG - 16) fill(pos);
  }
  // 12 bytes at stream offset pos (window already holding [pos, pos + 16))
  __device__ __forceinline__ void read12(uint32_t pos, uint32_t& a, uint32_t& b, uint32_t& c) const {
    const uint32_t off = pos - base;
    const uint32_t d = off >> 2, sh = (off & 3) * 8;
    const uint32_t x0 = r[64 * d], x1 = r[64 * (d + 1)], x2 = r[64 * (d + 2)], x3 = r[64 * (d + 3)];
    a = __builtin_amdgcn_alignbit(x1, x0, sh);
    b = __builtin_amdgcn_alignbit(x2, x1, sh);
    c = __builtin_amdgcn_alignbit(x3, x2, sh);
  }
  __device__ __forceinline__ void peek12(uint32_t pos, uint32_t& a, uint32_t& b, uint32_t& c) {
    ensure(pos);
    read12(pos, a, b, c);
  }
};

// The lanes of a wave refill their windows together: a lane whose next read
// leaves its window votes, and then every lane that reads this step refills
// at its read position.  Each refill waits for the wave's earlier stores
// (vmcnt retires in order), so per-lane refills at scattered steps would stall
// the wave on memory almost every step; together they cost one stall per
// window's worth of progress of the fastest lane.
__device__ __forceinline__ void sync_ensure(LaneWin& w, bool reads, uint32_t rp) {
  const bool need = reads && rp - w.base > 16 * kLaneWinG - 16;
  if (__ballot(need) != 0 && reads) w.fill(rp);
}

// Lanes [0, total) walk the rep streams, [total, 2 total) the def streams,
// [2 total, 3 total) the value streams, so a wave's lanes do alike work.
__global__ void __launch_bounds__(kWalkThreads) k_hybrid_walk(const PageDev* pages, const int* list, const int* total,
                                                              HStream* streams, RunEnt* runs, BlockDesc* blks,
                                                              LongWalk* longs, int long_cap) {
  static_assert(kWalkThreads == 64, "LaneWin: dword k of lane L at buf[64 k + L]");
  __shared__ uint32_t buf[4 * kLaneWinG * kWalkThreads];  // each lane's 128-byte window (LaneWin)
  const int nt = *total;
  int* const n_long = const_cast<int*>(total) + kCtrLongWalk;
  // level streams are decoded in place by k_page_levels: only the value streams
  // (dictionary indices, RLE booleans) are walked
  for (int g = blockIdx.x * kWalkThreads + threadIdx.x; g < nt; g += gridDim.x * kWalkThreads) {
    const PageDev& pg = pages[list[g]];
    const int hs = pg.hs_val;
    if (hs < 0) continue;
    HStream& S = streams[hs];
    const uint32_t w = (uint32_t)S.w;
    const uint32_t n = (uint32_t)S.n, count = (uint32_t)S.count;
    const uint32_t rb = (w + 7) >> 3;
    const uint64_t vmask = rb >= 4 ? 0xffffffffull : ((1ull << (8 * rb)) - 1);
    PQG_G uint32_t* R = (PQG_G uint32_t*)(gmut(runs) + S.run_base);
    PQG_G uint32_t* B = (PQG_G uint32_t*)(gmut(blks) + S.blk_base);
    LaneWin rd{gconst(S.p), n, 0xfffffff0u, lds_ptr(buf) + threadIdx.x};
    if (n > 0) rd.fill(0);
    uint32_t pos = 0, produced = 0, nr = 0;
    int status = kOK;
    // block under construction (see BlockDesc)
    uint32_t nb = 0, bv0 = 0, br0 = 0, bn = 0;
    uint64_t blo = ~0ull, bhi = 0;
    auto close_block = [&]() {
      if (bn == 0) return;
      const uint32_t lo = blo == ~0ull ? 0u : (uint32_t)blo;
      const uint32_t nbytes = blo == ~0ull ? 0u : (uint32_t)(bhi - blo);
      PQG_G uint32_t* d = B + 4 * nb;
      stg16((uintptr_t)d, make_uint4(bv0, br0, lo, (nbytes & 0xffff) | (bn << 16)));
      nb++;
    };
    while (produced < count) {
      // hybridDecoder.next: run header = readUVariant32 (helpers.go:149-165)
      if (pos >= n) { status = kEOF; break; }
      sync_ensure(rd, true, pos);
      uint32_t xa, xb, xc;
      rd.read12(pos, xa, xb, xc);
      uint64_t x = (uint64_t)xa | (uint64_t)xb << 32;
      uint32_t h, hl;
      if ((x & 0x80) == 0) {
        h = (uint32_t)x & 0x7f;
        hl = 1;
      } else {  // multi-byte header: exactly binary.ReadUvarint + the MaxInt32 check
        uint64_t v = 0;
        unsigned sft = 0;
        int e = kOK;
        hl = 0;
        for (uint32_t i = 0;; i++) {
          if (pos + i >= n) { e = kEOF; break; }
          uint32_t b;
          if (i < 8) {
            b = (uint32_t)(x >> (8 * i)) & 0xff;
          } else {
            uint32_t ya, yb, yc;
            rd.peek12(pos + i, ya, yb, yc);
            b = ya & 0xff;
          }
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
        if (e) { status = e; break; }
        h = (uint32_t)v;
        {
          uint32_t ya, yb, yc;
          rd.peek12(pos + hl, ya, yb, yc);
          x = ((uint64_t)ya | (uint64_t)yb << 32) << 8;  // the RLE value at byte 1, like the fast path
        }
      }
      pos += hl;
      uint32_t take, st, src;
      const uint32_t left = count - produced;
      if (h & 1) {  // bit-packed: h>>1 groups of 8 values, w bytes each
        const uint32_t groups = h >> 1;
        if (groups == 0) { status = kRLE; break; }  // "empty bit-packed run"
        take = groups >= (left + 7) >> 3 ? left : groups * 8;
        const uint32_t need = (take + 7) >> 3;
        // every group read must start inside the stream; a short one is zero padded (Q5)
        if ((uint64_t)pos + (uint64_t)(need - 1) * w >= n) {
          const uint32_t ok = pos < n ? (n - pos + w - 1) / w : 0;
          take = ok * 8;
          status = kEOF;
        }
        st = produced | kRunBP;
        src = pos;
        pos = (uint64_t)pos + (uint64_t)groups * w > 0xffffffffull ? 0xffffffffu : pos + groups * w;
      } else {  // RLE: h>>1 repeats of a ceil(w/8)-byte little-endian value
        const uint32_t cnt = h >> 1;
        if (cnt == 0) { status = kRLE; break; }
        if (pos >= n || n - pos < rb) { status = kEOF; break; }
        src = (uint32_t)((x >> 8) & vmask);
        pos += rb;
        if (w < 32 && (src >> w) != 0) { status = kRLE; break; }  // readRLERunValue :127-129
        take = cnt < left ? cnt : left;
        st = produced;
      }
      if (take > 0) {
        stg8((uintptr_t)(R + 2 * nr), st, src);
        const uint32_t rend = produced + take;
        if ((st & kRunBP) && take > (uint32_t)kLongWalk) {
          // a long bit-packed run (parquet-go's writer: the whole stream): its
          // blocks of K values each are written by k_walk_long in parallel
          const uint32_t K = min((uint32_t)kHBlock, ((8u * kHBlockBytes - 14u) / w) & ~7u);
          const uint32_t R = (take + K - 1) / K;
          const int li = atomicAdd(n_long, 1);
          if (li < long_cap) {
            close_block();
            LongWalk L;
            L.blk = S.blk_base + nb;
            L.v0 = produced;
            L.take = take;
            L.run = nr;
            L.src = src;
            L.w = (int32_t)w;
            L.K = (int32_t)K;
            longs[li] = L;
            nb += R;
            bv0 = rend;  // the next run opens a new block
            br0 = nr + 1;
            bn = 0;
            blo = ~0ull;
            bhi = 0;
            produced = rend;
            nr++;
            if (status) break;
            continue;
          }
        }
        // the run joins the open block, and every block it reaches into
        for (uint32_t v = produced; v < rend;) {
          if (bn == kHBlockRuns || v >= bv0 + kHBlock) {
            close_block();
            bv0 = v;
            br0 = nr;
            bn = 0;
            blo = ~0ull;
            bhi = 0;
          }
          uint32_t pe = rend < bv0 + kHBlock ? rend : bv0 + kHBlock;
          if (st & kRunBP) {
            const uint64_t rbit = (uint64_t)src * 8;  // bit of the run's value 0
            const uint64_t b0 = (rbit + (uint64_t)(v - produced) * w) >> 3;
            const uint64_t org = blo < b0 ? blo : b0;
            // values whose bits end within org + kHBlockBytes
            const uint64_t lim = (org + kHBlockBytes) * 8;
            const uint64_t fit = lim > rbit ? (lim - rbit) / w : 0;  // values [0, fit) of the run fit
            if (produced + fit <= v) {  // not even one more value: start a new block here
              close_block();
              bv0 = v;
              br0 = nr;
              bn = 0;
              blo = ~0ull;
              bhi = 0;
              continue;
            }
            if (produced + fit < pe) pe = (uint32_t)(produced + fit);
            const uint64_t b1 = (rbit + (uint64_t)(pe - produced) * w + 7) >> 3;
            blo = org;
            bhi = b1 > bhi ? b1 : bhi;
          }
          bn++;
          v = pe;
        }
        produced = rend;
        nr++;
      }
      if (status) break;
    }
    close_block();
    S.n_runs = (int32_t)nr;
    S.produced = (int32_t)produced;
    S.status = status;
    S.n_blocks = (int32_t)nb;
  }
}

// The block descriptors of the long bit-packed runs k_hybrid_walk handed
// over: block j of a run holds values [v0 + j K, v0 + min((j + 1) K, take)),
// one run, its payload bytes from the bit of its first value.  Every thread of
// the grid takes blocks of every run.
__global__ void __launch_bounds__(256) k_walk_long(const int* ctr, const LongWalk* longs, int long_cap,
                                                   BlockDesc* blks) {
  const int n = min(ctr[kCtrLongWalk], long_cap);
  const uint32_t tid = blockIdx.x * 256 + threadIdx.x, stride = gridDim.x * 256;
  for (int r = 0; r < n; r++) {
    const LongWalk L = longs[r];
    const uint32_t R = (L.take + (uint32_t)L.K - 1) / (uint32_t)L.K;
    for (uint32_t j = tid; j < R; j += stride) {
      const uint32_t a = j * (uint32_t)L.K;
      const uint32_t cnt = min((uint32_t)L.K, L.take - a);
      const uint64_t bit0 = (uint64_t)L.src * 8 + (uint64_t)a * (uint32_t)L.w;
      const uint64_t lo = bit0 >> 3, hi = (bit0 + (uint64_t)cnt * (uint32_t)L.w + 7) >> 3;
      stg16((uintptr_t)(blks + L.blk + j),
            make_uint4(L.v0 + a, L.run, (uint32_t)lo, (uint32_t)(hi - lo) | (1u << 16)));
    }
  }
}

// Long level runs (more than kLongLev values, recorded by k_page_levels):
// one wave per piece of kLevPiece values, 16 values per lane per step; the
// level bytes leave as aligned 16-byte granules (the piece's ragged ends
// byte by byte), notNull is added to the page.
__global__ void __launch_bounds__(64) k_level_long(PageDev* pages, const int* ctr, const LongLev* longs, int long_cap,
                                                   const LevPiece* pieces, int piece_cap, int* queue) {
  const int lane = lane_id();
  const int np = min(ctr[kCtrLevPieces], piece_cap);
  for (;;) {
    const int t = queue_next(queue);
    if (t >= np) return;
    const LevPiece pc = pieces[t];
    if (pc.run < 0 || pc.run >= long_cap) continue;
    const LongLev L = longs[pc.run];
    if (pages[L.pidx].decode_status != kOK) continue;  // a failing page: its levels are not used
    const uintptr_t ob = (uintptr_t)L.out;
    const uint32_t mask = (1u << L.w) - 1;
    const int64_t navail = L.p ? (int64_t)(L.end - L.p) : 0;
    uint32_t nn = 0;
    const uintptr_t a0 = (ob + pc.v0) & ~(uintptr_t)15;
    for (uintptr_t a = a0 + 16 * (uintptr_t)lane; a < ob + pc.v1; a += 1024) {
      const int64_t i0 = (int64_t)(a - ob);  // value of the granule's byte 0 (may be < v0)
      uint32_t v[16];
      if (L.p) {
        const int64_t ib = i0 < 0 ? 0 : i0;
        const int64_t bit = ib * L.w;
        const gcu8 p = gconst(L.p);
        const uint64_t x0 = load_u64_masked(p, navail, bit >> 3, navail);
        const uint64_t x1 = load_u64_masked(p, navail, (bit >> 3) + 8, navail);
        const uint32_t sh = (uint32_t)(bit & 7);
        const int64_t shift0 = (i0 < 0 ? -i0 : 0) * L.w;  // granule values before value 0 (never stored)
#pragma unroll
        for (int k = 0; k < 16; k++) {
          const int64_t b = (int64_t)sh + (int64_t)k * L.w - shift0;
          uint32_t x = 0;
          if (b >= 0) {
            x = b < 64 ? (uint32_t)(x0 >> b) | (b > 56 ? (uint32_t)(x1 << (64 - b)) : 0u) : (uint32_t)(x1 >> (b - 64));
          }
          v[k] = x & mask;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = L.value;
      }
      uint32_t wv[4];
#pragma unroll
      for (int k = 0; k < 4; k++) wv[k] = v[4 * k] | v[4 * k + 1] << 8 | v[4 * k + 2] << 16 | v[4 * k + 3] << 24;
      if (i0 >= (int64_t)pc.v0 && i0 + 16 <= (int64_t)pc.v1) {
        stg16o(a, make_uint4(wv[0], wv[1], wv[2], wv[3]));
#pragma unroll
        for (int k = 0; k < 16; k++) nn += v[k] == (uint32_t)L.maxl;
      } else {
#pragma unroll
        for (int k = 0; k < 16; k++) {
          if (i0 + k >= (int64_t)pc.v0 && i0 + k < (int64_t)pc.v1) {
            *(PQG_G uint8_t*)(a + k) = (uint8_t)v[k];
            nn += v[k] == (uint32_t)L.maxl;
          }
        }
      }
    }
    const int64_t tot = wave_sum((int64_t)nn);
    if (lane == 0 && L.maxl <= 255 && tot) atomicAdd(&pages[L.pidx].not_null, (int32_t)tot);
  }
}

// Setup and the level decode of one data page per wave (the speculative
// window parse above).  (A lane-per-page walk of the level streams was tried
// and dropped: with one lane per page a 35 000-page batch fills ~550 waves,
// and each lane's serial walk of ~1 100 runs and 1 250 granules ran 4x slower
// than this kernel: DESIGN.md.)
// Two instances: k_page_levels_w1 for the pages of jobs whose levels are at
// most 1 bit wide (maxR = 0, maxD <= 1: optional flat columns, required
// columns) — the w = 1 decoder alone, 64 VGPRs and 8 waves per SIMD without
// spills — and k_page_levels for every other page.  `split`: both kernels run
// on one list, each taking its own jobs' pages (0: this kernel takes all).
__device__ __forceinline__ bool w1_job(const JobDev& job) { return job.max_rep == 0 && job.max_def <= 1; }

// k_page_levels_w1's LDS: the whole-page decoder's window and table, or the
// batch decoder's (pages the whole-page decoder does not take)
union LevW1Shared {
  LevShared lev;
  Lev1Shared l1;
};
template <bool kW1>
using LevelsShared = typename std::conditional<kW1, LevW1Shared, LevShared>::type;
__device__ __forceinline__ LevShared& lev_sh(LevShared& s) { return s; }
__device__ __forceinline__ LevShared& lev_sh(LevW1Shared& s) { return s.lev; }

// split: bit 0 = both kernels run on one list, each taking its own jobs'
// pages; bit 1 (w = 1 kernel) = the whole-page decoder first (pqg_lev1.h)
template <bool kW1>
__device__ __forceinline__ void page_levels(JobDev* jobs, PageDev* pages, const int* list, const int* total, int* queue,
                                            uint8_t* scratch, HStream* streams, uint8_t* def_arena, uint8_t* rep_arena,
                                            LongLev* longs, int long_cap, LevPiece* pieces, int piece_cap, int split_flags) {
  __shared__ __attribute__((aligned(16))) LevelsShared<kW1> shu;
  LevShared& sh = lev_sh(shu);
  const int split = split_flags & 1;
  const bool whole = kW1 && (split_flags & 2);
  const int lane = lane_id();
  const LongTables lt{longs, pieces, const_cast<int*>(total), long_cap, piece_cap};
  for (;;) {
    const int t = queue_next(queue);
    if (t >= *total) return;
    const int pidx = __builtin_amdgcn_readfirstlane(list[t]);
    const PageDev pg = pages[pidx];
    const JobDev job = jobs[pg.job];
    if (split && w1_job(job) != kW1) continue;  // the other kernel's page
    if (lane == 0) {
      pages[pidx].hs_rep = pages[pidx].hs_def = pages[pidx].hs_val = -1;
      pages[pidx].vmode = -1;
    }
    if (pg.read_status != kOK || (pg.page_type != 0 && pg.page_type != 3)) continue;
    if (job.status == kCAPACITY) continue;
    const PageStreams ps = page_setup(job, pg, pidx, pages, streams, total, scratch, lane == 0);
    if (ps.e != kOK) continue;
    const int64_t n = pg.num_values;
    // ---- readValues (page_v1.go:27-55): rep levels, then def levels
    int64_t nn = 0;
    int de = kOK;
    if (n > 0) {
      if (!kW1 && job.max_rep > 0) {
        if (ps.rep_n < 0) de = kLEVELS;  // V2 with no rep-level bytes: "reader is not initialized"
        else {
          uint32_t unused;
          de = level_stream<kW1>(ps.rep, ps.rep_n, bits_len((uint32_t)job.max_rep), (uint32_t)n,
                                 gmut(rep_arena) + job.slot_base + pg.slot_offset, 0x100u, sh, &unused, lt, pidx);
        }
      }
      if (de == kOK) {
        if (job.max_def > 0) {
          if (ps.def_n < 0) de = kLEVELS;
          else {
            uint32_t c = 0;
            bool done = false;
            if constexpr (kW1) {
              if (whole && job.max_def == 1 && ps.def_n <= kL1MaxN)
                done = lev1_page(ps.def, (uint32_t)ps.def_n, (uint32_t)n,
                                 gmut(def_arena) + job.slot_base + pg.slot_offset, shu.l1, &c);
            }
            if (done) de = kOK;
            else
              de = level_stream<kW1>(ps.def, ps.def_n, bits_len((uint32_t)job.max_def), (uint32_t)n,
                                     gmut(def_arena) + job.slot_base + pg.slot_offset, (uint32_t)job.max_def, sh, &c,
                                     lt, pidx);
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
  }
}

__global__ void __launch_bounds__(64, PQG_LEVELS_WPE) k_page_levels(JobDev* jobs, PageDev* pages, const int* list, const int* total,
                                                    int* queue, uint8_t* scratch, HStream* streams,
                                                    uint8_t* def_arena, uint8_t* rep_arena, LongLev* longs,
                                                    int long_cap, LevPiece* pieces, int piece_cap, int split) {
  page_levels<false>(jobs, pages, list, total, queue, scratch, streams, def_arena, rep_arena, longs, long_cap, pieces,
                     piece_cap, split);
}

#ifndef PQG_LEVELS_W1_WPE
#define PQG_LEVELS_W1_WPE 4
#endif
__global__ void __launch_bounds__(64, PQG_LEVELS_W1_WPE) k_page_levels_w1(JobDev* jobs, PageDev* pages, const int* list,
                                                       const int* total, int* queue, uint8_t* scratch,
                                                       HStream* streams, uint8_t* def_arena, uint8_t* rep_arena,
                                                       LongLev* longs, int long_cap, LevPiece* pieces, int piece_cap,
                                                       int split) {
  page_levels<true>(jobs, pages, list, total, queue, scratch, streams, def_arena, rep_arena, longs, long_cap, pieces,
                    piece_cap, split);
}

// ---- K3d ---------------------------------------------------------------------
// notNull prefix per chunk + dictionary-page resolution; one 256-lane block per job.
__device__ void plan_parts(JobDev& job, int np, bool fail, const PageDev* pp, const HStream* streams,
                           const BlockDesc* blks, int* ctr, PartRec* parts, int64_t cap, int64_t* part);

// The job's dictionary page (page_dict.go:30-64): PLAIN entries of the column
// type.  The dictionary is published only when the page's read phase
// succeeds: the gather sinks bound keys by dict_count alone, so a short page
// must never be visible (the reference fails the chunk in readPages first).
// Thread 0 of k_dict_resolve, before the level decode, after the decompression stages (the page's read status is
// final then).
__device__ void resolve_dictionary(JobDev& job, PageDev* pages, uint8_t* scratch) {
  int np = job.num_pages < job.page_cap ? job.num_pages : job.page_cap;
  if (job.status == kCAPACITY) np = 0;
  if (job.dict_page < 0 || job.dict_page >= np) return;
  PageDev& dp = pages[job.page_base + job.dict_page];
  if (dp.read_status != kOK) return;
  const uint8_t* blk =
      dp.scratch_offset >= 0 ? scratch + job.scratch_base + dp.scratch_offset : job.data + dp.payload_offset;
  const int64_t blen = dp.usize;
  const int64_t cnt = dp.num_values;
  const int w = job.value_width;
  dp.block = blk;
  dp.block_len = blen;
  int st = kOK;
  int flags = 0;
  if (w > 0) {
    if (job.type == 3) {  // INT96: a partial final entry is left nil, not an error (Q8)
      const int64_t full = blen / 12, rem = blen % 12;
      if (cnt > full + (rem > 0 ? 1 : 0)) st = kEOF;
      else if (cnt == full + 1 && rem > 0) flags = 1;
    } else if (cnt * w > blen) {
      st = kEOF;
    }
  } else {
    // u32-length entries (type_bytearray.go:24-45): k_str_dict walks them
    // (every entry takes >= 4 bytes: a walk fails before entry blen/4 + 1)
    flags = 2;
    job.need_doffs = (cnt < blen / 4 ? cnt : blen / 4) + 2;
    if (job.need_doffs > job.doffs_cap) job.status = kCAPACITY;
  }
  if (st == kOK) {
    job.flags |= flags;
    job.dict_data = blk;
    job.dict_count = (flags & 2) ? 0 : cnt;  // byte arrays: published by k_str_dict after its walk
    job.dict_len = blen;
  } else {
    dp.read_status = st;
  }
}

__global__ void __launch_bounds__(256) k_dict_resolve(JobDev* jobs, int n_jobs, PageDev* pages, uint8_t* scratch) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j < n_jobs) resolve_dictionary(jobs[j], pages, scratch);
}

// The job's capacity checks (thread 0, after the notNull scan): returns 1
// when the job is out of capacity.
__device__ int nn_job_tail(JobDev& job, PageDev* pages, uint8_t* scratch, int np, int64_t carry, bool fail0) {
  int cap = fail0 || job.status == kCAPACITY;
  job.num_values = carry;
  const int64_t vb = job.value_width > 0 ? carry * job.value_width : 0;
  if (job.value_width > 0 && vb > job.value_cap) job.status = kCAPACITY, cap = 1;
  job.values_bytes = vb;
  return cap;
}

__device__ int64_t part_n(const PageDev& pg, const HStream* streams, int64_t* count, bool* hyb);
__device__ void plan_split_pages(JobDev& job, const PageDev* pp, const HStream* streams, const BlockDesc* blks,
                                 PartRec* parts, int64_t base, int nbig, const int* big, const int64_t* boff);
__device__ void plan_parts_from(JobDev& job, int np, const PageDev* pp, const HStream* streams, const BlockDesc* blks,
                                PartRec* parts, int64_t base);

// Jobs of <= kNnFastSeg x 1024 pages: one read of each page's fields (kept in
// registers), the notNull and part-count scans together, one write pass.
constexpr int kNnFastSeg = 12;

__global__ void __launch_bounds__(1024) k_nn_scan(JobDev* jobs, PageDev* pages, uint8_t* scratch,
                                                  const HStream* streams, const BlockDesc* blks, int* ctr,
                                                  PartRec* parts, int64_t parts_cap) {
  __shared__ int64_t part[17];
  __shared__ int s_cap;
  JobDev& job = jobs[blockIdx.x];
  int np = job.num_pages < job.page_cap ? job.num_pages : job.page_cap;
  if (job.status == kCAPACITY) np = 0;
  if (np <= kNnFastSeg * 1024) {
    __shared__ int64_t s_base, s_res;
    __shared__ int s_big[256];
    __shared__ int64_t s_boff[256];
    __shared__ int s_nbig;
    const int seg = (np + 1023) / 1024;
    const int s0 = (int)threadIdx.x * seg;
    PageDev* pp = pages + job.page_base;
    int32_t nnv[kNnFastSeg], kv[kNnFastSeg];
    int8_t vm[kNnFastSeg];
    int64_t nsum = 0, ksum = 0;
    // the fields first, with unconditional loads (clamped page index: a
    // guarded load would be waited for at its branch join), then the counts
    int32_t f_type[kNnFastSeg], f_nn[kNnFastSeg], f_rs[kNnFastSeg], f_ds[kNnFastSeg], f_enc[kNnFastSeg];
#pragma unroll
    for (int j = 0; j < kNnFastSeg; j++) {
      const int i = np > 0 ? (s0 + j < np ? s0 + j : np - 1) : 0;
      const PageDev& pg = pp[i];
      f_type[j] = pg.page_type;
      f_nn[j] = pg.not_null;
      f_rs[j] = pg.read_status;
      f_ds[j] = pg.decode_status;
      f_enc[j] = pg.encoding;
      vm[j] = (int8_t)pg.vmode;
    }
#pragma unroll
    for (int j = 0; j < kNnFastSeg; j++) {
      nnv[j] = kv[j] = 0;
      if (j < seg && s0 + j < np) {
        const bool data = f_type[j] == 0 || f_type[j] == 3;
        nnv[j] = data ? f_nn[j] : 0;
        // part_n (below) from the fields: big hybrid pages read their stream
        int32_t k = 0;
        if (!data || vm[j] < 0) k = 0;
        else if (f_rs[j] != kOK || f_ds[j] != kOK || vm[j] == 3) k = 1;
        else if (vm[j] == 2 && f_enc[j] != 0 && f_enc[j] != 8) k = 1;
        else if (f_nn[j] <= kSplitMin) k = 1;
        else {
          int64_t c;
          bool h;
          k = (int32_t)part_n(pp[s0 + j], streams, &c, &h);
        }
        kv[j] = k;
      }
      nsum += nnv[j];
      ksum += kv[j];
    }
    int64_t carry, ktot;
    int64_t run = block_excl_scan<1024>(nsum, &carry, part);
    int64_t koff = block_excl_scan<1024>(ksum, &ktot, part);
    const bool fail0 = job.status == kCAPACITY;
    if (threadIdx.x == 0) {
      int cap = nn_job_tail(job, pages, scratch, np, carry, fail0);
      int64_t base = 0;
      if (!cap) {
        base = atomicAdd(ctr + kCtrItems, (int)ktot);
        if (base + ktot > parts_cap) {
          job.status = kCAPACITY;
          cap = 1;
        }
      }
      job.item_base = base;
      job.n_items = cap ? 0 : (int32_t)ktot;
      s_base = base;
      s_cap = cap;
      s_nbig = 0;
      s_res = fail0 ? 0 : ktot;  // reserved slots (even when they do not fit)
      if (blockIdx.x == 0) ctr[kCtrPartsCap] = (int)(parts_cap < INT32_MAX ? parts_cap : INT32_MAX);
    }
    __syncthreads();
    if (s_cap) {  // a reservation past the table: its slots inside the table hold no part
      for (int64_t k = s_base + threadIdx.x; k < s_base + s_res && k < parts_cap; k += 1024) parts[k].vmode = -1;
    }
    // value offsets (always: the later stages read them), then the parts
#pragma unroll
    for (int j = 0; j < kNnFastSeg; j++)
      if (j < seg && s0 + j < np) {
        pp[s0 + j].value_offset = run;
        run += nnv[j];
      }
    if (s_cap) return;
    const int64_t base = s_base;
    bool more = false;
#pragma unroll
    for (int j = 0; j < kNnFastSeg; j++) {
      if (j < seg && s0 + j < np) {
        if (kv[j] == 1) {
          PartRec r;
          r.pidx = (int32_t)(job.page_base + s0 + j);
          r.p = 0;
          r.np = 1;
          r.v0 = 0;
          r.b0 = 0;
          r.vmode = vm[j];
          r.chars = r.cstart = r.prel = 0;
          parts[base + koff] = r;
        } else if (kv[j] > 1) {
          const int slot = atomicAdd(&s_nbig, 1);
          if (slot < 256) {
            s_big[slot] = s0 + j;
            s_boff[slot] = koff;
          } else {
            more = true;
          }
        }
        koff += kv[j];
      }
    }
    const bool any_more = __syncthreads_or(more);
    const int nbig = s_nbig < 256 ? s_nbig : 256;
    if (!any_more) {
      plan_split_pages(job, pp, streams, blks, parts, base, nbig, s_big, s_boff);
      return;
    }
    // more than 256 split pages: the general planner below writes every part again
    __syncthreads();
    plan_parts_from(job, np, pp, streams, blks, parts, base);
    return;
  }
  // each thread takes a contiguous segment of pages: its loads are
  // independent (one round trip per pass, not one per 1024 pages), one block
  // scan of the segment sums, then the offsets are written in a second pass
  const int seg = (np + 1023) / 1024;
  const int s0 = (int)threadIdx.x * seg, s1 = s0 + seg < np ? s0 + seg : np;
  PageDev* pp = pages + job.page_base;
  auto nn_of = [&](int i) -> int64_t {
    const PageDev& pg = pp[i];
    return (pg.page_type == 0 || pg.page_type == 3) ? (int64_t)pg.not_null : 0;
  };
  int64_t sum = 0;
#pragma unroll 8
  for (int i = s0; i < s1; i++) sum += nn_of(i);
  int64_t carry;
  int64_t run = block_excl_scan<1024>(sum, &carry, part);
#pragma unroll 8
  for (int i = s0; i < s1; i++) {
    pp[i].value_offset = run;
    run += nn_of(i);
  }
  const bool fail0 = job.status == kCAPACITY;
  if (threadIdx.x == 0) s_cap = nn_job_tail(job, pages, scratch, np, carry, fail0);
  __syncthreads();
  // values-stage parts (below)
  plan_parts(job, np, s_cap != 0, pp, streams, blks, ctr, parts, parts_cap, part);
}

}  // namespace pqg

namespace pqg {

// ---- values-stage parts -----------------------------------------------------
// Per job (the tail of k_nn_scan's 1024-thread block): every set-up data page
// gets one PartRec, a page of more than kSplitMin values (parquet-go's writer:
// the whole chunk) several (see pqg_common.h); the job's parts are contiguous,
// in page order, from a slot range taken with one atomic.
__device__ __forceinline__ int64_t part_count(const PageDev& pg, const HStream* streams, bool* hyb) {
  *hyb = false;
  if ((pg.page_type != 0 && pg.page_type != 3) || pg.vmode < 0) return -1;  // no part
  if (pg.read_status != kOK || pg.decode_status != kOK || pg.vmode == 3) return 0;  // one part
  const int enc = pg.encoding;
  if (pg.vmode == 2 && enc != 0 && enc != 8) return 0;  // DELTA_(LENGTH_)BYTE_ARRAY: one part
  const int64_t nn = pg.not_null;
  if (enc == 0 || nn <= kSplitMin) return nn;            // PLAIN: value ranges; small pages: one part
  if ((enc == 8 || enc == 3) && pg.hs_val >= 0) {         // hybrid value stream: block ranges
    const HStream& S = streams[pg.hs_val];
    *hyb = true;
    return nn < S.produced ? nn : S.produced;
  }
  return 0;
}

__device__ int64_t part_n(const PageDev& pg, const HStream* streams, int64_t* count, bool* hyb) {
  const int64_t c = part_count(pg, streams, hyb);
  *count = c;
  if (c < 0) return 0;
  return c > kSplitMin ? (c + kPart - 1) / kPart : 1;
}

// The parts of split pages (all threads of the block on each): big[q] is a
// page of the job, boff[q] its first part's slot (relative to base).
__device__ void plan_split_pages(JobDev& job, const PageDev* pp, const HStream* streams, const BlockDesc* blks,
                                 PartRec* parts, int64_t base, int nbig, const int* big, const int64_t* boff) {
  for (int q = 0; q < nbig; q++) {
    const int pi = big[q];
    const int64_t poff = boff[q];
    int64_t cnt;
    bool hyb;
    const PageDev& pg = pp[pi];
    const int64_t P = part_n(pg, streams, &cnt, &hyb);
    PartRec r;
    r.pidx = (int32_t)(job.page_base + pi);
    r.np = (int32_t)P;
    r.vmode = pg.vmode;
    r.chars = r.cstart = r.prel = 0;
    if (!hyb) {
      for (int64_t p = threadIdx.x; p < P; p += blockDim.x) {
        r.p = (int32_t)p;
        r.v0 = (uint32_t)(p * kPart);
        r.b0 = 0;
        parts[base + poff + p] = r;
      }
    } else {
      // part q starts at the first block whose first value is >= q kPart
      // (blocks hold <= kHBlock <= kPart values, so every part but an
      // empty tail one has a block start)
      const HStream& S = streams[pg.hs_val];
      const BlockDesc* B = blks + S.blk_base;
      const int nb = S.n_blocks;
      auto f = [&](int bi) -> int64_t {
        if (bi < 0) return -1;
        if (bi >= nb || (int64_t)B[bi].v0 >= cnt) return P;
        return (int64_t)B[bi].v0 / kPart;
      };
      for (int bi = threadIdx.x; bi <= nb; bi += blockDim.x) {
        const int64_t f1 = f(bi), f0 = f(bi - 1);
        for (int64_t p = f0 + 1; p <= f1 && p < P; p++) {
          r.p = (int32_t)p;
          r.v0 = p == 0 ? 0u : (bi < nb && (int64_t)B[bi].v0 < cnt ? B[bi].v0 : (uint32_t)cnt);
          r.b0 = bi;
          parts[base + poff + p] = r;
        }
      }
    }
  }
}

// Every part of the job's pages from slot `base` on: each thread takes a
// contiguous segment of pages (independent loads), one block scan gives every
// page its first slot; single-part pages are written by their thread, split
// pages go through an LDS list, all 1024 threads on each, in rounds of up to
// kBigList pages.
constexpr int kBigList = 256;
__device__ void plan_parts_from(JobDev& job, int np, const PageDev* pp, const HStream* streams, const BlockDesc* blks,
                                PartRec* parts, int64_t base) {
  __shared__ int64_t part2[17];
  __shared__ int s_big[kBigList];
  __shared__ int64_t s_boff[kBigList];
  __shared__ int s_nbig;
  const int seg = (np + 1023) / 1024;
  const int s0 = (int)threadIdx.x * seg, s1 = s0 + seg < np ? s0 + seg : np;
  int64_t sum = 0;
  for (int i = s0; i < s1; i++) {
    int64_t c;
    bool h;
    sum += part_n(pp[i], streams, &c, &h);
  }
  int64_t tot;
  int64_t off = block_excl_scan<1024>(sum, &tot, part2);
  int cur = s0;
  for (;;) {
    if (threadIdx.x == 0) s_nbig = 0;
    __syncthreads();
    // this thread's pages from its cursor: single parts written, split pages
    // listed (a full list stops the thread at that page, for the next round)
    for (; cur < s1; cur++) {
      int64_t c;
      bool h;
      const int64_t k = part_n(pp[cur], streams, &c, &h);
      if (k == 1) {
        PartRec r;
        r.pidx = (int32_t)(job.page_base + cur);
        r.p = 0;
        r.np = 1;
        r.v0 = 0;
        r.b0 = 0;
        r.vmode = pp[cur].vmode;
        r.chars = r.cstart = r.prel = 0;
        parts[base + off] = r;
      } else if (k > 1) {
        const int slot = atomicAdd(&s_nbig, 1);
        if (slot >= kBigList) break;
        s_big[slot] = cur;
        s_boff[slot] = off;
      }
      off += k;
    }
    __syncthreads();
    plan_split_pages(job, pp, streams, blks, parts, base, s_nbig < kBigList ? s_nbig : kBigList, s_big, s_boff);
    if (!__syncthreads_or(cur < s1)) break;
  }
}

// Called by k_nn_scan's block after its scan (the job's status in `fail`):
// the job's slot range, then its parts.
__device__ void plan_parts(JobDev& job, int np, bool fail, const PageDev* pp, const HStream* streams,
                           const BlockDesc* blks, int* ctr, PartRec* parts, int64_t cap, int64_t* part) {
  __shared__ int64_t s_base;
  __shared__ int s_fail;
  if (fail) np = 0;
  const int seg = (np + 1023) / 1024;
  const int s0 = (int)threadIdx.x * seg, s1 = s0 + seg < np ? s0 + seg : np;
  int64_t sum = 0;
  for (int i = s0; i < s1; i++) {
    int64_t c;
    bool h;
    sum += part_n(pp[i], streams, &c, &h);
  }
  int64_t tot;
  block_excl_scan<1024>(sum, &tot, part);
  if (threadIdx.x == 0) {
    const int64_t base = fail ? 0 : atomicAdd(ctr + kCtrItems, (int)tot);
    s_fail = fail || base + tot > cap;
    if (!fail && s_fail) job.status = kCAPACITY;
    job.item_base = base;
    job.n_items = s_fail ? 0 : (int32_t)tot;
    s_base = base;
    if (blockIdx.x == 0) ctr[kCtrPartsCap] = (int)(cap < INT32_MAX ? cap : INT32_MAX);
  }
  __syncthreads();
  if (s_fail) {  // a reservation past the table: its slots inside the table hold no part
    if (!fail)
      for (int64_t k = s_base + threadIdx.x; k < s_base + tot && k < cap; k += 1024) parts[k].vmode = -1;
    return;
  }
  plan_parts_from(job, np, pp, streams, blks, parts, s_base);
}

}  // namespace pqg
