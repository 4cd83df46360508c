// pqg_hybrid.h — expansion of RLE / bit-packed hybrid run tables (wave level).
//
// k_hybrid_walk (pqg_levels.hip) turns every hybrid stream into a run table
// (RunEnt) and block descriptors (BlockDesc: <= kHBlock values, <= kHBlockRuns
// runs, and the byte range of the bit-packed payload those values use).  An
// expander wave takes a stream one block at a time: the block's runs and
// payload bytes are staged in LDS, then every lane produces 8 consecutive
// values and hands them to a sink (level bytes, dictionary gather, booleans).
//
// The loads of block k+1 are issued before block k's sink runs.  vmcnt
// retires loads and stores in issue order, so a load issued after block k's
// stores would make its wait cover those stores too; issued before them, it
// overlaps with block k's gathers and stores.  The two register sets
// alternate in a 2x unrolled loop, so no in-flight register is copied at the
// loop latch (a copy would force a full vmcnt(0) wait there).
//
// Values are exactly hybridDecoder.next's (hybrid_decoder.go:82-166): RLE runs
// repeat their value; bit-packed runs are LSB-first w-bit fields
// (unpack8int32_w, bitbacking32.go); bytes past the end of the stream read as
// zero (the short-read zero padding, Q5).
#pragma once
#include "pqg_device.h"

namespace pqg {

constexpr int kStageGranules = 192;  // 16-byte payload granules per block (3 per lane)

struct ExpandShared {
  BlockDesc desc[64];
  RunEnt runs[kHBlockRuns];
  uint32_t stage[kStageGranules * 4 + 4];
};

__device__ __forceinline__ uint32_t run_start(const RunEnt& r) { return r.start & ~kRunBP; }

// One block's loads, held in registers between issue and install.
struct BlockRegs {
  uint32_t rs, rv;   // this lane's run entry
  uint4 g0, g1, g2;  // this lane's payload granules (lane, lane+64, lane+128)
};

struct BlockGeom {
  uint32_t v0, v1;  // values [v0, v1)
  uint32_t r0, nr;
  int64_t sb;       // stream offset of stage byte 0 (a 16-byte aligned address)
  int ng;           // granules staged
};

// Block k of the batch in sh.desc[0, nb); `end` bounds the last block.
__device__ __forceinline__ BlockGeom block_geom(const ExpandShared& sh, int k, int nb, uint32_t end,
                                                const HStream& S) {
  BlockGeom g;
  const BlockDesc& d = sh.desc[k];
  g.v0 = d.v0;
  g.v1 = k + 1 < nb ? sh.desc[k + 1].v0 : end;
  if (g.v1 > end) g.v1 = end;
  g.r0 = d.r0;
  g.nr = d.nr;
  const int64_t lo = d.lo;
  g.sb = lo - (int64_t)(((uintptr_t)S.p + (uintptr_t)lo) & 15);
  g.ng = d.nbytes ? (int)((lo + d.nbytes - g.sb + 15) >> 4) + 1 : 0;  // +1: the dword pair read past the end
  if (g.ng > kStageGranules) g.ng = kStageGranules;
  return g;
}

// The prefetch loads are unconditional: a load guarded by a branch is merged
// with the register's old value at the join, and that copy waits (vmcnt) for
// the load at once.  Lanes with nothing to load read a safe mapped address
// (`safe`) and block_process ignores the value.
__device__ __forceinline__ uintptr_t stage_addr(gcu8 sp, int64_t n, int64_t at, bool want, uintptr_t safe) {
  // a granule holding a stream byte < n is mapped
  return (want && at < n && at + 16 > 0) ? (uintptr_t)(sp + at) : safe;
}

__device__ __forceinline__ void block_fetch(BlockRegs& R, const BlockGeom& g, const PQG_G RunEnt* runs, gcu8 sp,
                                            int64_t n, int lane) {
  const uint32_t ri = (uint32_t)lane < g.nr ? (uint32_t)lane : 0u;  // nr >= 1
  R.rs = runs[g.r0 + ri].start;
  R.rv = runs[g.r0 + ri].src;
  const uintptr_t safe = (uintptr_t)(runs + g.r0) & ~(uintptr_t)15;
  R.g0 = ldg16(stage_addr(sp, n, g.sb + 16 * lane, lane < g.ng, safe));
  R.g1 = ldg16(stage_addr(sp, n, g.sb + 16 * (lane + 64), lane + 64 < g.ng, safe));
  R.g2 = ldg16(stage_addr(sp, n, g.sb + 16 * (lane + 128), lane + 128 < g.ng, safe));
}

// zero the bytes of a staged granule at or past the stream end (Q5)
__device__ __forceinline__ uint4 mask_tail(uint4 v, int64_t at, int64_t n) {
  if (at + 16 <= n) return v;
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int d = 0; d < 4; d++) {
    const int64_t b = at + 4 * d;
    if (b >= n) w[d] = 0;
    else if (b + 4 > n) w[d] &= 0xffffffffu >> (8 * (4 - (n - b)));
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

template <class Sink>
__device__ __forceinline__ void block_process(const BlockRegs& R, const BlockGeom& g, ExpandShared& sh,
                                              const HStream& S, uint32_t mask, int w, int lane, Sink& sink) {
  __builtin_amdgcn_wave_barrier();
  if ((uint32_t)lane < g.nr) {
    sh.runs[lane].start = R.rs;
    sh.runs[lane].src = R.rv;
  }
  PQG_L uint32_t* st = lds_ptr(sh.stage);
  if (lane < g.ng) sts16(st + 4 * lane, mask_tail(R.g0, g.sb + 16 * lane, S.n));
  if (lane + 64 < g.ng) sts16(st + 4 * (lane + 64), mask_tail(R.g1, g.sb + 16 * (lane + 64), S.n));
  if (lane + 128 < g.ng) sts16(st + 4 * (lane + 128), mask_tail(R.g2, g.sb + 16 * (lane + 128), S.n));
  __builtin_amdgcn_wave_barrier();
  const uint32_t i0 = g.v0 + lane * 8;
  if (i0 < g.v1) {
    const int cnt = (int)(g.v1 - i0 < 8 ? g.v1 - i0 : 8);
    int lo = 0, hi = (int)g.nr - 1;  // last run with start <= i0
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (run_start(sh.runs[mid]) <= i0) lo = mid; else hi = mid - 1;
    }
    int r = lo;
    RunEnt cur = sh.runs[r];
    uint32_t nxt = r + 1 < (int)g.nr ? run_start(sh.runs[r + 1]) : 0xffffffffu;
    uint32_t v[8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint32_t i = i0 + q;
      v[q] = 0;
      if (q < cnt) {
        while (i >= nxt) {
          r++;
          cur = sh.runs[r];
          nxt = r + 1 < (int)g.nr ? run_start(sh.runs[r + 1]) : 0xffffffffu;
        }
        if (!(cur.start & kRunBP)) {
          v[q] = cur.src;
        } else {
          const int64_t rb = (int64_t)cur.src * 8 + (int64_t)(i - run_start(cur)) * w - g.sb * 8;
          const int d = (int)(rb >> 5);
          const uint32_t lo32 = sh.stage[d], hi32 = sh.stage[d + 1];
          v[q] = __builtin_amdgcn_alignbit(hi32, lo32, (uint32_t)rb & 31) & mask;
        }
      }
    }
    sink.put(i0, v, cnt);
  }
}

// Sink: void put(uint32_t i0, const uint32_t (&v)[8], int cnt)  (cnt <= 8 values from i0)
template <class Sink>
__device__ __forceinline__ void hybrid_expand(const HStream& S, const RunEnt* __restrict__ runs_, const BlockDesc* __restrict__ blks_,
                              int64_t count, ExpandShared& sh, Sink& sink) {
  const int lane = lane_id();
  const int w = S.w;
  const uint32_t mask = w == 32 ? 0xffffffffu : ((1u << w) - 1);
  if (count > S.produced) count = S.produced;
  if (count <= 0) return;
  const uint32_t end_all = (uint32_t)count;
  const gcu8 sp = gconst(S.p);
  const int64_t n = S.n;
  const PQG_G RunEnt* runs = gconst(runs_) + S.run_base;
  const PQG_G BlockDesc* blks = gconst(blks_) + S.blk_base;
  const int nb_all = S.n_blocks;
  for (int b0 = 0; b0 < nb_all; b0 += 64) {
    const int nb = nb_all - b0 < 64 ? nb_all - b0 : 64;
    __builtin_amdgcn_wave_barrier();
    if (lane < nb) {
      const PQG_G BlockDesc& d = blks[b0 + lane];
      sh.desc[lane].v0 = d.v0;
      sh.desc[lane].r0 = d.r0;
      sh.desc[lane].lo = d.lo;
      sh.desc[lane].nbytes = d.nbytes;
      sh.desc[lane].nr = d.nr;
    }
    __builtin_amdgcn_wave_barrier();
    int nk = nb;  // blocks starting at or past `count` are not needed
    while (nk > 0 && sh.desc[nk - 1].v0 >= end_all) nk--;
    if (nk == 0) break;
    // values of the last block here end at the next batch's first block, or at count
    uint32_t tail_end = end_all;
    if (nk == nb && b0 + nb < nb_all) {
      const uint32_t nv0 = blks[b0 + nb].v0;
      tail_end = nv0 < end_all ? nv0 : end_all;
    }
    BlockRegs A, B;
    BlockGeom ga = block_geom(sh, 0, nk, tail_end, S), gb;
    block_fetch(A, ga, runs, sp, n, lane);
    for (int k = 0; k < nk; k += 2) {
      if (k + 1 < nk) {
        gb = block_geom(sh, k + 1, nk, tail_end, S);
        block_fetch(B, gb, runs, sp, n, lane);
      }
      block_process(A, ga, sh, S, mask, w, lane, sink);
      if (k + 1 >= nk) break;
      if (k + 2 < nk) {
        ga = block_geom(sh, k + 2, nk, tail_end, S);
        block_fetch(A, ga, runs, sp, n, lane);
      }
      block_process(B, gb, sh, S, mask, w, lane, sink);
    }
  }
  __builtin_amdgcn_wave_barrier();
}

}  // namespace pqg
