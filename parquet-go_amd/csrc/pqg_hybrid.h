// pqg_hybrid.h — expansion of RLE / bit-packed hybrid run tables (wave level).
//
// k_hybrid_walk (pqg_levels.hip) turns every hybrid stream into a run table
// (RunEnt) and block descriptors (BlockDesc: <= kHBlock values, <= kHBlockRuns
// runs and <= kHBlockBytes bytes of bit-packed payload).  An expander wave
// takes a stream kGroup blocks at a time:
//   1. every lane issues, for each block of the group, the load of one run
//      entry and one 16-byte payload granule (unconditionally: a guarded load
//      is merged with the register's old value at the branch join, and that
//      copy waits for the load on the spot);
//   2. one wait, then the runs and payload are installed in LDS;
//   3. every lane decodes 8 consecutive values of each block (binary search
//      over the block's runs, w-bit fields from the staged payload);
//   4. the sink issues all its loads for the group (dictionary gathers) before
//      any store, then stores.
// So a group of up to kGroup * kHBlock values costs about two memory round
// trips per wave (loads, gathers), instead of several per block: vmcnt retires
// loads and stores in issue order, and each dependent load/wait pair is a
// full round trip.
//
// Values are exactly hybridDecoder.next's (hybrid_decoder.go:82-166): RLE runs
// repeat their value; bit-packed runs are LSB-first w-bit fields
// (unpack8int32_w, bitbacking32.go); bytes past the end of the stream read as
// zero (the short-read zero padding, Q5).
#pragma once
#include "pqg_device.h"

namespace pqg {

#ifndef PQG_KGROUP
#define PQG_KGROUP 2
#endif
constexpr int kGroup = PQG_KGROUP;  // blocks per expander step

struct ExpandShared {
  BlockDesc desc[64];
  RunEnt runs[kGroup][kHBlockRuns];
  uint32_t stage[kGroup][64 * 4 + 4];  // 64 granules (+ the dword past the end)
  uint8_t rmap[kGroup][kHBlock];       // run starting at each value of the block (else 0)
};

__device__ __forceinline__ uint32_t run_start(const RunEnt& r) { return r.start & ~kRunBP; }

struct BlockGeom {
  uint32_t v0, v1;  // values [v0, v1)
  uint32_t r0, nr;
  int64_t sb;       // stream offset of stage byte 0 (a 16-byte aligned address)
  int ng;           // granules staged (<= 64)
};

// Block k of the batch in sh.desc[0, nb); `end` bounds the last block.
__device__ __forceinline__ BlockGeom block_geom(const ExpandShared& sh, int k, int nb, uint32_t end,
                                                uintptr_t p) {
  BlockGeom g;
  const BlockDesc& d = sh.desc[k];
  g.v0 = d.v0;
  g.v1 = k + 1 < nb ? sh.desc[k + 1].v0 : end;
  if (g.v1 > end) g.v1 = end;
  g.r0 = d.r0;
  g.nr = d.nr;
  const int64_t lo = d.lo;
  g.sb = lo - (int64_t)((p + (uintptr_t)lo) & 15);
  g.ng = d.nbytes ? (int)((lo + d.nbytes - g.sb + 15) >> 4) : 0;
  if (g.ng > 64) g.ng = 64;
  return g;
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

// Decode this lane's 8 values of block b (after install): the run of value i
// is the last run starting at or before i.  Runs mark their first value in
// rmap, a wave-wide prefix max turns the marks into a run index per value, so
// no lane walks runs one by one (a divergent, serial LDS chain).
__device__ __forceinline__ void block_values(const ExpandShared& sh, int b, const BlockGeom& g, uint32_t mask, int w,
                                             int lane, uint32_t (&v)[8]) {
  // marks of this lane's 8 values (written before the caller's barrier)
  const u32x2_t mk = *(const PQG_L u32x2_t*)(lds_ptr(sh.rmap[b]) + 8 * lane);
  uint32_t idx[8];
  uint32_t run_max = 0;
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const uint32_t m = ((q < 4 ? mk.x : mk.y) >> (8 * (q & 3))) & 0xff;
    run_max = m > run_max ? m : run_max;
    idx[q] = run_max;
  }
  // exclusive prefix max of the lanes' maxima
  uint32_t incl = run_max;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(incl, o, 64);
    if (lane >= o) incl = t > incl ? t : incl;
  }
  uint32_t before = __shfl_up(incl, 1, 64);
  if (lane == 0) before = 0;
  const int64_t sb8 = g.sb * 8;
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const uint32_t r = idx[q] > before ? idx[q] : before;
    const RunEnt e = sh.runs[b][r];
    const uint32_t i = g.v0 + lane * 8 + q;
    if (!(e.start & kRunBP)) {
      v[q] = e.src;
    } else {
      const uint32_t rb = (uint32_t)((int64_t)e.src * 8 - sb8) + (i - run_start(e)) * (uint32_t)w;
      const uint32_t d = rb >> 5;
      v[q] = __builtin_amdgcn_alignbit(sh.stage[b][d + 1], sh.stage[b][d], rb & 31) & mask;
    }
  }
}

// Block b holds a single run (nr == 1, the common case: runs of <= 512
// values start the blocks): no run marks or scans, the run's fields come in
// scalars (st = its start | kRunBP, src).
__device__ __forceinline__ void block_values_1(const ExpandShared& sh, int b, const BlockGeom& g, uint32_t st,
                                               uint32_t src, uint32_t mask, int w, int lane, uint32_t (&v)[8]) {
  if (!(st & kRunBP)) {
#pragma unroll
    for (int q = 0; q < 8; q++) v[q] = src;
    return;
  }
  const uint32_t rb0 = (uint32_t)((int64_t)src * 8 - g.sb * 8) + (g.v0 + lane * 8 - (st & ~kRunBP)) * (uint32_t)w;
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const uint32_t rb = rb0 + (uint32_t)(q * w);
    const uint32_t d = rb >> 5;
    v[q] = __builtin_amdgcn_alignbit(sh.stage[b][d + 1], sh.stage[b][d], rb & 31) & mask;
  }
}

// Sink:
//   void prepare(v, i0, cnt)  issue the group's loads (dictionary gathers), or nothing
//   void group(v, i0, cnt)    consume them and store
// values v[b][0..cnt[b]) belong at value indices i0[b]...; cnt[b] == 0: none.
// Between the two calls the expander issues the next group's run/payload
// loads, so that (vmcnt retires in issue order) the wait for the gathers
// never includes those loads, the wait for those loads never includes this
// group's stores, and the gather and payload latencies overlap.
// Blocks [blo, bhi) of the stream (a part of a big page, pqg_common.h; the
// whole stream: 0, S.n_blocks), values below `count`.
template <class Sink>
__device__ __forceinline__ void hybrid_expand(const HStream& S, const RunEnt* __restrict__ runs_,
                                              const BlockDesc* __restrict__ blks_, int64_t count, ExpandShared& sh,
                                              Sink& sink, int blo = 0, int bhi = -1) {
  const int lane = lane_id();
  const int w = S.w;
  const uint32_t mask = w == 32 ? 0xffffffffu : ((1u << w) - 1);
  if (count > S.produced) count = S.produced;
  if (count <= 0) return;
  const uint32_t end_all = (uint32_t)count;
  const gcu8 sp = gconst(S.p);
  const uintptr_t pa = (uintptr_t)S.p;
  const int64_t n = S.n;
  const PQG_G RunEnt* runs = gconst(runs_) + S.run_base;
  const PQG_G BlockDesc* blks = gconst(blks_) + S.blk_base;
  const int nb_all = bhi < 0 || bhi > S.n_blocks ? S.n_blocks : bhi;
  for (int b0 = blo; b0 < nb_all; b0 += 64) {
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
    // the last block here ends at the next batch's first block, or at count
    uint32_t tail_end = end_all;
    if (nk == nb && b0 + nb < S.n_blocks) {
      const uint32_t nv0 = blks[b0 + nb].v0;
      tail_end = nv0 < end_all ? nv0 : end_all;
    }
    // every lane issues, for each block of group k0, the load of one run entry
    // and one 16-byte payload granule (unconditionally: a guarded load is
    // merged with the register's old value at the branch join, and that copy
    // waits for the load on the spot)
    uint32_t rs[kGroup], rv[kGroup];
    uint4 gr[kGroup];
    auto issue = [&](int k0) {
#pragma unroll
      for (int b = 0; b < kGroup; b++) {
        const int k = k0 + b < nk ? k0 + b : nk - 1;  // past the end: repeat the last block, unused
        const BlockGeom g = block_geom(sh, k, nk, tail_end, pa);
        const uint32_t ri = (uint32_t)lane < g.nr ? (uint32_t)lane : 0u;  // nr >= 1
        rs[b] = runs[g.r0 + ri].start;
        rv[b] = runs[g.r0 + ri].src;
        // granule `lane`, if it holds a stream byte < n (mapped); else a safe address
        const int64_t at = g.sb + 16 * lane;
        const bool want = lane < g.ng && at < n;
        gr[b] = ldg16(want ? (uintptr_t)(sp + at) : ((uintptr_t)(runs + g.r0) & ~(uintptr_t)15));
      }
    };
    issue(0);
    for (int k0 = 0; k0 < nk; k0 += kGroup) {
      PQG_T(t0);
      BlockGeom g[kGroup];
#pragma unroll
      for (int b = 0; b < kGroup; b++) g[b] = block_geom(sh, k0 + b < nk ? k0 + b : nk - 1, nk, tail_end, pa);
      PQG_T(t1);
      PQG_ACC(0, t0, t1);
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int b = 0; b < kGroup; b++) {
        if (g[b].nr > 1) *(PQG_L u32x2_t*)(lds_ptr(sh.rmap[b]) + 8 * lane) = u32x2_t{0u, 0u};
        if ((uint32_t)lane < g[b].nr) {
          sh.runs[b][lane].start = rs[b];
          sh.runs[b][lane].src = rv[b];
        }
        if (lane < g[b].ng) sts16(lds_ptr(sh.stage[b]) + 4 * lane, mask_tail(gr[b], g[b].sb + 16 * lane, n));
      }
      __builtin_amdgcn_wave_barrier();
      uint32_t s0[kGroup], src0[kGroup];
#pragma unroll
      for (int b = 0; b < kGroup; b++) {
        // run r > 0 starts inside the block (run 0 holds value v0)
        if (lane > 0 && (uint32_t)lane < g[b].nr) sh.rmap[b][(rs[b] & ~kRunBP) - g[b].v0] = (uint8_t)lane;
        s0[b] = (uint32_t)__builtin_amdgcn_readfirstlane(rs[b]);
        src0[b] = (uint32_t)__builtin_amdgcn_readfirstlane(rv[b]);
      }
      __builtin_amdgcn_wave_barrier();
      PQG_T(t2);
      PQG_ACC(1, t1, t2);
      uint32_t v[kGroup][8], i0[kGroup];
      int cnt[kGroup];
#pragma unroll
      for (int b = 0; b < kGroup; b++) {
        i0[b] = g[b].v0 + lane * 8;
        cnt[b] = (k0 + b < nk && i0[b] < g[b].v1) ? (int)(g[b].v1 - i0[b] < 8 ? g[b].v1 - i0[b] : 8) : 0;
        if (g[b].nr == 1)
          block_values_1(sh, b, g[b], s0[b], src0[b], mask, w, lane, v[b]);
        else
          block_values(sh, b, g[b], mask, w, lane, v[b]);
      }
      PQG_T(t3);
      PQG_ACC(2, t2, t3);
      sink.prepare(v, i0, cnt);
      if (k0 + kGroup < nk) issue(k0 + kGroup);  // the next group's loads, under the gathers
      sink.group(v, i0, cnt);
      PQG_T(t4);
      PQG_ACC(3, t3, t4);
#ifdef PQG_PROFILE
      if (lane == 0) atomicAdd(&pqg_prof[4], 1ull);
#endif
    }
  }
  __builtin_amdgcn_wave_barrier();
}

}  // namespace pqg
