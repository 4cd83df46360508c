// pqg_hybrid.h — expansion of RLE / bit-packed hybrid run tables (wave level).
//
// k_hybrid_walk (pqg_levels.hip) turns every hybrid stream into a run table
// (RunEnt) plus a block index (run holding value k*kHBlock).  An expander
// wave takes a stream one block of kHBlock values at a time: the block's runs
// and the bit-packed payload bytes they cover are staged in LDS, then every
// lane produces 8 consecutive values and hands them to a sink (level bytes,
// dictionary gather, booleans).  Values are exactly hybridDecoder.next's
// (hybrid_decoder.go:82-166): RLE runs repeat their value, bit-packed runs
// are LSB-first w-bit fields (unpack8int32_w, bitbacking32.go), bytes past
// the end of the stream read as zero (the short-read zero padding, Q5).
#pragma once
#include "pqg_device.h"

namespace pqg {

constexpr int kStageBytes = 4096;  // staged payload bytes per block

struct ExpandShared {
  RunEnt runs[kHBlock + 2];
  uint32_t stage[kStageBytes / 4 + 2];
};

__device__ __forceinline__ uint32_t run_start(const RunEnt& r) { return r.start & ~kRunBP; }

// Global-memory fallback: w bits at stream bit `bit`, zero past n.
__device__ __forceinline__ uint32_t extract_global(const uint8_t* p, int64_t n, int64_t bit, int w) {
  int64_t byte = bit >> 3;
  uint64_t x = 0;
  for (int k = 0; k < 5; k++) {
    int64_t j = byte + k;
    if (j < n) x |= (uint64_t)p[j] << (8 * k);
  }
  x >>= (bit & 7);
  return (uint32_t)(x & (w == 32 ? 0xffffffffull : ((1ull << w) - 1)));
}

// Sink: void put(int64_t i0, const uint32_t (&v)[8], int cnt)  (cnt <= 8 values from i0)
template <class Sink>
__device__ void hybrid_expand(const HStream& S, const RunEnt* __restrict__ runs, const int32_t* __restrict__ blks,
                              int64_t count, ExpandShared& sh, Sink& sink) {
  const int lane = lane_id();
  const int w = S.w;
  const uint32_t mask = w == 32 ? 0xffffffffu : ((1u << w) - 1);
  if (count > S.produced) count = S.produced;
  const int64_t nblk = (count + kHBlock - 1) / kHBlock;
  const RunEnt* R = runs + S.run_base;
  for (int64_t k = 0; k < nblk; k++) {
    const int64_t v0 = k * kHBlock;
    const int64_t v1 = v0 + kHBlock < count ? v0 + kHBlock : count;
    const int r0 = blks[S.blk_base + k];
    const int r1 = (k + 1 < nblk) ? blks[S.blk_base + k + 1] : S.n_runs - 1;
    const int nr = r1 - r0 + 1;  // <= kHBlock + 1
    // runs [r0, r1] plus the entry after r1 (its start ends run r1)
    for (int i = lane; i <= nr; i += 64) {
      RunEnt e;
      if (r0 + i < S.n_runs) e = R[r0 + i];
      else { e.start = (uint32_t)S.produced; e.src = 0; }
      sh.runs[i] = e;
    }
    __builtin_amdgcn_wave_barrier();
    // payload bytes of the block's bit-packed values
    int64_t lo = INT64_MAX, hi = -1;
    for (int i = lane; i < nr; i += 64) {
      const RunEnt e = sh.runs[i];
      if (!(e.start & kRunBP)) continue;
      const int64_t s0 = run_start(e), s1 = run_start(sh.runs[i + 1]);
      const int64_t f = s0 > v0 ? s0 : v0, l = s1 < v1 ? s1 : v1;
      if (f >= l) continue;
      const int64_t b0 = (int64_t)e.src * 8 + (f - s0) * w, b1 = (int64_t)e.src * 8 + (l - s0) * w;
      lo = b0 >> 3 < lo ? b0 >> 3 : lo;
      hi = (b1 + 7) >> 3 > hi ? (b1 + 7) >> 3 : hi;
    }
    lo = wave_min(lo);
    hi = -wave_min(-hi);
    // staged from the 4-aligned address at or below byte lo: stream byte sb
    // (sb may be up to 3 bytes before the stream; those bytes are never used)
    const int64_t sb = lo - (int64_t)(((uintptr_t)S.p + (uintptr_t)lo) & 3);
    const bool staged = hi > lo && hi - sb <= kStageBytes;
    if (staged) {
      const int nd = (int)((hi - sb + 3) >> 2) + 1;
      for (int d = lane; d < nd; d += 64) {
        const int64_t b = sb + 4 * (int64_t)d;
        uint32_t x = 0;
        // a dword holding a byte < n is mapped; bytes at or past n read as 0 (Q5)
        if (b + 4 <= S.n) x = *(const uint32_t*)(S.p + b);
        else if (b < S.n) x = *(const uint32_t*)(S.p + b) & (0xffffffffu >> (8 * (4 - (S.n - b))));
        sh.stage[d] = x;
      }
    }
    __builtin_amdgcn_wave_barrier();
    // 8 consecutive values per lane
    const int64_t i0 = v0 + lane * 8;
    if (i0 < v1) {
      const int cnt = (int)(v1 - i0 < 8 ? v1 - i0 : 8);
      int lo2 = 0, hi2 = nr - 1;  // last run with start <= i0
      while (lo2 < hi2) {
        const int mid = (lo2 + hi2 + 1) >> 1;
        if ((int64_t)run_start(sh.runs[mid]) <= i0) lo2 = mid; else hi2 = mid - 1;
      }
      int r = lo2;
      RunEnt cur = sh.runs[r];
      int64_t nxt = run_start(sh.runs[r + 1]);
      uint32_t v[8];
#pragma unroll
      for (int q = 0; q < 8; q++) {
        const int64_t i = i0 + q;
        v[q] = 0;
        if (q < cnt) {
          while (i >= nxt && r + 1 < nr) {
            r++;
            cur = sh.runs[r];
            nxt = run_start(sh.runs[r + 1]);
          }
          if (!(cur.start & kRunBP)) {
            v[q] = cur.src;
          } else {
            const int64_t bit = (int64_t)cur.src * 8 + (i - run_start(cur)) * w;
            if (staged) {
              const int64_t rb = bit - sb * 8;
              const int d = (int)(rb >> 5);
              const uint64_t x = (uint64_t)sh.stage[d] | ((uint64_t)sh.stage[d + 1] << 32);
              v[q] = (uint32_t)(x >> (rb & 31)) & mask;
            } else {
              v[q] = extract_global(S.p, S.n, bit, w);
            }
          }
        }
      }
      sink.put(i0, v, cnt);
    }
    __builtin_amdgcn_wave_barrier();
  }
}

}  // namespace pqg
