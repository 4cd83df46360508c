// pqg_idxwalk.h — the in-kernel, wave-parallel walk of a dictionary page's
// index stream (IdxWalk) and its dictionary sinks, shared by the dictionary
// kernels (pqg_dict.hip) and the fused level + dictionary page kernel
// (pqg_fused.hip).
#pragma once
#include "pqg_common.h"
#include "pqg_device.h"
#include "pqg_hybrid.h"

namespace pqg {

// PageDev.flags: the page's values were decoded by k_page_fused (pqg_fused.hip);
// k_dict_plan gives it no work item.  Reported as PQG_PAGE_FLAG_FUSED.
constexpr int32_t kPageFused = 1 << 5;

// In-kernel walk of a small page's index stream (no run tables, see
// IdxWalk below): a ring window over the stream, the run marks / run index
// of a batch's values, the batch's run entries and the chain flags.
constexpr int kIWin = 4096;   // ring bytes; stream byte at absolute address a sits at (a & (kIWin - 1))
constexpr int kINeed = 3072;  // window bytes a step wants at and after its first header (the ring streams
                              // in 1 KiB quarters: a quarter is replaced once the step has left it)
constexpr int kIPos = 64;     // header positions parsed per step (one per lane)
constexpr int kISpan = 512;   // values per batch (8 per lane)
struct WalkShared {
  uint32_t win[kIWin / 4 + 4];  // + a copy of the ring's first granule: reads of dwords d, d + 1 (d < kIWin / 4) never wrap
  uint8_t tm[kISpan];   // 1 + run position at each run's first value; then the run of every value
  u32x2_t te[kIPos];    // per run position: {first value | bit 31 bit-packed, BP: payload bit in the ring; RLE: value}
  uint8_t cflag[kIPos];
};
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

// kPipe: a global dictionary's gathers are pipelined with the previous
// batch's stores (k_dict_walk_g); k_page_fused stores each batch at once
// (fewer registers: other waves hide the latency there).
template <class Dict, bool kPipe = Dict::kGlobal>
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
      if (o == 0) sts16(lds_ptr(sh->win) + kIWin / 4, x);  // the mirror
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
      if (o == 0) sts16(lds_ptr(sh->win) + kIWin / 4, x);  // the mirror
      __builtin_amdgcn_wave_barrier();
      wlo += 1024;
      whi += 1024;
      prefetch(whi);
    }
  }
  // bytes [q, q + 8) of the ring as two dwords
  __device__ __forceinline__ void rd8(uint32_t q, uint32_t& lo, uint32_t& hi) const {
    constexpr uint32_t M = kIWin / 4 - 1;
    const PQG_L uint32_t* W = lds_ptr(sh->win) + (((wb + q) >> 2) & M);  // dwords 0..2 from here: the mirror covers a wrap
    const uint32_t s = ((wb + q) & 3) * 8;
    const uint32_t a = W[0], b = W[1], c = W[2];
    lo = __builtin_amdgcn_alignbit(b, a, s);
    hi = __builtin_amdgcn_alignbit(c, b, s);
  }
  // w bits at ring bit `bit` (wraps)
  __device__ __forceinline__ uint32_t bits_at(uint32_t bit) const {
    constexpr uint32_t M = kIWin / 4 - 1;
    const PQG_L uint32_t* W = lds_ptr(sh->win) + ((bit >> 5) & M);
    return __builtin_amdgcn_alignbit(W[1], W[0], bit & 31) & vmask();
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
    if (kPipe && ptot) store8(pv, pbase, ptot);
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
    if (kPipe) {
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
      const uint32_t st = cm == 1 ? 0u : dpp_incl_add_sat(c) - c;  // values before the run (chain runs)
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

}  // namespace pqg
