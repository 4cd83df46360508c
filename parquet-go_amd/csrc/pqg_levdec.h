// pqg_levdec.h — the wave-parallel RLE / bit-packed level decoder
// (LevelDecoder) and the read phase of a data page (page_setup), used by
// k_page_levels and k_page_levels_w1 (pqg_levels.hip).
#pragma once
#include "pqg_common.h"
#include "pqg_device.h"
#include "pqg_hybrid.h"

namespace pqg {

// ---- K3a ---------------------------------------------------------------------
// The stream's run table / block index go to the page's region (k_page_list:
// every run but a truncated last one takes >= 2 bytes; blocks close at
// kHBlock values, kHBlockRuns runs or kHBlockBytes payload bytes).
__device__ __forceinline__ int reg_stream(const JobDev& job, const PageDev& pg, HStream* streams, int32_t* slot,
                                          int pidx, int kind, gcu8 p, int64_t n, int w, int64_t count) {
  const int64_t rb = pg.run_off, bb = pg.blk_off;
  const int id = pidx * 3 + (kind > 2 ? 2 : kind);
  HStream& S = streams[id];
  S.p = (const uint8_t*)p;
  S.n = n;
  S.run_base = job.run_base + rb;
  S.blk_base = job.blk_base + bb;
  S.page = pidx;
  S.kind = kind;
  S.w = w;
  S.count = (int32_t)count;
  S.n_runs = 0;
  S.produced = 0;
  S.status = kOK;
  S.n_blocks = 0;
  *slot = id;
  return id;
}

// ---- K3 fused: setup + level decode, one wave per data page -----------------
//
// The level streams (def/rep: bit widths 1..8) are run-dense (a run per ~10
// slots at 10% nulls), so they are decoded where they are read, without run
// tables: per window of 128 stream bytes (LDS),
//   1. each lane parses a run header speculatively at two positions (lane,
//      64 + lane): uvarint header, RLE value or bit-packed extent, errors;
//   2. a scalar loop follows the true chain with v_readlane (a few cycles per
//      run) and marks it;
//   3. a DPP prefix sum gives each run its first value index; the runs up to
//      the page's count (and <= kLSpan values, payload inside the window)
//      form the batch; errors are checked lane-parallel, in stream order;
//   4. each lane expands 16 consecutive values (its 16-byte output granule):
//      its run by a prefix max over run marks, RLE -> the run value,
//      bit-packed -> w bits of the staged payload; full granules are stored
//      with one dwordx4, the batch's ragged ends byte by byte; notNull counts
//      values == maxD.
// A run longer than one batch (long RLE, wide bit-packed) goes in pieces.
// Semantics are hybridDecoder.next (hybrid_decoder.go:82-166), exactly as the
// walker: header EOF/overflow (> MaxInt32), empty runs, RLE value > w bits,
// short bit-packed reads (the last needed group must start inside the
// stream; bytes past it read as zero, Q5).
constexpr int kLWin = 2048;   // stream window (LDS)
constexpr int kLNeed = 1280;  // window bytes wanted at a batch's first run (headers + <= 1 KiB payload)
constexpr int kLSpan = 1024;  // values per batch: 64 lanes x 16
constexpr int kLPos = 128;    // header positions parsed per window

struct LevShared {
  uint8_t win[kLWin + 16];
  uint32_t bm[kLSpan / 32 + 1];  // w == 1: the batch's values as a bitmap (bit j: value j from the granule base)
  uint8_t tmap[kLSpan];  // 1 + run position at the run's first value (relative to the batch's granule base)
  u32x2_t tent[kLPos];   // {first value (relative), BP: 0x80000000 | payload bit offset in the window; RLE: value}
  uint8_t cflag[kLPos];  // chain marks of the pointer-doubling walk
};

__device__ __forceinline__ uint32_t ldpp_incl_add_sat(uint32_t x) {
  // saturating 64-lane inclusive sum (row_shr 1/2/4/8, row_bcast 15/31)
  uint32_t t;
#define PQG_SAT_STEP(ctrl, rm, bc)                                                   \
  t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, ctrl, rm, 0xf, bc);           \
  x = x + t < x ? 0xffffffffu : x + t;
  PQG_SAT_STEP(0x111, 0xf, true) PQG_SAT_STEP(0x112, 0xf, true) PQG_SAT_STEP(0x114, 0xf, true)
  PQG_SAT_STEP(0x118, 0xf, true) PQG_SAT_STEP(0x142, 0xa, false) PQG_SAT_STEP(0x143, 0xc, false)
#undef PQG_SAT_STEP
  return x;
}
__device__ __forceinline__ uint32_t ldpp_incl_max(uint32_t x) {
  uint32_t t;
#define PQG_MAX_STEP(ctrl, rm, bc)                                                   \
  t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, ctrl, rm, 0xf, bc);           \
  x = t > x ? t : x;
  PQG_MAX_STEP(0x111, 0xf, true) PQG_MAX_STEP(0x112, 0xf, true) PQG_MAX_STEP(0x114, 0xf, true)
  PQG_MAX_STEP(0x118, 0xf, true) PQG_MAX_STEP(0x142, 0xa, false) PQG_MAX_STEP(0x143, 0xc, false)
#undef PQG_MAX_STEP
  return x;
}

// One speculative run header at stream position q (window bytes, zero past n).
struct LRun {
  uint32_t cnt;   // values the header declares (saturated)
  uint32_t next;  // stream position of the next header (saturated)
  uint32_t pay;   // BP: stream position of the payload; RLE: the value
  int err;        // read error of the header / RLE value (kOK: none)
  bool bp;
  bool cplx;      // header longer than 4 bytes: resolved serially
};

__device__ __forceinline__ LRun parse_lrun(const PQG_L uint8_t* win, uint32_t wo, uint32_t q, uint32_t n, int w) {
  const PQG_L uint32_t* d = (const PQG_L uint32_t*)(win + (wo & ~3u));
  const uint32_t a = d[0], b = d[1], c = d[2];
  const uint32_t sft = (wo & 3) * 8;
  const uint32_t lo = __builtin_amdgcn_alignbit(b, a, sft), hi = __builtin_amdgcn_alignbit(c, b, sft);
  LRun r;
  r.err = kOK;
  r.cplx = false;
  // readUVariant32 (helpers.go:149-165 via binary.ReadUvarint), 32-bit fast
  // path for headers of <= 4 bytes (< 2^28: no MaxInt32 overflow); longer
  // ones are walked serially.  Bytes past n read as zero (window fill), so a
  // header running past the stream end terminates at or past n: EOF.
  const uint32_t cont = ~lo & 0x80808080u;  // bytes without the continuation bit
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
    const uint32_t vp = q + hl;  // rb = 1 byte for w <= 8
    if (r.err == kOK && !r.cplx && vp >= n) r.err = kEOF;
    r.pay = (hl < 4 ? (lo >> (8 * hl)) : hi) & 0xff;
    if (r.err == kOK && !r.cplx && (r.pay >> w) != 0) r.err = kRLE;  // readRLERunValue :127-129
    r.next = vp + 1;
  }
  return r;
}

// The exact header walk for one position (5+ byte varints): err, h, header length.
__device__ int lrun_serial(const PQG_L uint8_t* win, uint32_t wo, uint32_t q, uint32_t n, uint32_t* h_out,
                           uint32_t* hl_out) {
  uint64_t v = 0;
  unsigned sft = 0;
  for (uint32_t i = 0;; i++) {
    if (q + i >= n) return kEOF;
    const uint32_t b = win[wo + i];
    if (b < 0x80) {
      if (i > 9 || (i == 9 && b > 1)) return kRLE;  // overflows uint64
      v |= sft < 64 ? (uint64_t)b << sft : 0;
      if (v > 0x7fffffffull) return kRLE;
      *h_out = (uint32_t)v;
      *hl_out = i + 1;
      return kOK;
    }
    if (sft < 64) v |= (uint64_t)(b & 0x7f) << sft;
    sft += 7;
  }
}

// kW1: a decoder for bit width 1 only (maxLevel 1: optional flat columns, the
// C2 shape); the w > 1 expansion is not compiled in, so the kernel that uses
// it needs fewer registers and runs more waves per SIMD.
template <bool kW1>
struct LevelDecoderT {
  gcu8 p;
  uint32_t n;      // stream bytes
  int w;           // bit width (1..8; 1 when kW1)
  uint32_t count;  // values wanted
  gu8 out;         // count bytes
  uint32_t maxl;
  LevShared* sh;
  // long runs (> kLongLev values) go to k_level_long (null: expanded here)
  LongLev* longs;
  LevPiece* pieces;
  int* ctr;
  int long_cap, piece_cap, pidx;
  uint32_t wbase = 0;  // stream offset of win[0] (16-aligned in memory, may precede the stream)
  bool have = false;
  bool deferred = false;  // a long run went to k_level_long: nn is not complete yet
  uint32_t nn = 0;     // per lane: values == maxl
#ifdef PQG_PROFILE
  uint64_t pacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // per-wave phase cycles / counts (one atomic per stream)
#define PQG_LT(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define PQG_LA(k, x) pacc[k] += (x)
#else
#define PQG_LT(v)
#define PQG_LA(k, x)
#endif

  __device__ void fill(uint32_t at) {
    const int lane = lane_id();
    const uint32_t mis = (uint32_t)((uintptr_t)(p + at) & 15);
    wbase = at - mis;  // wraps below 0 for the first window of a misaligned stream: offsets are modular
    have = true;
    uint4 v[kLWin / 1024];
    // granules holding a stream byte are mapped; bytes past n read as zero
    // (Q5).  Every load is unconditional (a granule holding no stream byte
    // reads the first one and is zeroed after all are issued: a load under a
    // branch is waited for inside it).
#pragma unroll
    for (int h = 0; h < kLWin / 1024; h++) {
      const int64_t g = (int64_t)at - mis + 1024 * h + 16 * lane;
      v[h] = ldg16((g < (int64_t)n && g + 16 > 0) ? (uintptr_t)(p + g) : ((uintptr_t)p & ~(uintptr_t)15));
    }
#pragma unroll
    for (int h = 0; h < kLWin / 1024; h++) {
      const int64_t g = (int64_t)at - mis + 1024 * h + 16 * lane;
      v[h] = (g < (int64_t)n && g + 16 > 0) ? mask_tail(v[h], g, n) : make_uint4(0, 0, 0, 0);
      if (g < 0 && g + 16 > 0) {  // bytes before the stream start: zero too (never read as data)
        uint32_t ww[4] = {v[h].x, v[h].y, v[h].z, v[h].w};
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int64_t b = g + 4 * k;
          if (b + 4 <= 0) ww[k] = 0;
          else if (b < 0) ww[k] &= 0xffffffffu << (8 * (int)(-b));
        }
        v[h] = make_uint4(ww[0], ww[1], ww[2], ww[3]);
      }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int h = 0; h < kLWin / 1024; h++) sts16(lds_ptr(sh->win) + 1024 * h + 16 * lane, v[h]);
    __builtin_amdgcn_wave_barrier();
  }
  __device__ __forceinline__ bool in_win(uint32_t a, uint32_t len) const {
    return have && a - wbase <= (uint32_t)kLWin && a - wbase + len <= (uint32_t)kLWin;
  }

  // Expand values [v0, v0 + cnt) of the page (cnt <= kLSpan - pre), given the
  // run tables; stores the granules and counts notNull.
  __device__ void expand(uint32_t v0, uint32_t cnt) {
    const int lane = lane_id();
    const uintptr_t oa = (uintptr_t)(out + v0);
    const uintptr_t a0 = oa & ~(uintptr_t)15;
    const int pre = (int)(oa - a0);
    const int end = pre + (int)cnt;
    const u32x4_t mk = *(const PQG_L u32x4_t*)(lds_ptr(sh->tmap) + 16 * lane);
    const uint32_t mw[4] = {mk.x, mk.y, mk.z, mk.w};
    uint32_t tix[16];
    uint32_t run_max = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint32_t m = (mw[k >> 2] >> (8 * (k & 3))) & 0xff;
      run_max = m > run_max ? m : run_max;
      tix[k] = run_max;
    }
    uint32_t before = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ldpp_incl_max(run_max), 0x138, 0xf, 0xf, false);
    const PQG_L u32x2_t* TE = lds_ptr(sh->tent);
    const PQG_L uint8_t* W = lds_ptr(sh->win);
    const uint32_t mask = (1u << w) - 1;
    uint32_t val[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint32_t t = (tix[k] > before ? tix[k] : before);
      const u32x2_t te = TE[(t - 1) & (kLPos - 1)];  // t >= 1 for every value of the batch
      const uint32_t rel = (uint32_t)(16 * lane + k) - te.x;
      const bool bp = (te.y & 0x80000000u) != 0;
      const uint32_t bit = bp ? (te.y & 0x7fffffffu) + rel * (uint32_t)w : 0u;
      const PQG_L uint32_t* dw = (const PQG_L uint32_t*)(W + ((bit >> 3) & ~3u));
      const uint32_t lo = dw[0], hi = dw[1];
      const uint32_t bits = __builtin_amdgcn_alignbit(hi, lo, bit & 31) & mask;
      val[k] = bp ? bits : te.y;
    }
    uint32_t wv[4];
#pragma unroll
    for (int k = 0; k < 4; k++) wv[k] = val[4 * k] | val[4 * k + 1] << 8 | val[4 * k + 2] << 16 | val[4 * k + 3] << 24;
    const int i0 = 16 * lane;
    if (i0 >= pre && i0 + 16 <= end) {
      stg16o(a0 + i0, make_uint4(wv[0], wv[1], wv[2], wv[3]));
#pragma unroll
      for (int k = 0; k < 16; k++) nn += val[k] == maxl;
    } else if (i0 + 16 > pre && i0 < end) {
#pragma unroll
      for (int k = 0; k < 16; k++) {
        if (i0 + k >= pre && i0 + k < end) {
          *(PQG_G uint8_t*)(a0 + i0 + k) = (uint8_t)val[k];
          nn += val[k] == maxl;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }

  // ---- w == 1 (maxLevel 1, the common optional / single-list case): values
  // are bits.  Each run ORs its bits into an LDS bitmap, one dword at a time
  // (RLE: ones or nothing; bit-packed: 32 payload bits via alignbit); each
  // lane then spreads its 16 bits into 16 level bytes (nibble x 0x00204081)
  // and counts notNull with one popcount.
  __device__ __forceinline__ void bits_or(uint32_t st, uint32_t len, bool bp, uint32_t info, uint32_t k) {
    const uint32_t lo = st > 32 * k ? st : 32 * k;
    const uint32_t e = st + len, hi = e < 32 * k + 32 ? e : 32 * k + 32;
    if (lo >= hi) return;
    const uint32_t cnt = hi - lo;
    const uint32_t m = cnt >= 32 ? 0xffffffffu : ((1u << cnt) - 1);
    uint32_t v;
    if (bp) {
      const uint32_t sb = info + (lo - st);  // payload bit in the window
      const PQG_L uint32_t* W = (const PQG_L uint32_t*)lds_ptr(sh->win);
      v = __builtin_amdgcn_alignbit(W[(sb >> 5) + 1], W[sb >> 5], sb & 31) & m;
    } else {
      v = info ? m : 0u;
    }
    v <<= (lo - 32 * k);
    if (v) __hip_atomic_fetch_or(&sh->bm[k], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  }
  __device__ __forceinline__ void bits_clear() {
    const int lane = lane_id();
    if (lane <= kLSpan / 32) lds_ptr(sh->bm)[lane] = 0u;
    __builtin_amdgcn_wave_barrier();
  }
  // store values [v0, v0 + cnt) from the bitmap (granule base = out + v0 rounded down to 16)
  __device__ void bits_store(uint32_t v0, uint32_t cnt) {
    const int lane = lane_id();
    __builtin_amdgcn_wave_barrier();
    const uintptr_t oa = (uintptr_t)(out + v0);
    const uintptr_t a0 = oa & ~(uintptr_t)15;
    const int pre = (int)(oa - a0);
    const int end = pre + (int)cnt;
    const uint32_t b16 = (lds_ptr(sh->bm)[lane >> 1] >> ((lane & 1) * 16)) & 0xffffu;
    uint32_t wv[4];
#pragma unroll
    for (int g = 0; g < 4; g++) wv[g] = (((b16 >> (4 * g)) & 0xfu) * 0x00204081u) & 0x01010101u;
    const int i0 = 16 * lane;
#ifdef PQG_NOSTORE_EXPERIMENT
    constexpr bool kStore = false;
#else
    constexpr bool kStore = true;
#endif
    if (i0 >= pre && i0 + 16 <= end) {
      if (kStore) stg16o(a0 + i0, make_uint4(wv[0], wv[1], wv[2], wv[3]));
      if (maxl == 1) nn += __builtin_popcount(b16);
    } else if (i0 + 16 > pre && i0 < end) {
      uint32_t vm = 0;
#pragma unroll
      for (int k = 0; k < 16; k++) {
        if (i0 + k >= pre && i0 + k < end) {
          if (kStore) *(PQG_G uint8_t*)(a0 + i0 + k) = (uint8_t)((b16 >> k) & 1);
          vm |= 1u << k;
        }
      }
      if (maxl == 1) nn += __builtin_popcount(b16 & vm);
    }
    __builtin_amdgcn_wave_barrier();
  }

  // decode `count` values; kOK or the stream's first error
  __device__ int run() {
    const int lane = lane_id();
    uint32_t pos = 0, produced = 0;
    const uintptr_t oa0 = (uintptr_t)out;
    while (produced < count) {
      if (pos >= n) return kEOF;
      PQG_LT(ta);
      if (!in_win(pos, kLNeed)) {
        fill(pos);
        PQG_LA(6, 1);
      }
      PQG_LT(tb);
      PQG_LA(0, tb - ta);
      const uint32_t wo = pos - wbase;
      const uint32_t pre = (uint32_t)((oa0 + produced) & 15);
      const uint32_t left = count - produced;
      // ---- 1. speculative headers
      const LRun r0 = parse_lrun(lds_ptr(sh->win), wo + lane, pos + lane, n, w);
      const LRun r1 = parse_lrun(lds_ptr(sh->win), wo + 64 + lane, pos + 64 + lane, n, w);
      auto nxt = [&](const LRun& r, uint32_t rel) -> int {
        if (r.err != kOK || r.cplx) return kLPos;
        const uint32_t d = r.next - pos;  // > rel
        return d < (uint32_t)kLPos ? (int)d : kLPos;
      };
      const int n0 = nxt(r0, lane), n1 = nxt(r1, 64 + lane);
      // ---- 2. the chain
      // (two tight loops, one per half: a bit set, a readlane and a compare
      // per run, so the CU's shared scalar unit is not the bottleneck)
      uint64_t cm0 = 0, cm1 = 0;
#ifdef PQG_LEV_SERIAL_CHAIN
      int pp = 0;
      while (pp < 64) {
        cm0 |= 1ull << pp;
        pp = __builtin_amdgcn_readlane(n0, pp);
      }
      while (pp < kLPos) {
        cm1 |= 1ull << (pp - 64);
        pp = __builtin_amdgcn_readlane(n1, pp - 64);
      }
#else
      chain_marks128(n0, n1, lds_ptr(sh->cflag), cm0, cm1);
#endif
      const bool on0 = (cm0 >> lane) & 1, on1 = (cm1 >> lane) & 1;
      PQG_LT(tc);
      PQG_LA(1, tc - tb);
      // ---- 3. value offsets, takes, checks
      const uint32_t c0 = on0 ? r0.cnt : 0u, c1 = on1 ? r1.cnt : 0u;
      const uint32_t i0 = ldpp_incl_add_sat(c0);
      const uint32_t t0 = (uint32_t)__builtin_amdgcn_readlane((int)i0, 63);
      uint32_t i1 = ldpp_incl_add_sat(c1);
      i1 = i1 + t0 < i1 ? 0xffffffffu : i1 + t0;
      const uint32_t s0 = i0 - c0, s1 = i1 - c1;  // values before the run (within this window)
      // a run is needed while values before it < left; its take is min(cnt, left - before)
      auto assess = [&](const LRun& r, uint32_t st, bool on, int& e, uint32_t& take, bool& cut) {
        e = kOK;
        take = 0;
        cut = false;
        if (!on || st >= left) return;
        if (r.cplx) { e = kCOMPLEX; return; }
        if (r.err != kOK) { e = r.err; return; }
        take = r.cnt < left - st ? r.cnt : left - st;
        if (r.bp) {
          const uint64_t need = (take + 7) >> 3;
          if ((uint64_t)r.pay + (need - 1) * (uint32_t)w >= n) {  // short read: whole groups that start in the stream
            const uint32_t ok = r.pay < n ? (n - r.pay + (uint32_t)w - 1) / (uint32_t)w : 0u;
            take = ok * 8;
            e = kEOF;
          }
          const uint64_t pend = (uint64_t)r.pay + (((uint64_t)take * (uint32_t)w + 7) >> 3) + 8;
          cut = !in_win(r.pay, (uint32_t)(pend - r.pay));
        }
        cut |= pre + st + take > (uint32_t)kLSpan;
      };
      int e0, e1;
      uint32_t k0, k1;
      bool x0, x1;
      assess(r0, s0, on0, e0, k0, x0);
      assess(r1, s1, on1, e1, k1, x1);
      const uint64_t eb0 = __ballot(e0 != kOK), eb1 = __ballot(e1 != kOK);
      const uint64_t xb0 = __ballot(x0), xb1 = __ballot(x1);
      const uint64_t nb0 = __ballot(on0 && s0 < left), nb1 = __ballot(on1 && s1 < left);  // needed runs
      const int first_err = eb0 ? __ffsll((long long)eb0) - 1 : eb1 ? 64 + __ffsll((long long)eb1) - 1 : kLPos;
      const int first_cut = xb0 ? __ffsll((long long)xb0) - 1 : xb1 ? 64 + __ffsll((long long)xb1) - 1 : kLPos;
      PQG_LT(td);
      PQG_LA(2, td - tc);
      if (first_err < first_cut) {
        // runs before the error are fine: the stream fails there (for levels the
        // values do not matter then); a 5+ byte header is walked serially
        const int l = first_err & 63;
        const int e = __builtin_amdgcn_readlane(first_err < 64 ? e0 : e1, l);
        if (e != kCOMPLEX) return e;
        // serial header at the complex run, then that single run as a long run
        const uint32_t q = pos + (uint32_t)first_err;
        // produce the runs before it first
        const uint32_t before_v = (uint32_t)__builtin_amdgcn_readlane((int)(first_err < 64 ? s0 : s1), l);
        if (first_err > 0) {
          const int ee = emit_batch(cm0, cm1, first_err, r0, r1, s0, s1, k0, k1, produced, before_v);
          if (ee) return ee;
        }
        produced += before_v;
        uint32_t h, hl;
        const int es = lrun_serial(lds_ptr(sh->win), q - wbase, q, n, &h, &hl);
        if (es) return es;
        if ((h >> 1) == 0) return kRLE;
        const int el = long_run(q, h, hl, produced, pos);
        if (el) return el;
        continue;
      }
      if (first_cut == 0) {
        // run 0 alone is longer than a batch (or its payload leaves the window)
        uint32_t h;  // rebuild the header fields of run 0
        const bool bp = __builtin_amdgcn_readlane((int)r0.bp, 0) != 0;
        const uint32_t cnt = (uint32_t)__builtin_amdgcn_readlane((int)r0.cnt, 0);
        const uint32_t pay = (uint32_t)__builtin_amdgcn_readlane((int)r0.pay, 0);
        const uint32_t nx = (uint32_t)__builtin_amdgcn_readlane((int)r0.next, 0);
        const int el = long_run_fields(bp, cnt, pay, nx, produced, pos);
        PQG_LA(7, 1);
        (void)h;
        if (el) return el;
        continue;
      }
      // ---- 4. the batch: needed runs before the cut
      const int nruns = first_cut;  // positions < nruns
      const uint64_t need0 = nb0, need1 = nb1;
      const int e = emit_batch(cm0 & need0, cm1 & need1, nruns, r0, r1, s0, s1, k0, k1, produced, 0xffffffffu);
      if (e) return e;
      // values and the next header position: from the last batch run
      const uint64_t bm0 = cm0 & need0 & (nruns >= 64 ? ~0ull : ((1ull << nruns) - 1));
      const uint64_t bm1 = nruns > 64 ? cm1 & need1 & (nruns >= 128 ? ~0ull : ((1ull << (nruns - 64)) - 1)) : 0ull;
      const bool last_hi = bm1 != 0;
      const int ll = 63 - __builtin_clzll(last_hi ? bm1 : bm0);
      const uint32_t lst = (uint32_t)__builtin_amdgcn_readlane((int)(last_hi ? s1 : s0), ll);
      const uint32_t ltk = (uint32_t)__builtin_amdgcn_readlane((int)(last_hi ? k1 : k0), ll);
      const uint32_t lnx = (uint32_t)__builtin_amdgcn_readlane((int)(last_hi ? r1.next : r0.next), ll);
      produced += lst + ltk;
      pos = lnx;
      PQG_LT(te);
      PQG_LA(3, te - td);
      PQG_LA(4, 1);
      PQG_LA(5, __popcll(bm0) + __popcll(bm1));
    }
    return kOK;
  }

  // Run tables + expansion for the chain's runs at positions < nruns (masks
  // m0/m1), values [produced, produced + total).  A run's value limit is its take.
  __device__ int emit_batch(uint64_t m0, uint64_t m1, int nruns, const LRun& r0, const LRun& r1, uint32_t s0,
                            uint32_t s1, uint32_t k0, uint32_t k1, uint32_t produced, uint32_t limit) {
    const int lane = lane_id();
    const uint64_t lm0 = nruns >= 64 ? ~0ull : ((1ull << nruns) - 1);
    const uint64_t lm1 = nruns > 64 ? (nruns >= 128 ? ~0ull : ((1ull << (nruns - 64)) - 1)) : 0ull;
    m0 &= lm0;
    m1 &= lm1;
    const bool b0 = (m0 >> lane) & 1, b1 = (m1 >> lane) & 1;
    const uint32_t pre = (uint32_t)(((uintptr_t)out + produced) & 15);
    if (kW1 || w == 1) {
      bits_clear();
      const bool hi = m1 != 0;
      const int ll = 63 - __builtin_clzll(hi ? m1 : m0);
      uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)(hi ? s1 : s0), ll) +
                       (uint32_t)__builtin_amdgcn_readlane((int)(hi ? k1 : k0), ll);
      if (total > limit) total = limit;
      // each run lane ORs the dwords its values cover
      const uint32_t st0 = pre + s0, st1 = pre + s1;
      const uint32_t l0 = b0 ? (k0 < total - s0 ? k0 : total - s0) : 0u;
      const uint32_t l1 = b1 ? (s1 < total ? (k1 < total - s1 ? k1 : total - s1) : 0u) : 0u;
      const uint32_t inf0 = r0.bp ? (r0.pay - wbase) * 8 : r0.pay, inf1 = r1.bp ? (r1.pay - wbase) * 8 : r1.pay;
      if (l0) for (uint32_t k = st0 >> 5; k <= (st0 + l0 - 1) >> 5; k++) bits_or(st0, l0, r0.bp, inf0, k);
      if (l1) for (uint32_t k = st1 >> 5; k <= (st1 + l1 - 1) >> 5; k++) bits_or(st1, l1, r1.bp, inf1, k);
      if (total) bits_store(produced, total);
      return kOK;
    }
    if constexpr (!kW1) {
    PQG_L uint8_t* TM = lds_ptr(sh->tmap);
    PQG_L u32x2_t* TE = lds_ptr(sh->tent);
    *(PQG_L u32x4_t*)(TM + 16 * lane) = u32x4_t{0u, 0u, 0u, 0u};
    __builtin_amdgcn_wave_barrier();
    if (b0) {
      TE[lane] = u32x2_t{pre + s0, r0.bp ? (0x80000000u | ((r0.pay - wbase) * 8)) : r0.pay};
      TM[pre + s0] = (uint8_t)(lane + 1);
    }
    if (b1) {
      TE[64 + lane] = u32x2_t{pre + s1, r1.bp ? (0x80000000u | ((r1.pay - wbase) * 8)) : r1.pay};
      TM[pre + s1] = (uint8_t)(65 + lane);
    }
    __builtin_amdgcn_wave_barrier();
    // total values: the last run's start + take
    const bool hi = m1 != 0;
    const int ll = 63 - __builtin_clzll(hi ? m1 : m0);
    uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)(hi ? s1 : s0), ll) +
                     (uint32_t)__builtin_amdgcn_readlane((int)(hi ? k1 : k0), ll);
    if (total > limit) total = limit;
    if (total) expand(produced, total);
    }
    return kOK;
  }

  // One run [header at q] in pieces of <= kLSpan values.
  __device__ int long_run(uint32_t q, uint32_t h, uint32_t hl, uint32_t& produced, uint32_t& pos) {
    const bool bp = (h & 1) != 0;
    const uint32_t g = h >> 1;
    uint32_t cnt, pay, nx;
    if (bp) {
      cnt = g > 0x1fffffffu ? 0xffffffffu : g * 8;
      pay = q + hl;
      const uint64_t t = (uint64_t)q + hl + (uint64_t)g * (uint32_t)w;
      nx = t > 0xffffffffull ? 0xffffffffu : (uint32_t)t;
    } else {
      const uint32_t vp = q + hl;
      if (vp >= n) return kEOF;
      if (!in_win(vp, 1)) fill(vp);
      pay = lds_ptr(sh->win)[vp - wbase];
      if ((pay >> w) != 0) return kRLE;
      cnt = g;
      nx = vp + 1;
    }
    return long_run_fields(bp, cnt, pay, nx, produced, pos);
  }

  // Record the run [produced, produced + take) for k_level_long (pieces of
  // kLevPiece values); false (nothing recorded) when the tables are full.
  __device__ bool defer_long(bool bp, uint32_t take, uint32_t pay, uint32_t produced) {
    const int lane = lane_id();
    const uint32_t P = (take + kLevPiece - 1) / kLevPiece;
    int li = 0, pb = 0;
    if (lane == 0) {
      li = atomicAdd(ctr + kCtrLongLev, 1);
      pb = li < long_cap ? atomicAdd(ctr + kCtrLevPieces, (int)P) : 0;
    }
    li = __builtin_amdgcn_readfirstlane(li);
    pb = __builtin_amdgcn_readfirstlane(pb);
    if (li >= long_cap) return false;
    const bool ok = (int64_t)pb + P <= (int64_t)piece_cap;
    if (lane == 0) {
      LongLev L;
      L.out = (uint8_t*)(out + produced);
      L.p = bp ? (const uint8_t*)(p + pay) : nullptr;
      L.end = (const uint8_t*)(p + n);
      L.count = take;
      L.value = bp ? 0u : pay;
      L.w = w;
      L.maxl = (int32_t)maxl;
      L.pidx = pidx;
      L.pad = 0;
      longs[li] = L;
    }
    // the reserved pieces (those inside the table): the run's, or empty when
    // the table cannot hold them all (the run is then expanded here)
    for (uint32_t j = (uint32_t)lane; j < P && (int64_t)pb + j < (int64_t)piece_cap; j += 64) {
      LevPiece pc;
      pc.run = ok ? li : -1;
      pc.v0 = j * kLevPiece;
      pc.v1 = min(take, (j + 1) * (uint32_t)kLevPiece);
      pieces[pb + j] = pc;
    }
    return ok;
  }

  __device__ int long_run_fields(bool bp, uint32_t cnt, uint32_t pay, uint32_t nx, uint32_t& produced, uint32_t& pos) {
    const int lane = lane_id();
    const uint32_t left = count - produced;
    uint32_t take = cnt < left ? cnt : left;
    int status = kOK;
    if (bp) {
      const uint64_t need = (take + 7) >> 3;
      if ((uint64_t)pay + (need - 1) * (uint32_t)w >= n) {
        const uint32_t ok = pay < n ? (n - pay + (uint32_t)w - 1) / (uint32_t)w : 0u;
        take = ok * 8;
        status = kEOF;
      }
    }
    if (status != kOK) return status;  // levels: the values of a failing stream do not matter
    if (take > (uint32_t)kLongLev && longs && defer_long(bp, take, pay, produced)) {
      deferred = true;
      produced += take;
      pos = nx;
      return kOK;
    }
    uint32_t done = 0;
    while (done < take) {
      const uint32_t pre = (uint32_t)(((uintptr_t)out + produced) & 15);
      uint32_t piece = take - done;
      if (piece > (uint32_t)kLSpan - pre) piece = (uint32_t)kLSpan - pre;
      uint32_t info = pay;
      if (bp) {
        const uint64_t b0 = (uint64_t)pay * 8 + (uint64_t)done * (uint32_t)w;  // stream bit of the piece
        const uint32_t byte0 = (uint32_t)(b0 >> 3);
        const uint32_t nbytes = (uint32_t)(((uint64_t)piece * (uint32_t)w + 7) >> 3) + 8;
        if (!in_win(byte0, nbytes)) fill(byte0);
        info = 0x80000000u | (uint32_t)(((uint64_t)(byte0 - wbase) << 3) + (b0 & 7));
      }
      if (kW1 || w == 1) {
        // one dword of the piece per lane
        bits_clear();
        if ((uint32_t)lane <= (pre + piece - 1) >> 5) bits_or(pre, piece, bp, bp ? (info & 0x7fffffffu) : pay, lane);
        bits_store(produced, piece);
        produced += piece;
        done += piece;
        continue;
      }
      if constexpr (!kW1) {
      PQG_L uint8_t* TM = lds_ptr(sh->tmap);
      *(PQG_L u32x4_t*)(TM + 16 * lane) = u32x4_t{0u, 0u, 0u, 0u};
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) {
        lds_ptr(sh->tent)[0] = u32x2_t{pre, info};
        TM[pre] = 1;
      }
      __builtin_amdgcn_wave_barrier();
      expand(produced, piece);
      produced += piece;
      done += piece;
      }
    }
    pos = nx;
    return kOK;
  }
};

struct LongTables {
  LongLev* longs;
  LevPiece* pieces;
  int* ctr;
  int long_cap, piece_cap;
};

using LevelDecoder = LevelDecoderT<false>;

template <bool kW1 = false>
__device__ __forceinline__ int level_stream(gcu8 p, int64_t n, int w, uint32_t count, gu8 out, uint32_t maxl,
                                            LevShared& sh, uint32_t* nn, const LongTables& lt, int pidx,
                                            bool* deferred = nullptr) {
  LevelDecoderT<kW1> dec{p, (uint32_t)n, kW1 ? 1 : w, count, out, maxl, &sh, lt.longs, lt.pieces, lt.ctr, lt.long_cap,
                         lt.piece_cap, pidx};
  const int e = dec.run();
#ifdef PQG_PROFILE
  for (int k = 0; k < 8; k++) PQG_ACC(k, 0, dec.pacc[k]);
#endif
  *nn = (uint32_t)wave_sum((int64_t)dec.nn);
  if (deferred) *deferred = dec.deferred;
  return e;
}

// The read phase of one data page (V1 initSize: page_v1.go:99-105,
// hybrid_decoder.go:57-67; V2 raw level bytes: page_v2.go:103-121): its block,
// level and value streams, the value stream registered for the walker
// (dictionary indices type_dict.go:22-37, RLE booleans type_boolean.go:100-120)
// and its values stage.  `writer`: this thread writes the page record.
struct PageStreams {
  gcu8 rep, def;
  int64_t rep_n, def_n;  // -1: the level decoder is not initialised
  int e;                 // read-phase error
  gcu8 val;              // the values section (what the page record's val / val_n hold)
  int64_t val_n;
  int vmode;             // the page's values stage (PageDev.vmode)
};
__device__ __forceinline__ PageStreams page_setup(const JobDev& job, const PageDev& pg, int pidx, PageDev* pages,
                                                  HStream* streams, const int* total, const uint8_t* scratch,
                                                  bool writer) {
  PageStreams r{nullptr, nullptr, -1, -1, kOK, nullptr, 0, -1};
  gcu8 block;
  int64_t blen;
  int32_t levels = 0;
  if (pg.page_type == 3) {
    levels = (int32_t)((uint32_t)pg.rep_len + (uint32_t)pg.def_len);
    blen = (int32_t)((uint32_t)pg.csize - (uint32_t)levels);
    if (pg.scratch_offset >= 0) blen = (int32_t)((uint32_t)pg.usize - (uint32_t)levels);
  } else {
    blen = pg.scratch_offset >= 0 ? pg.usize : pg.csize;
  }
  if (pg.scratch_offset >= 0) block = gconst(scratch) + job.scratch_base + pg.scratch_offset;
  else block = gconst(job.data) + pg.payload_offset + (levels > 0 ? levels : 0);
  int64_t vpos = 0;
  if (pg.page_type == 0) {
    // rDecoder.initSize then dDecoder.initSize (page_v1.go:99-105)
    if (job.max_rep > 0) {
      if (blen - vpos < 4) r.e = kEOF;
      else {
        const int64_t sz = rd_u32(block + vpos);
        const int64_t take = min(sz, blen - vpos - 4);
        r.rep = block + vpos + 4;
        r.rep_n = take;
        vpos += 4 + take;
      }
    }
    if (r.e == kOK && job.max_def > 0) {
      if (blen - vpos < 4) r.e = kEOF;
      else {
        const int64_t sz = rd_u32(block + vpos);
        const int64_t take = min(sz, blen - vpos - 4);
        r.def = block + vpos + 4;
        r.def_n = take;
        vpos += 4 + take;
      }
    }
  } else {
    // V2: raw level bytes, a decoder only for a non-empty section (page_v2.go:110-120)
    gcu8 lv = gconst(job.data) + pg.payload_offset;
    if (levels > 0 && pg.rep_len > 0) { r.rep = lv; r.rep_n = pg.rep_len; }
    if (levels > 0 && pg.def_len > 0) { r.def = lv + pg.rep_len; r.def_n = levels - pg.rep_len; }
  }
  if (r.e != kOK) {
    if (writer) pages[pidx].read_status = r.e;
    return r;
  }
  const int64_t n = pg.num_values;
  const int64_t vn = blen - vpos;
  gcu8 val = block + vpos;
  r.val = val;
  r.val_n = vn;
  r.vmode = job.value_width == 0 || (pg.encoding == 7 && job.type == 7) ? 2
            : (pg.encoding == 8 && job.value_width == 4)                ? 1
            : pg.encoding == 5                                          ? 3
                                                                        : 0;
  if (writer) {
    PageDev& P = pages[pidx];
    P.block = (const uint8_t*)block;
    P.block_len = blen;
    P.val = (const uint8_t*)val;
    P.val_n = vn;
    P.rep = (const uint8_t*)r.rep;
    P.rep_n = r.rep_n;
    P.def = (const uint8_t*)r.def;
    P.def_n = r.def_n;
    // values: RLE_DICTIONARY indices (first byte = bit width) / RLE booleans (u32 length)
    if (pg.encoding == 8 && vn >= 1) {
      const int wv = val[0];
      P.dict_width = wv;
      if (wv >= 1 && wv <= 32 && n > 0) reg_stream(job, pg, streams, &P.hs_val, pidx, 2, val + 1, vn - 1, wv, n);
    } else if (pg.encoding == 3 && job.type == 0 && vn >= 4) {
      const int64_t sz = rd_u32(val);
      const int64_t take = min(sz, vn - 4);
      if (n > 0) reg_stream(job, pg, streams, &P.hs_val, pidx, 3, val + 4, take, 1, n);
    }
    // value-stage page lists: 4-byte dictionary pages (the hot path, a kernel
    // of its own), variable-length values (pqg_strings.hip) and everything else
    // (DELTA_BYTE_ARRAY on FLBA: the strings stage, values of type_length bytes)
    const int vm = r.vmode;
    P.vmode = vm;
    int* present = const_cast<int*>(total) + kModePresentOff;
    if (present[vm] == 0) present[vm] = 1;
    // flag 4: DELTA_LENGTH_BYTE_ARRAY / DELTA_BYTE_ARRAY pages (k_str_delta, k_str_dba)
    if (vm == 2 && (pg.encoding == 6 || pg.encoding == 7) && present[4] == 0) present[4] = 1;
  }
  return r;
}

}  // namespace pqg
