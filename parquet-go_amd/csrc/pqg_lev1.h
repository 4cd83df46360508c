// pqg_lev1.h — the whole-page decoder for 1-bit level streams (maxLevel 1:
// optional flat columns, the C2 shape), used by k_page_levels_w1.
//
// The page's def stream (<= kL1MaxN bytes) is staged in LDS with one round of
// loads and decoded with no per-batch loop:
//   1. backward exit table: lane l owns stream positions [l S, l S + S) (S =
//      ceil(n / 64) <= 64) and walks them from the last to the first, parsing
//      a run header at every position (hybridDecoder.readRunHeader,
//      hybrid_decoder.go:143-166; RLE value / bit-packed extent :116-141).
//      Position p's exit — the first header position at or past the segment's
//      end on the chain from p — is the successor's exit when the successor is
//      inside the segment (already known: headers are >= 2 bytes apart), else
//      the successor itself.  One byte per position (offset past the
//      segment's end, "far", or "bad": an error or a 5-byte header on the way);
//   2. link: the true chain's entry into every segment, 64 dependent table
//      reads (entry(l + 1) = exit(entry(l)) from position 0);
//   3. each lane walks its segment's part of the chain twice: the value count
//      (a saturating wave scan gives every lane its first value), then the
//      bits, OR-ed into an LDS bitmap of the page's values;
//   4. the wave expands the bitmap 16 values per lane (nibble x 0x00204081)
//      into aligned 16-byte stores of level bytes and counts notNull.
// No global store happens before every check has passed; a page this path
// does not take (longer stream, more values, an error or a 5+ byte header on
// the chain, a chain short of the page's values, a short bit-packed read) is
// decoded by the exact batch decoder (pqg_levdec.h), which reports the
// reference's error (hybridDecoder.next, hybrid_decoder.go:82-114).
#pragma once
#include "pqg_levdec.h"

namespace pqg {

constexpr int kL1MaxN = 4096;               // stream bytes
constexpr int kL1MaxCount = 32768 - 16;     // values (+ <= 15 alignment bits: a 4 KiB bitmap)
constexpr int kL1Win = kL1MaxN + 64;        // window: 15 alignment bytes, the stream, zeros for reads past n
constexpr uint32_t kL1Far = 254, kL1Bad = 255;

struct Lev1Shared {
  uint8_t win[kL1Win];
  uint32_t tab[kL1MaxN / 4 + 2];  // exit codes (one byte per position), then the value bitmap
};

struct L1Hdr {
  uint32_t nx;   // position of the next header
  uint32_t cnt;  // values of the run
  uint32_t pay;  // bit-packed: payload position; RLE: the value
  bool bp, bad;
};

// The run header at stream position q (win[mis + q] = byte q, zeros past n):
// readUVariant32 (helpers.go:149-165) for headers of <= 4 bytes; 5+ byte
// headers, EOF inside the header or the RLE value, empty runs and RLE values
// >= 2 are `bad` (the exact decoder settles them).
// lo / hi: stream bytes q..q+3 / q+4..q+7.
__device__ __forceinline__ L1Hdr l1_hdr(uint32_t lo, uint32_t hi, uint32_t q, uint32_t n) {
  // branch-free (every position of a segment is parsed: divergent bit-packed
  // / RLE branches would run both sides)
  const uint32_t cont = ~lo & 0x80808080u;
  const uint32_t hl = (cont ? (uint32_t)__builtin_ctz(cont) >> 3 : 4u) + 1;  // 5: no terminating byte in four
  const uint32_t hf = (lo & 0x7f) | ((lo >> 1) & 0x3f80) | ((lo >> 2) & 0x1fc000) | ((lo >> 3) & 0xfe00000);
  const uint32_t h = __builtin_amdgcn_ubfe(hf, 0, 7 * hl);  // hl 5: garbage, and bad below
  const uint32_t g = h >> 1;
  const bool bp = (h & 1) != 0;
  const uint32_t vb = (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * hl)) & 0xff;  // the byte after the header
  const uint32_t ve = q + hl;
  L1Hdr r;
  r.bp = bp;
  // readRLERunValue: the value byte must be there and < 2^w (:116-131)
  r.bad = (hl > 4) | (ve > n) | (g == 0) | (!bp & ((ve >= n) | (vb > 1)));  // bitwise: no branches
  r.cnt = bp ? g * 8 : g;  // g < 2^27
  r.pay = bp ? ve : vb;
  r.nx = ve + (bp ? g : 1u);
  return r;
}
__device__ __forceinline__ L1Hdr l1_parse(const PQG_L uint8_t* win, uint32_t mis, uint32_t q, uint32_t n) {
  const uint32_t wo = mis + q;
  const PQG_L uint32_t* d = (const PQG_L uint32_t*)(win + (wo & ~3u));
  const uint32_t a = d[0], b = d[1], c = d[2];
  const uint32_t sft = (wo & 3) * 8;
  return l1_hdr(__builtin_amdgcn_alignbit(b, a, sft), __builtin_amdgcn_alignbit(c, b, sft), q, n);
}
// A header on the chain (checked by the table walk: <= 4 bytes, no error):
// the fields the value walks need, without the checks.
struct L1Run {
  uint32_t hl, g, vb;  // header bytes, h >> 1, the byte after the header
  bool bp;
};
__device__ __forceinline__ L1Run l1_run(const PQG_L uint8_t* win, uint32_t mis, uint32_t q) {
  const uint32_t wo = mis + q;
  const PQG_L uint32_t* d = (const PQG_L uint32_t*)(win + (wo & ~3u));
  const uint32_t a = d[0], b = d[1], c = d[2];
  const uint32_t sft = (wo & 3) * 8;
  const uint32_t lo = __builtin_amdgcn_alignbit(b, a, sft), hi = __builtin_amdgcn_alignbit(c, b, sft);
  const uint32_t cont = ~lo & 0x80808080u;
  L1Run r;
  r.hl = (cont ? (uint32_t)__builtin_ctz(cont) >> 3 : 3u) + 1;
  const uint32_t hf = (lo & 0x7f) | ((lo >> 1) & 0x3f80) | ((lo >> 2) & 0x1fc000) | ((lo >> 3) & 0xfe00000);
  const uint32_t h = __builtin_amdgcn_ubfe(hf, 0, 7 * r.hl);
  r.g = h >> 1;
  r.bp = (h & 1) != 0;
  r.vb = (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * r.hl)) & 0xff;
  return r;
}

// the exit code of a header whose successor lies at or past the segment's end e
__device__ __forceinline__ uint32_t l1_code(const L1Hdr& h, uint32_t e) {
  const uint32_t d = h.nx - e;
  return h.bad ? kL1Bad : (d < kL1Far ? d : kL1Far);
}

// OR the bits of values [s, s + len) of one run into the bitmap: bit-packed
// runs take window bits from `sbit`, RLE runs of value 1 ones.
__device__ __forceinline__ void l1_or_run(PQG_L uint32_t* bm, const PQG_L uint32_t* W, uint32_t s, uint32_t len,
                                          bool bp, uint32_t sbit) {
  const uint32_t e = s + len;
  for (uint32_t k = s >> 5; 32 * k < e; k++) {
    const uint32_t lo = s > 32 * k ? s : 32 * k;
    const uint32_t hi = e < 32 * k + 32 ? e : 32 * k + 32;
    const uint32_t cnt = hi - lo;
    const uint32_t m = cnt >= 32 ? 0xffffffffu : ((1u << cnt) - 1);
    uint32_t v = m;
    if (bp) {
      const uint32_t sb = sbit + (lo - s);
      v = __builtin_amdgcn_alignbit(W[(sb >> 5) + 1], W[sb >> 5], sb & 31) & m;
    }
    v <<= (lo - 32 * k);
    if (v) __hip_atomic_fetch_or(bm + k, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  }
}

// Decode `count` 1-bit levels of stream [p, p + n) into out[0, count) and
// count the ones (notNull for maxLevel 1).  false: not taken (nothing stored;
// the caller runs the exact decoder).
__device__ __forceinline__ bool lev1_page(gcu8 p, uint32_t n, uint32_t count, gu8 out, Lev1Shared& sh, uint32_t* nn_out) {
  const int lane = lane_id();
  if (n == 0 || n > (uint32_t)kL1MaxN || count > (uint32_t)kL1MaxCount) return false;
  PQG_L uint8_t* win = lds_ptr(sh.win);
  PQG_T(t0);
  // ---- 0. stage the stream: 16-byte granules from the aligned base; bytes
  // past the stream read as zero.  Every load is issued (clamped to the base:
  // a guarded load is waited for inside its branch), then masked and stored.
  const uintptr_t pa = (uintptr_t)p;
  const uint32_t mis = (uint32_t)(pa & 15);
  const uintptr_t base = pa - mis;
  const uint32_t lim = mis + n;
  constexpr int kR = (kL1Win + 1023) / 1024;  // 5 rounds of 1 KiB
  uint4 v[kR];
#pragma unroll
  for (int h = 0; h < kR; h++) {
    const uint32_t g = 1024u * h + 16u * lane;
    v[h] = ldg16(g < lim ? base + g : base);
  }
#pragma unroll
  for (int h = 0; h < kR; h++) {
    const uint32_t g = 1024u * h + 16u * lane;
    if (g < (uint32_t)kL1Win) sts16(win + g, g < lim ? mask_tail(v[h], g, lim) : make_uint4(0, 0, 0, 0));
  }
  __builtin_amdgcn_wave_barrier();
  PQG_T(t1);
  PQG_ACC(20, t0, t1);
  // ---- 1. exit codes, each lane over its segment from the end
  PQG_L uint8_t* T = (PQG_L uint8_t*)lds_ptr(sh.tab);
  const uint32_t S = (((n + 63) >> 6) + 3) & ~3u;  // a multiple of 4, <= 64
  const uint32_t a = (uint32_t)lane * S;
  const uint32_t e = a + S < n ? a + S : n;
  // the top (e - a) % 4 positions one at a time, then groups of four: the
  // four headers from one 16-byte read, their successors' codes read together
  // (a header's successor is >= 2 positions on: the group's two upper codes
  // are forwarded to its two lower positions in registers)
  int q = (int)e - 1;
  for (int r = (int)((e > a ? e - a : 0u) & 3); r > 0; r--, q--) {
    const L1Hdr h = l1_parse(win, mis, (uint32_t)q, n);
    uint32_t code = l1_code(h, e);
    if (!h.bad && h.nx < e) code = T[h.nx];
    T[q] = (uint8_t)code;
  }
  for (; q >= (int)a + 3; q -= 4) {
    const uint32_t q0 = (uint32_t)q - 3;  // positions q0 .. q0 + 3
    const uint32_t wo = mis + q0;
    const PQG_L uint32_t* d = (const PQG_L uint32_t*)(win + (wo & ~3u));
    const uint32_t d0 = d[0], d1 = d[1], d2 = d[2], d3 = d[3];
    const uint32_t o = wo & 3;  // byte of position q0 in d0
    L1Hdr h[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t oj = o + j;  // 0..6
      const uint32_t sft = (oj & 3) * 8;
      const bool up = oj >= 4;
      const uint32_t x0 = up ? d1 : d0, x1 = up ? d2 : d1, x2 = up ? d3 : d2;
      h[j] = l1_hdr(__builtin_amdgcn_alignbit(x1, x0, sft), __builtin_amdgcn_alignbit(x2, x1, sft), q0 + j, n);
    }
    uint32_t t[4], c[4];
    bool in[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      in[j] = !h[j].bad & (h[j].nx < e);
      t[j] = T[in[j] ? h[j].nx : q0 + 3];  // unconditional (clamped) read
      c[j] = l1_code(h[j], e);
    }
    // successors inside the group come from registers (q0 + 2 / q0 + 3: written below)
    const uint32_t c3 = in[3] ? t[3] : c[3];
    const uint32_t c2 = in[2] ? t[2] : c[2];  // successor >= q0 + 4
    const uint32_t c1 = in[1] ? (h[1].nx == q0 + 3 ? c3 : t[1]) : c[1];
    const uint32_t c0 = in[0] ? (h[0].nx == q0 + 3 ? c3 : h[0].nx == q0 + 2 ? c2 : t[0]) : c[0];
    *(PQG_L uint32_t*)(T + q0) = c0 | c1 << 8 | c2 << 16 | c3 << 24;  // q0 = a + 4k: aligned
  }
  __builtin_amdgcn_wave_barrier();
  PQG_T(t2);
  PQG_ACC(21, t1, t2);
  // ---- 2. the chain's entry into every segment
  uint32_t E = 0, myE = 0;
  bool ok = true;
  for (int l = 0; l < 64; l++) {
    const uint32_t al = (uint32_t)l * S;
    if (lane == l) myE = E;
    if (al >= n) continue;
    const uint32_t el = al + S < n ? al + S : n;
    if (E >= el) continue;  // a bit-packed payload covers the segment
    const uint32_t code = (uint32_t)__builtin_amdgcn_readfirstlane((int)T[E]);
    if (code == kL1Bad) { ok = false; break; }
    if (code == kL1Far) {  // an exit past the table's reach: walk it
      uint32_t q = E;
      while (q < el) {
        const L1Hdr h = l1_parse(win, mis, q, n);
        if (h.bad) { ok = false; break; }
        q = (uint32_t)__builtin_amdgcn_readfirstlane((int)h.nx);
      }
      if (!ok) break;
      E = q;
    } else {
      E = el + code;
    }
  }
  PQG_T(t3);
  PQG_ACC(22, t2, t3);
  if (!ok) { PQG_ACC(27, 0, 1); return false; }
#ifdef PQG_L1_STOP_AFTER_LINK  // timing experiment only (wrong outputs)
  *nn_out = 0;
  return true;
#endif
  // ---- 3a. values per segment and the segment's chain positions (bit q - a)
  uint32_t C = 0;
  uint64_t cm = 0;
  for (uint32_t q = myE; q < e;) {
    const L1Run r = l1_run(win, mis, q);
    const uint32_t cnt = r.bp ? r.g * 8 : r.g;
    C = C + cnt < (1u << 24) ? C + cnt : (1u << 24);  // > any page count: the scan cannot wrap
    cm |= 1ull << (q - a);
    q += r.hl + (r.bp ? r.g : 1u);
  }
  const uint32_t incl = ldpp_incl_add_sat(C);
  const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  if (total < count) return false;  // the stream ends early: EOF (the exact decoder reports where)
  const uint32_t B = incl - C;
  PQG_T(t4);
  PQG_ACC(23, t3, t4);
  // ---- 3b. the bits: bitmap bit pre + i = value i.  Each lane appends its
  // runs' bits to a word accumulator in value order; its whole words are
  // plain stores, its first and last (shared with the neighbouring lanes)
  // atomic ORs.  The runs come from the chain mask, so their header reads do
  // not wait for one another.
  const uintptr_t oa = (uintptr_t)out;
  const uintptr_t a0 = oa & ~(uintptr_t)15;
  const uint32_t pre = (uint32_t)(oa - a0);
  const uint32_t end = pre + count;
  PQG_L uint32_t* bm = lds_ptr(sh.tab);
  const uint32_t nw = (end + 31) >> 5;
  __builtin_amdgcn_wave_barrier();
  for (uint32_t k = (uint32_t)lane; k <= nw; k += 64) bm[k] = 0u;
  __builtin_amdgcn_wave_barrier();
  const PQG_L uint32_t* W = (const PQG_L uint32_t*)win;
  bool fail = false;
  uint32_t c = B;
  uint32_t k = (pre + c) >> 5, fill = (pre + c) & 31;
  uint64_t acc = 0;  // bits [32 k, 32 k + fill) of the bitmap (a run of <= 32 values is one step)
  const uint32_t kfirst = k;
  uint32_t nn = 0;
  uint64_t m = c < count ? cm : 0ull;
#ifdef PQG_L1_SKIP_EMIT  // timing experiment only (wrong outputs)
  m = 0;
#endif
  auto flush = [&](uint32_t word) {
    if (k == kfirst) __hip_atomic_fetch_or(bm + k, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    else bm[k] = word;
    nn += __builtin_popcount(word);
    k++;
  };
  // the next run's header is read while the current one's bits are placed
  uint32_t rq = 0;
  L1Run r{};
  if (m) {
    rq = a + (uint32_t)__builtin_ctzll(m);
    m &= m - 1;
    r = l1_run(win, mis, rq);
  }
  bool more = c < count && cm != 0;
  while (more) {
    const L1Run cur = r;
    const uint32_t cq = rq;
    const bool next = m != 0;
    if (next) {
      rq = a + (uint32_t)__builtin_ctzll(m);
      m &= m - 1;
      r = l1_run(win, mis, rq);
    }
    const uint32_t cnt = cur.bp ? cur.g * 8 : cur.g;
    uint32_t take = cnt < count - c ? cnt : count - c;
    const uint32_t pay = cq + cur.hl;  // bit-packed payload
    // a short read: the last needed group must start inside the stream (Q5)
    if (cur.bp && pay + ((take + 7) >> 3) - 1 >= n) { fail = true; break; }
    c += take;
    const uint32_t pat = cur.vb ? 0xffffffffu : 0u;  // RLE
    const bool bp = cur.bp;
    uint32_t sb = bp ? (mis + pay) * 8 : 0u;
    while (take) {
      const uint32_t nb = take < 32 ? take : 32;
      const uint32_t src = __builtin_amdgcn_alignbit(W[(sb >> 5) + 1], W[sb >> 5], sb & 31);
      const uint32_t bits = (bp ? src : pat) & (nb >= 32 ? 0xffffffffu : ((1u << nb) - 1));
      acc |= (uint64_t)bits << fill;
      fill += nb;
      take -= nb;
      sb += nb;
      if (fill >= 32) {
        flush((uint32_t)acc);
        acc >>= 32;
        fill -= 32;
      }
    }
    more = next && c < count;
  }
  if (fill) {
    __hip_atomic_fetch_or(bm + k, (uint32_t)acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    nn += __builtin_popcount((uint32_t)acc);
  }
  if (__ballot(fail)) return false;
  PQG_T(t5);
  PQG_ACC(24, t4, t5);
  __builtin_amdgcn_wave_barrier();
  // ---- 4. level bytes, 16 per lane per step (whole granules: one aligned
  // 1 KiB wave store per step), the ragged first / last granule bytewise
  const PQG_L uint16_t* B16 = (const PQG_L uint16_t*)lds_ptr(sh.tab);
#ifdef PQG_L1_SKIP_EXPAND  // timing experiment only (wrong outputs)
  const uint32_t g0 = 1, g1 = 0;
#else
  const uint32_t g0 = (pre + 15) >> 4, g1 = end >> 4;  // whole granules [g0, g1)
#endif
  for (uint32_t g = g0 + (uint32_t)lane; g < g1; g += 64) {
    const uint32_t b16 = B16[g];
    uint32_t wv[4];
#pragma unroll
    for (int j = 0; j < 4; j++) wv[j] = (((b16 >> (4 * j)) & 0xfu) * 0x00204081u) & 0x01010101u;
    stg16o(a0 + 16 * g, make_uint4(wv[0], wv[1], wv[2], wv[3]));
  }
  if (lane < 32) {
    // the bytes outside whole granules: lanes 0..15 those of the first
    // granule, 16..31 those of the last (the same one for a short page: the
    // same bytes twice)
    const uint32_t gr = lane < 16 ? (pre >> 4) : (end >> 4);
    const uint32_t i = 16 * gr + (uint32_t)(lane & 15);
    if (i >= pre && i < end && (i < 16 * g0 || i >= 16 * g1))
      *(PQG_G uint8_t*)(a0 + i) = (uint8_t)((B16[gr] >> (lane & 15)) & 1);
  }
  *nn_out = (uint32_t)wave_sum((int64_t)nn);
  PQG_T(t6);
  PQG_ACC(25, t5, t6);
  PQG_ACC(26, 0, 1);
  return true;
}

}  // namespace pqg
