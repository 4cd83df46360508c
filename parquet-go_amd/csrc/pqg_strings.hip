// pqg_strings.hip — K7: variable-length values (BYTE_ARRAY, and FIXED_LEN_BYTE_ARRAY
// with length 0), PLAIN and RLE_DICTIONARY.
//
// Reference: byteArrayPlainDecoder (type_bytearray.go:13-55): every value is a
// u32 LE length (negative -> "bytearray/plain: len is negative") followed by
// that many bytes (io.ReadFull: short -> EOF); the dictionary page holds the
// same records (page_dict.go:30-64), and dictDecoder (type_dict.go:39-59)
// hands out dictionary entries by key.
//
// Output of a chunk: chars (the value bytes, concatenated in value order) and
// int64 offsets[num_values + 1] (offsets[0] = 0, offsets[i + 1] = end of
// value i) — Arrow's large-binary layout.
//
//   K7a k_str_dict   one block per chunk with a byte-array dictionary: the
//                    dictionary page's records -> record starts doffs[count + 1],
//                    then the dictionary is published
//   K7b k_str_plain  one block per PLAIN byte-array data page: the length chain
//                    -> page-relative value ends, written into the chunk's
//                    offsets; page.chars
//       k_str_count  one wave per dictionary-encoded byte-array page: the sum
//                    of its keys' entry lengths -> page.chars; the keys are
//                    parked in the value's offsets slot
//   K7c k_char_scan  one block per chunk: exclusive scan of page.chars
//   K7d k_str_copy   one block per byte-array data page: final offsets + chars
//                    (copied from the page records, or gathered from the
//                    dictionary)
//
// The length chain is the one serial dependency of the format; K7a/K7b cut it
// into segments walked in parallel from guessed starts and verified in order
// (block_walk below).
#include <hip/hip_runtime.h>

#include "pqg_common.h"
#include "pqg_device.h"
#include "pqg_hybrid.h"

namespace pqg {

#ifdef PQG_PROFILE
// host reader of this translation unit's phase counters (see pqg_debug_counters)
int prof_read_strings(unsigned long long* out) {
  unsigned long long z[64] = {0};
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pqg_prof), sizeof(z)) != hipSuccess) return -1;
  hipMemcpyToSymbol(HIP_SYMBOL(pqg_prof), z, sizeof(z));
  return 0;
}
#define PQG_ACC0(slot, v) do { if (threadIdx.x == 0) atomicAdd(&pqg_prof[slot], (unsigned long long)(v)); } while (0)
#else
#define PQG_ACC0(slot, v) do { } while (0)
#endif

// ---------------------------------------------------------------------------
// Block-parallel length-chain walk (PLAIN byte arrays and byte-array
// dictionary pages).
//
// The chain 0 -> 4 + len(0) -> ... is serial, but it is walked in parallel,
// 17 KiB of the stream at a time: the chunk is staged in LDS with one round
// of coalesced loads (the next chunk's loads are in flight meanwhile), each of
// the 256 threads takes a 68-byte segment, guesses where the chain enters it
// (the first position whose length chain is valid for three records; the
// segment holding the known chain position takes that) and walks its records
// from there, keeping their ends in registers.  The guesses are then checked
// all at once: every segment's entry must be the exit of the nearest segment
// before it that holds records (a block max-scan), and the first segment's is
// the known chain position.  When they all hold, a block scan of the record
// counts places every record and the ends are written; when one does not (or
// a record fails), thread 0 walks the chunk's true chain itself.  The result
// is exactly the serial chain whatever the data; the guess only decides
// whether the chunk takes the serial walk (for text-like records: never).
// ---------------------------------------------------------------------------
constexpr int kWalkT = 512;
constexpr int kPwT = kPwThreads;            // block_walk / k_str_plain block size (pqg_common.h)
constexpr int kPwSeg = 68;                  // bytes per thread segment (17 dwords: the lanes' reads
                                            // at the same offset of their segments hit distinct banks)
constexpr int kPwChunk = kPwT * kPwSeg;   // bytes per chunk (LDS)
constexpr int kPwRec = kPwSeg / 4;          // records a segment can hold (>= 4 bytes each)
constexpr int kPwAhead = 4096;              // staged past the chunk: the guesses' chain checks
constexpr int kPwStage = kPwChunk + kPwAhead + 64;
constexpr int kPwG = (kPwStage / 16 + kPwT - 1) / kPwT;  // staged granules per thread

struct BlockWalkShared {
  uint8_t buf[kPwG * kPwT * 16];  // the chunk from its 16-aligned start, + kPwAhead + 64 bytes
  uint32_t X[kPwT];          // per segment: exit (chain position after its records)
  int64_t part[kPwT / 64 + 1];
  int keys[kPwT / 64];
  uint32_t cur;                // the true chain position (the first record start not yet placed)
  uint32_t idx;                // records placed
  uint32_t last_end;           // end of record count - 1
  int status;
  int serial;
};

// u32 at LDS byte offset o (any alignment)
__device__ __forceinline__ uint32_t lds_u32(const PQG_L uint8_t* b, uint32_t o) {
  const PQG_L uint32_t* q = (const PQG_L uint32_t*)(b + (o & ~3u));
  return __builtin_amdgcn_alignbit(q[1], q[0], (o & 3) * 8);
}

// byteArrayPlainDecoder.next for records [0, count) of [p, p+n), the whole
// block.  mode 0 (data page): out[i] = char end of value i = end(i) - 4 (i + 1);
// mode 1 (dictionary page): out[i] = end(i), the next record's start.
// Returns the status (all threads); *chars = sum of the lengths.
__device__ int block_walk(gcu8 p, uint32_t n, uint32_t count, PQG_G int64_t* out, int mode, int64_t* chars,
                          BlockWalkShared& sh) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (t == 0) {
    sh.cur = 0;
    sh.idx = 0;
    sh.last_end = 0;
    sh.status = kOK;
  }
  const uintptr_t pend = (uintptr_t)(p + n);
  // granule k of the chunk from c0 (aligned start): mapped when it holds a stream byte
  // unconditional loads (a guarded load is waited for at its branch join,
  // which would make this prefetch synchronous): granules past the stream's
  // last one re-read that one; their bytes are never interpreted (every
  // length read checks n first)
  const uintptr_t lastg = (pend - 1) & ~(uintptr_t)15;
  auto load_chunk = [&](uint32_t c0, uint4 (&v)[kPwG]) {
    const uintptr_t A = (uintptr_t)(p + c0) & ~(uintptr_t)15;
#pragma unroll
    for (int k = 0; k < kPwG; k++) {
      const uintptr_t g = A + 16 * (uintptr_t)(t + kPwT * k);
      v[k] = ldg16(g < lastg ? g : lastg);
    }
  };
  uint4 nx[kPwG];
  if (count > 0 && n > 0) load_chunk(0, nx);
  __syncthreads();
  for (uint32_t c0 = 0; count > 0 && c0 < n; c0 += kPwChunk) {
    const uint32_t c1 = n - c0 > (uint32_t)kPwChunk ? c0 + kPwChunk : n;
    PQG_T(tq0);
    const uint32_t cur = sh.cur, idx0 = sh.idx;
    if (idx0 >= count) break;
    if (cur >= c1) {  // a record spans the chunk
      if (c1 < n) load_chunk(c1, nx);
      continue;
    }
    // stage this chunk, then start the next one's loads
#pragma unroll
    for (int k = 0; k < kPwG; k++) sts16(lds_ptr(sh.buf) + 16 * (t + kPwT * k), nx[k]);
    __syncthreads();
    if (c1 < n) load_chunk(c1, nx);
    PQG_ACC0(21, 1);
    PQG_T(tq1);
    PQG_ACC0(16, tq1 - tq0);
    const uint32_t off0 = (uint32_t)(((uintptr_t)(p + c0)) & 15);  // buf index of stream position c0
    const PQG_L uint8_t* B = lds_ptr(sh.buf);
    auto len_at = [&](uint32_t q) { return lds_u32(B, q - c0 + off0); };  // q + 4 <= c1 + kPwAhead + 48
    // ---- guess and walk this thread's segment
    const uint32_t lo = c0 + kPwSeg * (uint32_t)t, hi = lo + kPwSeg < c1 ? lo + kPwSeg : c1;
    bool has = false, fail = false;
    uint32_t g = 0, x = 0, k = 0;
    uint32_t ends[kPwRec];
    if (lo < hi && cur < hi) {
      if (cur >= lo) {
        g = cur;
        has = true;
      } else {
        // every position of the segment is a candidate whose records up to hi
        // and two more after them (inside the staged bytes, or to the end of
        // the stream) are valid; the one with the most records in the segment
        // wins (the true entry starts the longest run: a false start two or
        // three bytes before a record may jump onto the true chain, but only
        // after leaving the segment), then the nearest exit
        // 1. screen: the positions whose own length is valid, from two aligned
        //    LDS dwords per four positions (no dependent reads), as a bit mask
        uint32_t m0 = 0, m1 = 0, m2 = 0;  // bit i: position lo + i (i < kPwSeg <= 96)
        const uint32_t b_lo = (lo - c0 + off0) & ~3u, b_hi = hi - c0 + off0;
        for (uint32_t b4 = b_lo; b4 < b_hi; b4 += 4) {
          const uint32_t w0 = *(const PQG_L uint32_t*)(B + b4), w1 = *(const PQG_L uint32_t*)(B + b4 + 4);
#pragma unroll
          for (int kq = 0; kq < 4; kq++) {
            const uint32_t q = c0 - off0 + b4 + kq;
            const uint32_t l0 = kq ? __builtin_amdgcn_alignbit(w1, w0, 8 * kq) : w0;
            const bool ok = q >= lo && q < hi && n - q >= 4 && (int32_t)l0 >= 0 && n - q - 4 >= l0;
            const uint32_t i = q - lo;  // < 96 when ok
            const uint32_t bit = ok ? 1u << (i & 31) : 0u;
            m0 |= i < 32 ? bit : 0u;
            m1 |= i >= 32 && i < 64 ? bit : 0u;
            m2 |= i >= 64 ? bit : 0u;
          }
        }
        // 2. the candidates in order (a wave loops as often as its lane with
        //    the most candidates): every record up to hi and two more after
        //    them valid (inside the staged bytes, or to the end of the
        //    stream); the one with the most records in the segment wins (the
        //    true entry starts the longest run: a false start two or three
        //    bytes before a record may jump onto the true chain, but only
        //    after leaving the segment), then the nearest exit
        uint32_t best_k = 0, best_x = 0xffffffffu;
        while (m0 | m1 | m2) {
          const uint32_t i = m0 ? __builtin_ctz(m0) : m1 ? 32 + __builtin_ctz(m1) : 64 + __builtin_ctz(m2);
          if (i < 32) m0 &= m0 - 1;
          else if (i < 64) m1 &= m1 - 1;
          else m2 &= m2 - 1;
          const uint32_t q = lo + i;
          {
          uint32_t r = q, kk = 0, x = 0;  // x: this candidate's exit (its first record start >= hi)
          bool ok = true, xs = false;
          int extra = 0;
          while (ok && extra < 2) {
            if (!xs && r >= hi) {
              x = r;
              xs = true;
            }
            if (r == n) break;
            if (r >= c1 + kPwAhead) break;  // leaves the staged bytes: no further check
            if (n - r < 4) { ok = false; break; }
            const uint32_t l = len_at(r);
            if ((int32_t)l < 0 || n - r - 4 < l) { ok = false; break; }
            if (r < hi) kk++;
            else extra++;
            r += 4 + l;
          }
          if (!ok) continue;
          if (!xs) x = r;  // (r >= hi here: n and the staged end lie at or past hi)
          if (kk > best_k || (kk == best_k && x < best_x)) {
            best_k = kk;
            best_x = x;
            g = q;
            has = true;
          }
          }
        }
      }
      if (has) {
        uint32_t pos = g;
        while (pos < hi) {
          if (n - pos < 4) { fail = true; break; }
          const uint32_t l = len_at(pos);
          if ((int32_t)l < 0 || n - pos - 4 < l) { fail = true; break; }
          pos += 4 + l;
#pragma unroll
          for (int j = 0; j < kPwRec; j++)
            if ((uint32_t)j == k) ends[j] = pos;
          k++;
        }
        x = pos;
      }
    }
    // ---- check every guess at once: entry == exit of the nearest segment before with records
    PQG_T(tq2);
    PQG_ACC0(17, tq2 - tq1);
    sh.X[t] = x;
    int key = has ? t + 1 : 0;  // inclusive max-scan of the segments with records
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(key, o, 64);
      if (lane >= o) key = y > key ? y : key;
    }
    if (lane == 63) sh.keys[wv] = key;
    __syncthreads();
    int before = 0;
    for (int w = 0; w < wv; w++) before = sh.keys[w] > before ? sh.keys[w] : before;
    int ex = __shfl_up(key, 1, 64);
    if (lane == 0) ex = 0;
    ex = ex > before ? ex : before;               // nearest segment before t with records, + 1
    const uint32_t P = ex ? sh.X[ex - 1] : cur;  // the chain position entering segment t
    const bool bad = (lo < hi && cur < hi) && (has ? (g != P || fail) : P < hi);
    const int any_bad = __syncthreads_or(bad);
    if (!any_bad) {
      int64_t tot;
      const int64_t base = (int64_t)idx0 + block_excl_scan<kPwT>(has ? (int64_t)k : 0, &tot, sh.part);
#pragma unroll
      for (int j = 0; j < kPwRec; j++) {
        const int64_t i = base + j;
        if ((uint32_t)j < k && i < (int64_t)count) {
          out[i] = mode ? (int64_t)ends[j] : (int64_t)ends[j] - 4 * (i + 1);
          if (i == (int64_t)count - 1) sh.last_end = ends[j];
        }
      }
      // the last segment with records hands the chain on (the exit of the chunk)
      const int last = __shfl(key, 63, 64);  // this wave's; the block's is the max over waves
      int blast = 0;
      for (int w = 0; w < kPwT / 64; w++) blast = sh.keys[w] > blast ? sh.keys[w] : blast;
      (void)last;
      if (t == 0) {
        sh.idx = idx0 + (uint32_t)(tot < (int64_t)(count - idx0) ? tot : (int64_t)(count - idx0));
        if (blast) sh.cur = sh.X[blast - 1];
      }
    } else if (t == 0) {
      // the serial walk of the chunk's true chain (exact errors: reference order)
      PQG_ACC0(20, 1);
      uint32_t pos = cur, i = idx0;
      int st = kOK;
      while (pos < c1 && i < count) {
        if (n - pos < 4) { st = kEOF; break; }
        const uint32_t l = len_at(pos);
        if ((int32_t)l < 0) { st = kBYTE_ARRAY; break; }
        if (n - pos - 4 < l) { st = kEOF; break; }
        pos += 4 + l;
        out[i] = mode ? (int64_t)pos : (int64_t)pos - 4 * ((int64_t)i + 1);
        if (i == count - 1) sh.last_end = pos;
        i++;
      }
      sh.cur = pos;
      sh.idx = i;
      sh.status = st;
    }
    __syncthreads();
    PQG_T(tq3);
    PQG_ACC0(18, tq3 - tq2);
    if (sh.status != kOK) return sh.status;
  }
  __syncthreads();
  if (sh.idx < count) return kEOF;  // the stream ends before record `idx`
  *chars = count ? (int64_t)sh.last_end - 4 * (int64_t)count : 0;
  return kOK;
}

// ---------------------------------------------------------------------------
// Dictionary pages (k_str_dict: one block per chunk, so the whole page's
// parallelism must come from one block): the page is cut into 512 segments
// walked at once through 64-byte register windows from global memory (a
// two-guess start per segment, thread 0 chains the guesses, a second pass
// writes), instead of block_walk's 32 KiB chunks one after another.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t pick4(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) {
  return (k & 2) ? ((k & 1) ? d : c) : ((k & 1) ? b : a);
}

// Walk records from `pos` while pos < stop and fewer than `limit` records are
// done.  Returns the records walked; *end = the position after them, *fail = 1
// when the record at *end is not valid (length negative or past n, or fewer
// than 4 bytes left).  sink(k, pos_after) sees record k of the walk.
template <class F>
__device__ __forceinline__ uint32_t seg_walk(gcu8 p, uint32_t n, uint32_t pos, uint32_t stop, uint32_t limit,
                                             uint32_t* end, int* fail, F&& sink) {
  uintptr_t wb = 0;
  uint4 g0 = make_uint4(0, 0, 0, 0), g1 = g0, g2 = g0, g3 = g0;
  const uintptr_t pend = (uintptr_t)(p + n);
  uint32_t k = 0;
  *fail = 0;
  while (pos < stop && k < limit) {
    if (n - pos < 4) { *fail = 1; break; }
    const uintptr_t a = (uintptr_t)(p + pos);
    if (a < wb || a + 4 > wb + 64) {
      wb = a & ~(uintptr_t)15;
      // four loads issued together, unconditionally (a guarded load would be
      // waited for at its branch join): granules past the stream's last one
      // re-read that one, their bytes are never used
      const uintptr_t lastg = (pend - 1) & ~(uintptr_t)15;
      g0 = ldg16(wb);
      g1 = ldg16(wb + 16 < lastg ? wb + 16 : lastg);
      g2 = ldg16(wb + 32 < lastg ? wb + 32 : lastg);
      g3 = ldg16(wb + 48 < lastg ? wb + 48 : lastg);
    }
    const uint32_t off = (uint32_t)(a - wb), d = off >> 2, e = d + 1 < 16 ? d + 1 : 15;
    const uint32_t lo = pick4(pick4(g0.x, g0.y, g0.z, g0.w, d), pick4(g1.x, g1.y, g1.z, g1.w, d),
                              pick4(g2.x, g2.y, g2.z, g2.w, d), pick4(g3.x, g3.y, g3.z, g3.w, d), d >> 2);
    const uint32_t hi = pick4(pick4(g0.x, g0.y, g0.z, g0.w, e), pick4(g1.x, g1.y, g1.z, g1.w, e),
                              pick4(g2.x, g2.y, g2.z, g2.w, e), pick4(g3.x, g3.y, g3.z, g3.w, e), e >> 2);
    const uint32_t l = __builtin_amdgcn_alignbit(hi, lo, (off & 3) * 8);
    if ((int32_t)l < 0 || n - pos - 4 < l) { *fail = 1; break; }
    pos += 4 + l;
    sink(k, pos);
    k++;
  }
  *end = pos;
  return k;
}

struct BlockWalkSharedG {
  uint32_t start[kWalkT];  // pass A: first guessed start (0xffffffff: none); pass B: verified start
  uint32_t exit_[kWalkT];  // position after the segment's records
  uint32_t cnt[kWalkT];    // records walked
  uint32_t start2[kWalkT], exit2[kWalkT], cnt2[kWalkT];  // the second guess
  uint32_t base[kWalkT];   // pass B: index of the segment's first record (0xffffffff: segment unused)
  uint8_t fail[kWalkT], fail2[kWalkT];
  uint32_t last_end;       // end of record count-1
  int status;
};

// byteArrayPlainDecoder.next for records [0, count) of [p, p+n), the whole
// block.  mode 0 (data page): out[i] = char end of value i = end(i) - 4 (i + 1);
// mode 1 (dictionary page): out[i] = end(i), the next record's start.
// Returns the status (all threads); *chars = sum of the lengths.
__device__ int block_walk_g(gcu8 p, uint32_t n, uint32_t count, PQG_G int64_t* out, int mode, int64_t* chars,
                            BlockWalkSharedG& sh) {
  const int t = threadIdx.x;
  const uint32_t L = ((n + kWalkT - 1) / kWalkT + 63) & ~63u;  // segment bytes (>= 64)
  const uint32_t lo = (uint32_t)t * L < n ? (uint32_t)t * L : n;
  const uint32_t hi = lo + L < n ? lo + L : n;
  const uint32_t kNone = 0xffffffffu;
  auto nop = [](uint32_t, uint32_t) {};
  PQG_T(tp0);
  // ---- pass A: guess two starts, walk the segment from each
  // (a false start is typically the byte before a record — [c, len, 0, 0] reads
  // as a short length — so the next candidate is usually the true record)
  if (count > 0) {
    uint32_t st = kNone, st2 = kNone;
    if (t == 0) {
      st = 0;
    } else {
      // positions whose length chain is valid for three records; a candidate
      // is first screened on its own length (one 64-byte window load per 60
      // positions), the deeper check walks from it
      uintptr_t wb = 0;
      uint4 g0 = make_uint4(0, 0, 0, 0), g1 = g0, g2 = g0, g3 = g0;
      const uintptr_t pend = (uintptr_t)(p + n), lastg = (pend - 1) & ~(uintptr_t)15;
      for (uint32_t q = lo; q < hi && n - q >= 4; q++) {
        if (st != kNone && q > st + 64) break;
        const uintptr_t a = (uintptr_t)(p + q);
        if (a + 4 > wb + 64) {
          wb = a & ~(uintptr_t)15;
          g0 = ldg16(wb);
          g1 = ldg16(wb + 16 < lastg ? wb + 16 : lastg);
          g2 = ldg16(wb + 32 < lastg ? wb + 32 : lastg);
          g3 = ldg16(wb + 48 < lastg ? wb + 48 : lastg);
        }
        const uint32_t off = (uint32_t)(a - wb), d = off >> 2, e1 = d + 1 < 16 ? d + 1 : 15;
        const uint32_t w0 = pick4(pick4(g0.x, g0.y, g0.z, g0.w, d), pick4(g1.x, g1.y, g1.z, g1.w, d),
                                  pick4(g2.x, g2.y, g2.z, g2.w, d), pick4(g3.x, g3.y, g3.z, g3.w, d), d >> 2);
        const uint32_t w1 = pick4(pick4(g0.x, g0.y, g0.z, g0.w, e1), pick4(g1.x, g1.y, g1.z, g1.w, e1),
                                  pick4(g2.x, g2.y, g2.z, g2.w, e1), pick4(g3.x, g3.y, g3.z, g3.w, e1), e1 >> 2);
        const uint32_t l = __builtin_amdgcn_alignbit(w1, w0, (off & 3) * 8);
        if ((int32_t)l < 0 || n - q - 4 < l) continue;
        uint32_t e;
        int f;
        const uint32_t k = seg_walk(p, n, q, n, 3, &e, &f, nop);
        if (k == 3 || (f && e == n)) {
          if (st == kNone) {
            st = q;
          } else {
            st2 = q;
            break;
          }
        }
      }
    }
    sh.start[t] = st;
    sh.start2[t] = st2;
    sh.fail[t] = sh.fail2[t] = 0;
    sh.cnt[t] = sh.cnt2[t] = 0;
    sh.exit_[t] = st;
    sh.exit2[t] = st2;
    uint32_t e;
    int f;
    if (st != kNone && st < hi) {
      sh.cnt[t] = seg_walk(p, n, st, hi, 0xffffffffu, &e, &f, nop);
      sh.exit_[t] = e;
      sh.fail[t] = (uint8_t)f;
    }
    if (st2 != kNone && st2 < hi) {
      sh.cnt2[t] = seg_walk(p, n, st2, hi, 0xffffffffu, &e, &f, nop);
      sh.exit2[t] = e;
      sh.fail2[t] = (uint8_t)f;
    }
  }
  __syncthreads();
  PQG_T(tp1);
  // ---- thread 0: follow the true chain through the segments
  if (t == 0) {
    uint32_t redo = 0, redo_k = 0;
    (void)redo;
    (void)redo_k;
    for (int s = 0; s < kWalkT; s++) sh.base[s] = kNone;
    uint32_t cur = 0, idx = 0;
    int status = kOK;
    bool failed = false;
    for (int s = 0; s < kWalkT && idx < count; s++) {
      const uint32_t slo = (uint32_t)s * L < n ? (uint32_t)s * L : n;
      const uint32_t shi = slo + L < n ? slo + L : n;
      if (shi <= slo) break;     // past the end of the stream
      if (cur >= shi) continue;  // a record spans the whole segment
      uint32_t k, e;
      int f;
      if (sh.start[s] == cur) {  // a guess was right: take the segment's walk
        k = sh.cnt[s];
        e = sh.exit_[s];
        f = sh.fail[s];
      } else if (sh.start2[s] == cur) {
        k = sh.cnt2[s];
        e = sh.exit2[s];
        f = sh.fail2[s];
      } else {
        k = seg_walk(p, n, cur, shi, 0xffffffffu, &e, &f, nop);
        redo++;
        redo_k += k;
      }
      sh.start[s] = cur;
      sh.base[s] = idx;
      idx += k;
      cur = e;
      if (f) {
        failed = true;
        break;
      }
    }
    if (idx < count) {
      // record `idx` at `cur` fails: fewer than 4 bytes (EOF), a negative
      // length, or fewer bytes than its length (EOF)
      status = kEOF;
      if (failed && n - cur >= 4) {
        const uint32_t l = (uint32_t)p[cur] | (uint32_t)p[cur + 1] << 8 | (uint32_t)p[cur + 2] << 16 |
                           (uint32_t)p[cur + 3] << 24;
        if ((int32_t)l < 0) status = kBYTE_ARRAY;
      }
    }
    sh.status = status;
    sh.last_end = 0;
    PQG_ACC0(28, redo);
    PQG_ACC0(29, redo_k);
  }
  __syncthreads();
  PQG_T(tp2);
  const int status = sh.status;
  if (status != kOK) return status;
  // ---- pass B: outputs from the verified starts
  if (count > 0 && sh.base[t] != kNone && sh.base[t] < count) {
    const uint32_t b = sh.base[t];
    uint32_t e;
    int f;
    seg_walk(p, n, sh.start[t], hi, count - b, &e, &f,
             [&](uint32_t k, uint32_t pos) {
               const uint32_t i = b + k;
               out[i] = mode ? (int64_t)pos : (int64_t)pos - 4 * ((int64_t)i + 1);
               if (i == count - 1) sh.last_end = pos;
             });
  }
  __syncthreads();
  PQG_T(tp3);
#ifdef PQG_PROFILE
  PQG_ACC0(24, tp1 - tp0);
  PQG_ACC0(25, tp2 - tp1);
  PQG_ACC0(26, tp3 - tp2);
  PQG_ACC0(27, 1);
#endif
  *chars = count ? (int64_t)sh.last_end - 4 * (int64_t)count : 0;
  return kOK;
}

// ---- K7a ---------------------------------------------------------------------
__global__ void __launch_bounds__(kWalkT) k_str_dict(JobDev* jobs, PageDev* pages, int64_t* doffs_arena) {
  __shared__ BlockWalkSharedG sh;
  JobDev& job = jobs[blockIdx.x];
  if (job.status == kCAPACITY || !(job.flags & 2) || job.dict_page < 0) return;
  PageDev& dp = pages[job.page_base + job.dict_page];
  if (dp.read_status != kOK) return;
  const int64_t cnt = dp.num_values;
  PQG_G int64_t* doffs = gmut(doffs_arena) + job.doffs_base;
  int64_t chars;
  const int st = block_walk_g(gconst(job.dict_data), (uint32_t)job.dict_len, (uint32_t)cnt, doffs + 1, 1, &chars, sh);
  if (threadIdx.x == 0) {
    if (st == kOK) {
      doffs[0] = 0;
      job.dict_offs = (const int64_t*)doffs;
      job.dict_count = cnt;
    } else {
      dp.read_status = st;  // dictPageReader.read: any error is fatal (page_dict.go:50-56)
    }
  }
}

// ---- K7b (PLAIN) -------------------------------------------------------------
#ifndef PQG_PW_WPE
#define PQG_PW_WPE 4
#endif
__global__ void __attribute__((amdgpu_flat_work_group_size(1, kPwT), amdgpu_waves_per_eu(PQG_PW_WPE))) k_str_plain(JobDev* jobs, PageDev* pages, const int* list, const int* total,
                                                      int* queue, int64_t* offs_arena) {
  __shared__ BlockWalkShared sh;
  __shared__ int s_t;
  for (;;) {
    if (threadIdx.x == 0) s_t = queue_pull(queue);
    __syncthreads();
    const int t = s_t;
    __syncthreads();
    if (t >= *total) return;
    const int pidx = list[t];
    const PageDev& pg = pages[pidx];
    if (pg.read_status != kOK || pg.decode_status != kOK || (pg.page_type != 0 && pg.page_type != 3) || pg.vmode != 2 ||
        pg.encoding != 0 || pg.not_null == 0)
      continue;
    const JobDev& job = jobs[pg.job];
    if (job.status == kCAPACITY) continue;
    int64_t chars;
    const int de = block_walk(gconst(pg.val), (uint32_t)pg.val_n, (uint32_t)pg.not_null,
                              gmut(offs_arena) + job.offs_base + pg.value_offset + 1, 0, &chars, sh);
    if (threadIdx.x == 0) {
      pages[pidx].chars = de == kOK ? chars : 0;
      if (de != kOK) pages[pidx].decode_status = de;
    }
  }
}

// ---- dictionary sinks (type_dict.go:39-59 over variable-length entries) ------
// Sums the entry lengths of the keys and parks each key in its value's
// offsets slot (k_str_copy turns it into the value's end).
struct StrDictCount {
  const PQG_G int64_t* doffs;
  PQG_G int64_t* keys;  // chunk offsets + value_offset + 1
  int64_t count;
  int64_t bad;   // first value index with an invalid key
  int64_t sum;   // lane's chars
  __device__ __forceinline__ void prepare(const uint32_t (&)[kGroup][8], const uint32_t (&)[kGroup], const int (&)[kGroup]) {}
  // every entry-offset gather of the group is issued first, unconditionally
  // (a key past the dictionary or a value past cnt reads entry 0), then the
  // keys are parked and the lengths summed: one round trip per group instead
  // of one per value (a guarded load is waited for inside its branch, and a
  // load issued after the key stores would wait for them)
  __device__ __forceinline__ void group(const uint32_t (&v)[kGroup][8], const uint32_t (&i0)[kGroup],
                                        const int (&cnt)[kGroup]) {
    int64_t a[kGroup][8], c[kGroup][8];
#pragma unroll
    for (int b = 0; b < kGroup; b++)
#pragma unroll
      for (int q = 0; q < 8; q++) {
        const uint32_t key = v[b][q];
        const uint32_t kc = (q < cnt[b] && (int64_t)key < count) ? key : 0u;
        a[b][q] = doffs[kc];
        c[b][q] = doffs[kc + 1];
      }
#pragma unroll
    for (int b = 0; b < kGroup; b++)
#pragma unroll
      for (int q = 0; q < 8; q++) {
        if (q >= cnt[b]) continue;
        const uint32_t key = v[b][q];
        keys[i0[b] + q] = key;
        if ((int64_t)key < count) sum += c[b][q] - a[b][q] - 4;
        else if ((int64_t)(i0[b] + q) < bad) bad = (int64_t)(i0[b] + q);
      }
  }
};

// copy `len` bytes (any alignment); source dwords are read aligned, so no
// byte outside the source's dwords is touched
__device__ __forceinline__ void copy_bytes(gu8 dst, gcu8 src, int64_t len) {
  int64_t k = 0;
  for (; k + 4 <= len; k += 4) {
    const uintptr_t a = (uintptr_t)(src + k);
    const PQG_G uint32_t* q = (const PQG_G uint32_t*)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3) * 8;
    const uint32_t x = sh ? __builtin_amdgcn_alignbit(q[1], q[0], sh) : q[0];
    gu8 o = dst + k;
    if (((uintptr_t)o & 3) == 0) {
      *(PQG_G uint32_t*)o = x;
    } else {
      o[0] = (uint8_t)x;
      o[1] = (uint8_t)(x >> 8);
      o[2] = (uint8_t)(x >> 16);
      o[3] = (uint8_t)(x >> 24);
    }
  }
  for (; k < len; k++) dst[k] = src[k];
}

// ---- K7b ---------------------------------------------------------------------
// Work items are the pages' parts (k_part_plan): a big dictionary page is
// counted by many waves, each over its blocks; the part's chars go to its
// PartRec (k_char_scan scans them).
__global__ void __launch_bounds__(64) k_str_count(JobDev* jobs, PageDev* pages, PartRec* parts, const int* total,
                                                  int* queue, int64_t* offs_arena, const HStream* streams,
                                                  const RunEnt* runs, const BlockDesc* blks) {
  __shared__ __attribute__((aligned(16))) ExpandShared sh;
  const int lane = lane_id();
  const int n_items = min(total[kCtrItems], total[kCtrPartsCap]);
  for (;;) {
    const int t = queue_next(queue);
    if (t >= n_items) return;
    const PartRec pr = parts[t];
    if (pr.vmode != 2) continue;
    const int pidx = __builtin_amdgcn_readfirstlane(pr.pidx);
    const PageDev pg = pages[pidx];
    if (pg.read_status != kOK || (pg.page_type != 0 && pg.page_type != 3) || pg.vmode != 2) continue;
    const JobDev job = jobs[pg.job];
    if (job.status == kCAPACITY) continue;
    const int enc = pg.encoding;
    const gcu8 val = gconst(pg.val);
    const int64_t vn = pg.val_n;
    const int64_t nn = pg.not_null;
    // valuesDecoder.init (read phase): the dictionary decoder reads its width byte
    if (enc == 8) {
      int re = kOK;
      if (vn < 1) re = kEOF;
      else if (val[0] > 32) re = kBIT_WIDTH;
      if (re != kOK) {
        if (lane == 0) pages[pidx].read_status = re;
        continue;
      }
    }
    if (pg.decode_status != kOK || nn == 0) continue;
    int de = kOK;
    int64_t chars = 0;
    if (enc == 0) {
      continue;  // PLAIN: k_str_plain
    } else if (enc == 8) {
      const int64_t dcount = job.dict_offs ? job.dict_count : 0;
      const int dw = pg.dict_width;
      PQG_G int64_t* keys = gmut(offs_arena) + job.offs_base + pg.value_offset + 1;
      if (dw == 0) {
        // zero-width indices: key 0 forever (hybrid_decoder.go:84-86)
        if (dcount < 1) de = kDICT_INDEX;
        else {
          chars = nn * (gconst(job.dict_offs)[1] - 4);
          for (int64_t i = lane; i < nn; i += 64) keys[i] = 0;
        }
      } else {
        const HStream S = streams[pg.hs_val];
        const int serr = (S.status != kOK && S.produced < nn) ? S.status : kOK;
        const bool last = pr.p + 1 >= pr.np;
        const int64_t v_hi = last ? nn : (int64_t)parts[t + 1].v0;
        StrDictCount sk{gconst(job.dict_offs ? job.dict_offs : (const int64_t*)offs_arena), keys, dcount, nn, 0};
        hybrid_expand(S, runs, blks, v_hi, sh, sk, pr.b0, last ? -1 : parts[t + 1].b0);
        const int64_t bad = wave_min(sk.bad);
        chars = wave_sum(sk.sum);
        if (bad < nn && (serr == kOK || bad < S.produced)) de = kDICT_INDEX;
        else de = serr;
      }
    } else if (enc == 6 || enc == 7) {
      continue;  // DELTA_LENGTH_BYTE_ARRAY / DELTA_BYTE_ARRAY: k_str_delta
    } else {
      de = kUNSUPPORTED;
    }
    if (lane == 0) {
      parts[t].chars = chars;
      if (de != kOK) atomicMin(&pages[pidx].decode_status, de);  // parts of a page: kDICT_INDEX wins
    }
  }
}

// ---- K7e: DELTA_LENGTH_BYTE_ARRAY / DELTA_BYTE_ARRAY lengths -------------------
// deltaBitPackDecoder32 (deltabp_decoder.go:38-175) walked exactly as
// decodeInt32 (helpers.go:119-129) drives it from byteArrayDeltaLengthDecoder /
// byteArrayDeltaDecoder.init (type_bytearray.go:103-111, 194-212): every one of
// the header's valuesCount values, 8 at a time (a group is read when position %
// 8 == 0, a miniblock header when a block's miniblocks are used up; the last
// group skips the rest of the block with the sic width of miniBlockBitWidth
// [currentMiniBlock]).  The stream is read through an LDS window; lanes 0..7
// unpack a group's 8 deltas, and a DPP prefix sum turns them into values.
struct DbpWalk32 {
  Window win;
  int64_t r;           // reader position (stream offset)
  int32_t bs, mbc, total, mbvc;
  int32_t prev, mind;
  int64_t wpos;        // stream offset of the current block's width bytes
  int32_t cur, mbpos, cw;
  int32_t position;

  __device__ int init(gcu8 p, int64_t n, PQG_L uint8_t* lds, int64_t start) {
    win = Window{p, n, kFarAway, lds};
    r = start;
    int e;
    uint64_t first;
    if ((e = read_u32var_delta(win, r, &bs))) return e;
    if (bs <= 0 && bs % 128 != 0) return kDELTA;
    if ((e = read_u32var_delta(win, r, &mbc))) return e;
    if (mbc <= 0 || bs % mbc != 0) return kDELTA;
    mbvc = bs / mbc;
    if (mbvc == 0) return kDELTA;
    if ((e = read_u32var_delta(win, r, &total))) return e;
    if ((e = read_signed(win, r, false, &first))) return e;
    prev = (int32_t)first;
    position = 0;
    return mini_header();
  }
  // readMiniBlockHeader :89-112
  __device__ int mini_header() {
    uint64_t md;
    int e = read_signed(win, r, false, &md);
    if (e) return e;
    mind = (int32_t)md;
    if (win.n - r < mbc) {  // io.ReadFull of the widths
      r = win.n;
      return kEOF;
    }
    wpos = r;
    for (int32_t m = 0; m < mbc; m++)
      if (win.get(r + m) > 32) return kBIT_WIDTH;
    r += mbc;
    cur = 0;
    return kOK;
  }
  // next() for positions [position, position + 8) (those < total): lane j < 8
  // gets the value of position + j in *v.  kOK or the error of the group.
  __device__ int group(int32_t* v) {
    const int lane = lane_id();
    if (position % mbvc == 0) {
      if (cur >= mbc) {
        const int e = mini_header();
        if (e) return e;
      }
      cw = win.get(wpos + cur);
      mbpos = 0;
      cur++;
    }
    if (win.n - r < cw) {  // io.ReadFull of the group
      r = win.n;
      return kEOF;
    }
    // the group's bytes into the window, then lane j < 8 unpacks delta j
    if (cw > 0 && (r < win.base || r + cw > win.base + kWin)) win.fill(r);
    uint32_t d = 0;
    if (cw > 0 && lane < 8) {
      const int64_t b0 = (int64_t)lane * cw;  // bit of delta j in the group
      const PQG_L uint8_t* g = win.lds + (r - win.base);
      uint64_t x = 0;
      for (int k = 0; k < 5; k++) {
        const int64_t by = (b0 >> 3) + k;
        if (by < cw) x |= (uint64_t)g[by] << (8 * k);
      }
      x >>= (b0 & 7);
      d = (uint32_t)(cw == 32 ? x : (x & ((1ull << cw) - 1)));
    }
    r += cw;
    mbpos += cw;
    if ((int64_t)position + 8 >= total) {
      const int64_t l = (int64_t)(mbvc / 8) * cw - mbpos;
      if (l < 0) return kDELTA;  // "invalid stream"
      r = r + l < win.n ? r + l : win.n;  // errors ignored
      if (cur < mbc) {
        const int w2 = win.get(wpos + cur);  // sic: miniBlockBitWidth[currentMiniBlock]
        if (w2 != 0) {
          const int64_t skip = (int64_t)(mbc - cur) * (int64_t)(mbvc / 8) * w2;
          r = r + skip < win.n ? r + skip : win.n;
        }
      }
    }
    // value(position + j) = prev + sum_{k < j} (delta_k + mind), int32 wrapping
    const uint32_t step = (lane < 8) ? d + (uint32_t)mind : 0u;
    uint32_t incl = step;
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) {
      const uint32_t t = __shfl_up(incl, o, 64);
      if ((lane & 7) >= o) incl += t;
    }
    *v = (int32_t)((uint32_t)prev + incl - step);
    prev = (int32_t)((uint32_t)prev + (uint32_t)__shfl(incl, 7, 64));
    position += 8;
    return kOK;
  }
  // group() for every remaining position (position .. total), without the
  // values: the reader ends where those calls would leave it, with their
  // errors.  One step per run of groups inside one miniblock (a miniblock
  // starts at a group start that is a multiple of mbvc), so the work is
  // bounded by the stream's bytes (every miniblock has a width byte), not by
  // the header's count (the oracle's DeltaBP::skip_rest).  Wave-uniform.
  __device__ int skip_rest() {
    const int64_t L = (int64_t)mbvc / gcd8(mbvc) * 8;  // lcm(8, mbvc)
    const int64_t last = ((int64_t)total - 1) / 8 * 8;  // the group holding the last value
    while (position < total) {
      if (position % mbvc == 0) {
        if (cur >= mbc) {
          const int e = mini_header();
          if (e) return e;
        }
        cw = win.get(wpos + cur);
        mbpos = 0;
        cur++;
      }
      const int64_t next_start = ((int64_t)position / L + 1) * L;
      const bool tail = last < next_start;
      const int64_t g = tail ? (last - position) / 8 + 1 : (next_start - position) / 8;
      if (win.n - r < g * cw) {  // io.ReadFull of a group
        r = win.n;
        return kEOF;
      }
      r += g * cw;
      mbpos = (int32_t)((uint32_t)mbpos + (uint32_t)(g * cw));
      if (!tail) {
        position = (int32_t)next_start;
        continue;
      }
      const int64_t l = (int64_t)(mbvc / 8) * cw - mbpos;
      if (l < 0) return kDELTA;  // "invalid stream"
      r = r + l < win.n ? r + l : win.n;  // errors ignored
      if (cur < mbc) {
        const int w2 = win.get(wpos + cur);  // sic: miniBlockBitWidth[currentMiniBlock]
        if (w2 != 0) {
          const int64_t skip = (int64_t)(mbc - cur) * (int64_t)(mbvc / 8) * w2;
          r = r + skip < win.n ? r + skip : win.n;
        }
      }
      position = total;
    }
    return kOK;
  }
  __device__ static int64_t gcd8(int32_t v) {
    int64_t a = v, b = 8;
    while (b) {
      const int64_t t = a % b;
      a = b;
      b = t;
    }
    return a;
  }
};

// One wave per DELTA_LENGTH_BYTE_ARRAY / DELTA_BYTE_ARRAY page: the read phase
// (every length decoded, the prefix/suffix count check) and the lengths of the
// page's notNull values: page-relative value ends (DLBA) or, for
// DELTA_BYTE_ARRAY, prefix << 32 | suffix end, in the chunk's offsets (K7f /
// k_str_copy turn them into chunk offsets); page.chars, page.cstart.  The
// first failing value, in order, is the page's decode error
// (byteArrayDeltaLengthDecoder.next :113-126; byteArrayDeltaDecoder
// .decodeValues :214-240).
struct DeltaStrShared {
  uint8_t win[2][kWin];
};
__global__ void __launch_bounds__(64) k_str_delta(JobDev* jobs, PageDev* pages, const int* list, const int* total,
                                                  int* queue, int64_t* offs_arena) {
  __shared__ __attribute__((aligned(16))) DeltaStrShared sh;
  const int lane = lane_id();
  if (total[kModePresentOff + 4] == 0) return;  // no DELTA_*_BYTE_ARRAY page
  for (;;) {
    const int t = queue_next(queue);
    if (t >= *total) return;
    const int pidx = __builtin_amdgcn_readfirstlane(list[t]);
    const PageDev pg = pages[pidx];
    if (pg.read_status != kOK || (pg.page_type != 0 && pg.page_type != 3) || pg.vmode != 2 ||
        (pg.encoding != 6 && pg.encoding != 7))
      continue;
    const JobDev job = jobs[pg.job];
    if (job.status == kCAPACITY) continue;
    const bool dba = pg.encoding == 7;
    const gcu8 val = gconst(pg.val);
    const int64_t vn = pg.val_n;
    const int64_t nn = pg.decode_status == kOK ? pg.not_null : 0;
    // ---- read phase: lengths (DBA: prefixes, then suffix lengths)
    DbpWalk32 A, B;  // A: prefix lengths (DBA) / lengths; B: suffix lengths (DBA)
    // every length of the header's count is read (type_bytearray.go:104-113,
    // 195-207); those past the page's NumValues are never used, so they are
    // walked by miniblock (skip_rest: work bounded by the stream's bytes)
    int re = A.init(val, vn, lds_ptr(sh.win[0]), 0);
    int64_t a_end = 0;
    if (re == kOK) {
      const int32_t keep = A.total < pg.num_values ? A.total : pg.num_values;
      for (int32_t p = 0; p < keep && re == kOK; p += 8) {
        int32_t v;
        re = A.group(&v);
      }
      if (re == kOK) re = A.skip_rest();
      a_end = A.r;
    }
    if (re == kOK && dba) {
      re = B.init(val, vn, lds_ptr(sh.win[1]), a_end);
      if (re == kOK) {
        const int32_t keep = B.total < pg.num_values ? B.total : pg.num_values;
        for (int32_t p = 0; p < keep && re == kOK; p += 8) {
          int32_t v;
          re = B.group(&v);
        }
        if (re == kOK) re = B.skip_rest();
      }
      if (re == kOK && A.total != B.total) re = kDELTA;  // "different number of suffixes and prefixes"
    }
    if (re != kOK) {
      if (lane == 0) pages[pidx].read_status = re;
      continue;
    }
    if (nn == 0) continue;
    // ---- decodeValues over the notNull values: walk the length stream(s)
    // again, 8 values at a time, checking each value in order
    const int64_t cs = dba ? B.r : A.r;  // the value bytes start where the lengths end
    const int32_t cnt = dba ? B.total : A.total;
    PQG_G int64_t* slots = gmut(offs_arena) + job.offs_base + pg.value_offset + 1;
    int e = A.init(val, vn, lds_ptr(sh.win[0]), 0);
    if (dba) e = B.init(val, vn, lds_ptr(sh.win[1]), a_end);
    (void)e;
    int64_t bad = INT64_MAX;  // first failing value
    int bad_e = kOK;
    int64_t send = 0;         // suffix / value bytes so far
    int64_t chars = 0;        // output bytes so far
    int64_t prevlen = 0;      // DBA: length of the previous value
    for (int64_t i0 = 0; i0 < nn; i0 += 8) {
      if (i0 >= cnt) {  // next(): position >= len(lens) -> io.EOF
        if (i0 < bad) { bad = i0; bad_e = kEOF; }
        break;
      }
      int32_t pl = 0, sl = 0;
      if (dba) {
        A.group(&pl);
        B.group(&sl);
      } else {
        A.group(&sl);
      }
      const int64_t i = i0 + lane;
      const bool live = lane < 8 && i < nn;
      // per value, in the reference's order: position, negative length, short
      // read, (DBA) capacity, previous-value length
      int ve = kOK;
      int64_t my_send = 0, my_len = 0;
      {
        const int64_t s64 = (live && i < cnt && sl > 0) ? sl : 0;
        int64_t incl = s64;
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) {
          const int64_t tt = __shfl_up(incl, o, 64);
          if ((lane & 7) >= o) incl += tt;
        }
        my_send = send + incl;
        // (lanes past the values read the streams' miniblock padding: no bytes)
        const int64_t eff_pl = live && i < cnt && dba && pl > 0 ? pl : 0;
        my_len = eff_pl + s64;
        int64_t li = my_len;
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) {
          const int64_t tt = __shfl_up(li, o, 64);
          if ((lane & 7) >= o) li += tt;
        }
        int64_t prev_l = __shfl_up(my_len, 1, 64);
        if (lane == 0) prev_l = prevlen;
        if (live) {
          if (i >= cnt) ve = kEOF;
          else if (sl < 0) ve = kBYTE_ARRAY;                     // make([]byte, negative)
          else if (cs + my_send > vn) ve = kEOF;                 // io.ReadFull: "there is no byte left"
          else if (dba && (int64_t)pl + sl < 0) ve = kBYTE_ARRAY; // negative capacity
          else if (dba && prev_l < (int64_t)pl) ve = kBYTE_ARRAY; // "invalid prefix len in the stream"
          else if (job.value_width > 0 && my_len != job.value_width) ve = kFIXED_LEN;  // FLBA: DESIGN.md
        }
        if (live && ve == kOK)
          slots[i] = dba ? (int64_t)(((uint64_t)eff_pl << 32) | (uint64_t)(uint32_t)my_send) : my_send;
        const int64_t tot_s = __shfl(incl, 7, 64), tot_l = __shfl(li, 7, 64);
        send += tot_s;
        chars += tot_l;
        prevlen = __shfl(my_len, 7, 64);
      }
      const uint64_t eb = __ballot(ve != kOK);
      if (eb) {
        const int l = __ffsll((long long)eb) - 1;
        bad = i0 + l;
        bad_e = __builtin_amdgcn_readlane(ve, l);
        break;
      }
    }
    if (lane == 0) {
      PageDev& o = pages[pidx];
      o.cstart = cs;
      o.chars = bad_e == kOK ? chars : 0;
      if (bad_e != kOK) o.decode_status = bad_e;
    }
  }
}

// ---- K7f: DELTA_BYTE_ARRAY values ----------------------------------------------
// value i = value(i - 1)[:prefix_i] + suffix_i (type_bytearray.go:214-240): one
// wave per page, values in order.  The previous value stays in LDS (values up
// to kDbaPrev bytes; a longer one is rebuilt from the output it was written
// to), each group's 64 suffixes are staged into LDS with one round of loads,
// and each value is assembled in LDS and stored, 64 bytes per lane step.
constexpr int kDbaPrev = 16384;
constexpr int kDbaStage = 8192;
struct DbaShared {
  uint8_t prev[kDbaPrev];
  uint8_t stage[kDbaStage + 64];
};
__global__ void __launch_bounds__(64) k_str_dba(JobDev* jobs, PageDev* pages, const int* list, const int* total,
                                                int* queue, uint8_t* value_arena, int64_t* offs_arena) {
  __shared__ __attribute__((aligned(16))) DbaShared sh;
  const int lane = lane_id();
  if (total[kModePresentOff + 4] == 0) return;
  for (;;) {
    const int t = queue_next(queue);
    if (t >= *total) return;
    const int pidx = __builtin_amdgcn_readfirstlane(list[t]);
    const PageDev pg = pages[pidx];
    if (pg.read_status != kOK || pg.decode_status != kOK || (pg.page_type != 0 && pg.page_type != 3) ||
        pg.vmode != 2 || pg.encoding != 7 || pg.not_null == 0)
      continue;
    const JobDev job = jobs[pg.job];
    if (job.status == kCAPACITY) continue;
    // FLBA (fixed width): value i at (value_offset + i) * type_length, no offsets out
    const bool fixed = job.value_width > 0;
    const int64_t nn = pg.not_null, base = fixed ? pg.value_offset * job.value_width : pg.char_offset;
    const gu8 chars = gmut(value_arena) + job.value_base + base;
    PQG_G int64_t* slots = gmut(offs_arena) + job.offs_base + pg.value_offset + 1;
    const gcu8 suf = gconst(pg.val) + pg.cstart;
    int64_t oend = 0, sprev = 0;  // output end, suffix start of the next value
    int64_t plen = 0;             // length of the previous value
    bool in_lds = true;           // the previous value is in sh.prev
    int64_t pstart = 0;           // its output offset (page-relative)
    for (int64_t i0 = 0; i0 < nn; i0 += 64) {
      const int64_t i = i0 + lane;
      int64_t pl = 0, se = sprev;
      if (i < nn) {
        const uint64_t x = (uint64_t)slots[i];
        pl = (int64_t)(x >> 32);
        se = (int64_t)(uint32_t)x;
      }
      int64_t ss = __shfl_up(se, 1, 64);
      if (lane == 0) ss = sprev;
      const int64_t len = i < nn ? pl + (se - ss) : 0;
      int64_t incl;
      const int64_t ex = wave_excl_scan_i64(len, &incl);
      const int64_t ostart = oend + ex;
      if (i < nn && !fixed) slots[i] = base + ostart + len;
      const int nv = (int)(nn - i0 < 64 ? nn - i0 : 64);
      const int64_t g_ss = sprev, g_se = __shfl(se, nv - 1, 64);
      // the group's suffixes into LDS (when they fit)
      const bool staged = g_se - g_ss <= kDbaStage;
      if (staged)
        for (int64_t b = lane; b < g_se - g_ss; b += 64) sh.stage[b] = suf[g_ss + b];
      __builtin_amdgcn_wave_barrier();
      for (int k = 0; k < nv; k++) {
        const int64_t kpl = __shfl(pl, k, 64), kss = __shfl(ss, k, 64), kse = __shfl(se, k, 64);
        const int64_t klen = __shfl(len, k, 64), kost = __shfl(ostart, k, 64);
        const int64_t ksl = kse - kss;
        if (klen <= kDbaPrev) {
          if (!in_lds && kpl > 0) {
            // the previous value was too long for LDS: its prefix from the output
            __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0): this wave's stores of it are done
            for (int64_t b = lane; b < kpl; b += 64)
              sh.prev[b] = (uint8_t)(ld_l2_u32((const PQG_G uint32_t*)((uintptr_t)(chars + pstart + b) & ~(uintptr_t)3)) >>
                                     (8 * ((uintptr_t)(chars + pstart + b) & 3)));
            __builtin_amdgcn_wave_barrier();
          }
          for (int64_t b = lane; b < ksl; b += 64)
            sh.prev[kpl + b] = staged ? sh.stage[kss - g_ss + b] : suf[kss + b];
          __builtin_amdgcn_wave_barrier();
          for (int64_t b = lane; b < klen; b += 64) chars[kost + b] = sh.prev[b];
          __builtin_amdgcn_wave_barrier();
          in_lds = true;
        } else {
          // a value longer than the LDS buffer: prefix from the previous value's
          // output (LDS or memory), suffix from the page
          __builtin_amdgcn_s_waitcnt(0);
          for (int64_t b = lane; b < kpl; b += 64) {
            uint8_t c;
            if (in_lds) c = sh.prev[b];
            else {
              const uintptr_t a = (uintptr_t)(chars + pstart + b);
              c = (uint8_t)(ld_l2_u32((const PQG_G uint32_t*)(a & ~(uintptr_t)3)) >> (8 * (a & 3)));
            }
            chars[kost + b] = c;
          }
          for (int64_t b = lane; b < ksl; b += 64) chars[kost + kpl + b] = suf[kss + b];
          in_lds = false;
        }
        plen = klen;
        pstart = kost;
      }
      (void)plen;
      oend += incl;
      sprev = g_se;
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// ---- K7c ---------------------------------------------------------------------
// Per chunk: the chars of every part (dictionary parts: k_str_count; PLAIN
// parts: from the page-relative value ends k_str_plain wrote; DELTA pages:
// k_str_delta), an exclusive scan in part order -> each part's chunk char
// offset (and a page's, its part 0's), the chunk's chars.  A PLAIN part also
// keeps the page-relative start of its first value: k_str_copy rewrites the
// ends in place, so a part cannot read its predecessor's last end then.
__global__ void __launch_bounds__(256) k_char_scan(JobDev* jobs, PageDev* pages, PartRec* parts, int64_t* offs_arena) {
  __shared__ int64_t part[5];
  JobDev& job = jobs[blockIdx.x];
  if (job.value_width != 0 || job.status == kCAPACITY) return;
  const int ni = job.n_items;
  PartRec* pr = parts + job.item_base;
  int64_t carry = 0;
  for (int b = 0; b < ni; b += 256) {
    const int i = b + threadIdx.x;
    int64_t v = 0, prel = 0;
    int pidx = -1, p = 0;
    if (i < ni) {
      const PartRec r = pr[i];
      pidx = r.pidx;
      p = r.p;
      const PageDev& pg = pages[pidx];
      if ((pg.page_type == 0 || pg.page_type == 3) && pg.read_status == kOK && pg.decode_status == kOK &&
          pg.vmode == 2) {
        if (pg.encoding == 8) {
          v = r.chars;
        } else if (pg.encoding == 0) {
          const PQG_G int64_t* ends = gconst(offs_arena) + job.offs_base + pg.value_offset + 1;
          const int64_t lo = r.v0, hi = r.p + 1 < r.np ? (int64_t)pr[i + 1].v0 : (int64_t)pg.not_null;
          prel = lo > 0 ? ends[lo - 1] : 0;
          v = hi > lo ? ends[hi - 1] - prel : 0;
        } else {
          v = pg.chars;  // DELTA_LENGTH_BYTE_ARRAY / DELTA_BYTE_ARRAY: one part
        }
      }
    }
    int64_t tot;
    const int64_t ex = block_excl_scan<256>(v, &tot, part);
    if (i < ni) {
      pr[i].cstart = carry + ex;
      pr[i].prel = prel;
      if (p == 0) pages[pidx].char_offset = carry + ex;
    }
    carry += tot;
  }
  if (threadIdx.x == 0) {
    job.values_bytes = carry;
    if (carry > job.value_cap) job.status = kCAPACITY;
    offs_arena[job.offs_base] = 0;
  }
}

}  // namespace pqg

namespace pqg {

// ---- K7d -----------------------------------------------------------------------
// One block per byte-array data page part, one value per thread.  PLAIN: value
// i's chars [e(i-1), e(i)) come from its record at e(i-1) + 4 (i + 1) of the
// page's value section (k_str_plain left the page-relative ends in the
// offsets).  Dictionary: the slot holds the key (k_str_count); the value is
// dictionary entry `key`, and its start is a block scan of the entry lengths.
// The ends become chunk offsets.  A round's 512 values are assembled in LDS
// and leave as aligned 16-byte granules (only the round's two edge granules,
// shared with the neighbouring rounds or pages, are written bytewise); a round
// of more than kCopyStage bytes copies value by value.
constexpr int kCopyStage = 16384;

// len bytes from global src to LDS dst (any alignment)
__device__ __forceinline__ void lds_copy(PQG_L uint8_t* dst, gcu8 src, int64_t len) {
  int64_t k = 0;
  for (; k + 4 <= len; k += 4) {
    const uintptr_t a = (uintptr_t)(src + k);
    const PQG_G uint32_t* q = (const PQG_G uint32_t*)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3) * 8;
    const uint32_t x = sh ? __builtin_amdgcn_alignbit(q[1], q[0], sh) : q[0];
    dst[k] = (uint8_t)x;
    dst[k + 1] = (uint8_t)(x >> 8);
    dst[k + 2] = (uint8_t)(x >> 16);
    dst[k + 3] = (uint8_t)(x >> 24);
  }
  for (; k < len; k++) dst[k] = src[k];
}

// A value of <= 32 bytes from global src to LDS dst: its (at most 10)
// aligned source dwords are loaded together, unconditionally (clamped to the
// value's last dword), so a round of values costs one round trip instead of
// one per 4 bytes (the dictionary gathers of k_str_copy)
__device__ __forceinline__ void lds_copy_short(PQG_L uint8_t* dst, gcu8 src, int64_t len) {
  const uintptr_t a = (uintptr_t)src, base = a & ~(uintptr_t)3;
  const uintptr_t last = len > 0 ? (a + (uintptr_t)len - 1) & ~(uintptr_t)3 : base;
  const uint32_t sh = (uint32_t)(a & 3) * 8;
  uint32_t w[9];
#pragma unroll
  for (int k = 0; k < 9; k++) {
    const uintptr_t q = base + 4 * (uintptr_t)k;
    w[k] = *(const PQG_G uint32_t*)(q < last ? q : last);
  }
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const uint32_t x = sh ? __builtin_amdgcn_alignbit(w[k + 1], w[k], sh) : w[k];
#pragma unroll
    for (int b = 0; b < 4; b++)
      if (4 * k + b < len) dst[4 * k + b] = (uint8_t)(x >> (8 * b));
  }
}

// len bytes LDS -> LDS (any alignment): aligned dword reads, byte writes
__device__ __forceinline__ void lds_copy_l(PQG_L uint8_t* dst, const PQG_L uint8_t* src, int64_t len) {
  int64_t k = 0;
  for (; k + 4 <= len; k += 4) {
    const uint32_t a = (uint32_t)(uintptr_t)(src + k);
    const PQG_L uint32_t* q = (const PQG_L uint32_t*)(src + k - (a & 3));
    const uint32_t x = __builtin_amdgcn_alignbit(q[1], q[0], (a & 3) * 8);
    dst[k] = (uint8_t)x;
    dst[k + 1] = (uint8_t)(x >> 8);
    dst[k + 2] = (uint8_t)(x >> 16);
    dst[k + 3] = (uint8_t)(x >> 24);
  }
  for (; k < len; k++) dst[k] = src[k];
}
constexpr int kSrcStage = kCopyStage + 4 * 512 + 64;  // a PLAIN round's records: chars + length prefixes

// k_str_copy waves per SIMD: 4 blocks of 512 per CU (its LDS allows 4; at 8
// waves/SIMD it keeps 64 VGPRs, 8 spilled): C4 1.01 -> 0.92 ms, C5 2.57 ->
// 2.61 ms.  (k_str_count at 4 waves/SIMD spills 36 VGPRs: C5 0.97 -> 1.15 ms.)
#ifndef PQG_COPY_WPE
#define PQG_COPY_WPE 8
#endif
__global__ void __attribute__((amdgpu_flat_work_group_size(1, 512), amdgpu_waves_per_eu(PQG_COPY_WPE))) k_str_copy(JobDev* jobs, PageDev* pages, const PartRec* parts, const int* total,
                                                  int* queue, uint8_t* value_arena, int64_t* offs_arena) {
  __shared__ int s_t;
  __shared__ int64_t s_prev;  // page-relative end of the value before the round
  __shared__ int64_t part[9];
  __shared__ __attribute__((aligned(16))) uint8_t stage[kCopyStage];
  __shared__ __attribute__((aligned(16))) uint8_t sstage[kSrcStage + 16];  // PLAIN / DLBA sources of a round
  const int n_items = min(total[kCtrItems], total[kCtrPartsCap]);
  for (;;) {
    if (threadIdx.x == 0) s_t = queue_pull(queue);
    __syncthreads();
    const int t = s_t;
    __syncthreads();
    if (t >= n_items) return;
    const PartRec& pr = parts[t];
    if (pr.vmode != 2) continue;
    const int pidx = pr.pidx;
    const PageDev& pg = pages[pidx];
    if (pg.read_status != kOK || pg.decode_status != kOK || (pg.page_type != 0 && pg.page_type != 3) || pg.vmode != 2 ||
        pg.not_null == 0 || pg.encoding == 7)  // DELTA_BYTE_ARRAY: k_str_dba
      continue;
    const JobDev& job = jobs[pg.job];
    if (job.status == kCAPACITY) continue;
    const int64_t base = pg.char_offset;
    // the part's values [v_lo, nn): a page's part ends at the next part's first value
    const int64_t v_lo = pr.v0, nn = pr.p + 1 < pr.np ? (int64_t)parts[t + 1].v0 : (int64_t)pg.not_null;
    if (threadIdx.x == 0) s_prev = pg.encoding == 0 ? pr.prel : pg.encoding == 8 ? pr.cstart - base : 0;
    __syncthreads();
    const bool dlba = pg.encoding == 6;  // value bytes back to back from cstart
    const gu8 chars = gmut(value_arena) + job.value_base + base;
    PQG_G int64_t* ends = gmut(offs_arena) + job.offs_base + pg.value_offset + 1;
    const bool dict = pg.encoding == 8;
    const gcu8 src = dict ? gconst(job.dict_data) : gconst(pg.val);
    const PQG_G int64_t* doffs = gconst(job.dict_offs);
    for (int64_t i0 = v_lo; i0 < nn; i0 += 512) {
      const int64_t i = i0 + threadIdx.x;
      const int64_t r_lo = s_prev;  // the round's first byte (read before any barrier moves it)
      int64_t e = 0, s0 = 0, from = 0;
      if (dict) {
        // unconditional loads (the value index clamped to nn - 1): a load
        // under a branch is waited for inside it
        const int64_t key = ends[i < nn ? i : nn - 1];
        const int64_t f0 = doffs[key] + 4, f1 = doffs[key + 1];
        int64_t len = 0;
        if (i < nn) {
          from = f0;
          len = f1 - f0;
        }
        int64_t tot;
        s0 = r_lo + block_excl_scan<512>(len, &tot, part);
        e = s0 + len;
        if (threadIdx.x == 0) s_prev += tot;  // after the scan's last barrier
      } else {
        if (i < nn) {
          e = ends[i];
          s0 = threadIdx.x ? ends[i - 1] : r_lo;
          from = dlba ? pg.cstart + s0 : s0 + 4 * (i + 1);
        }
        __syncthreads();  // every end of the round is read before any is rewritten
        if (i == (i0 + 512 < nn ? i0 + 511 : nn - 1)) s_prev = e;
      }
      __syncthreads();
      const int64_t r_hi = s_prev;
      const uintptr_t abs_lo = (uintptr_t)(chars + r_lo), abs_hi = (uintptr_t)(chars + r_hi);
      const uintptr_t A0 = abs_lo & ~(uintptr_t)15;
      if (abs_hi - A0 <= (uintptr_t)kCopyStage) {
        // PLAIN / DLBA: the round's source bytes are contiguous in the page
        // (records, or values back to back): staged in LDS with one round of
        // coalesced loads, then every value is copied LDS -> LDS
        const int64_t i_last = i0 + 512 < nn ? i0 + 511 : nn - 1;
        const int64_t S_lo = dlba ? pg.cstart + r_lo : r_lo + 4 * (i0 + 1);
        const int64_t S_hi = dlba ? pg.cstart + r_hi : r_hi + 4 * (i_last + 1);
        const uintptr_t SA0 = (uintptr_t)(src + S_lo) & ~(uintptr_t)15;
        const bool sstaged = !dict && S_hi > S_lo && (uintptr_t)(src + S_hi) - SA0 <= (uintptr_t)kSrcStage;
        if (sstaged) {
          const uintptr_t last = ((uintptr_t)(src + S_hi) - 1) & ~(uintptr_t)15;
          constexpr int kSG = (kSrcStage + 16 + 16 * 512 - 1) / (16 * 512);
          uint4 v[kSG];
#pragma unroll
          for (int k = 0; k < kSG; k++) {  // unconditional loads (clamped)
            const uintptr_t g = SA0 + 16 * (uintptr_t)(threadIdx.x + 512 * k);
            v[k] = ldg16(g < last ? g : last);
          }
#pragma unroll
          for (int k = 0; k < kSG; k++) {
            const uint32_t o = 16 * (threadIdx.x + 512 * k);
            if (o < (uint32_t)(kSrcStage + 16)) sts16(lds_ptr(sstage) + o, v[k]);
          }
          __syncthreads();
          if (i < nn) {
            lds_copy_l(lds_ptr(stage) + ((uintptr_t)(chars + s0) - A0),
                       lds_ptr(sstage) + ((uintptr_t)(src + from) - SA0), e - s0);
            ends[i] = base + e;
          }
        } else if (i < nn) {
          PQG_L uint8_t* d = lds_ptr(stage) + ((uintptr_t)(chars + s0) - A0);
          if (e - s0 <= 32) lds_copy_short(d, src + from, e - s0);
          else lds_copy(d, src + from, e - s0);
          ends[i] = base + e;
        }
        __syncthreads();
        for (uintptr_t g = A0 + 16 * (uintptr_t)threadIdx.x; g < abs_hi; g += 16 * 512) {
          const u32x4_t v = *(const PQG_L u32x4_t*)(lds_ptr(stage) + (g - A0));
          if (g >= abs_lo && g + 16 <= abs_hi) {
            stg16o(g, make_uint4(v.x, v.y, v.z, v.w));
          } else {
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
            for (int b = 0; b < 16; b++)
              if (g + b >= abs_lo && g + b < abs_hi) *(PQG_G uint8_t*)(g + b) = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
          }
        }
      } else if (i < nn) {
        copy_bytes(chars + s0, src + from, e - s0);
        ends[i] = base + e;
      }
      __syncthreads();
    }
  }
}

}  // namespace pqg
