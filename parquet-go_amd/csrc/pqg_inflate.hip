// pqg_inflate.hip — GZIP pages: gzipCompressor.DecompressBlock (compress.go:63-76):
// gzip.NewReader + ioutil.ReadAll over the page's compressed block, i.e. Go's
// compress/gzip in its default multistream mode (RFC 1952 members, one after
// another, until the block ends exactly after one) around compress/flate
// (RFC 1951).  The decoded bytes of a valid stream are the format's; errors
// (bad header, bad DEFLATE data, CRC-32 / ISIZE mismatch, a truncated member,
// trailing bytes that are not a member) are PQG_ERR_GZIP, as the oracle
// classifies them (oracle/pq_oracle.cpp gzip_decode); a decoded length other
// than the page's uncompressed size is PQG_ERR_SIZE (compress.go:117).
//
// One wave per compressed page (k_inflate_s: an 8 KiB history ring, older
// matches read back from the stored output; k_inflate: the 32 KiB window, for
// pqg_block_decompress and the pages k_inflate_s hands back).  DEFLATE is a
// serial bit stream, so the symbol decode runs wave-uniform (the decoder
// state is scalar; table reads are LDS broadcasts moved to scalar registers)
// with canonical-Huffman tables built per block in LDS by ballots (a 9-bit
// fast table with a literal flag, then the count / symbol walk of RFC 1951
// codes).  Runs of literals take a tight loop (lit_run: two per step, bytes
// gathered one per lane and written to the ring 64 at a time); the lanes
// split the byte work: copies of a match from the LDS history ring, the
// flush of decoded bytes to HBM in 16-byte granules, and the CRC-32 of every
// flushed piece (per-lane slices combined in a tree with x^(8n) mod P shifts
// from a table of x^(2^k)).
#include <hip/hip_runtime.h>

#include "pqg_common.h"
#include "pqg_device.h"
#include "pqg_hybrid.h"

namespace pqg {

#ifdef PQG_PROFILE
// host reader of this translation unit's counters (pqg_debug_counters 160..191)
int prof_read_inflate(unsigned long long* out) {
  unsigned long long z[64] = {0};
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pqg_prof), sizeof(z)) != hipSuccess) return -1;
  hipMemcpyToSymbol(HIP_SYMBOL(pqg_prof), z, sizeof(z));
  return 0;
}
#define PQG_CNT(i, v) (f_cnt[i] += (v))
#else
#define PQG_CNT(i, v) ((void)0)
#endif

namespace {

constexpr int kRing = 32768;      // DEFLATE window: the whole history a distance can reach
#ifndef PQG_INFLATE_RING
#define PQG_INFLATE_RING 8192
#endif
constexpr int kRingSmall = PQG_INFLATE_RING;  // k_inflate_s: older history is read back from the flushed output
constexpr int kInStage = 1024;    // compressed bytes staged in LDS per refill
constexpr int kInflateRedo = 0x7ffe;  // k_inflate_s: a page for the 32 KiB-ring pass (not a status)
constexpr int kFastBits = 9;
constexpr uint32_t kCrcPoly = 0xedb88320u;  // CRC-32 (IEEE, reflected): gzip trailer

struct Huff {
  uint16_t count[16];    // codes per length
  uint16_t symbol[288];  // symbols by (length, value)
  uint16_t fast[1 << kFastBits];  // next 9 stream bits -> literal << 15 | length << 9 | symbol, 0: longer code
};

template <int kRingT>
struct InflateShared {
  uint8_t ring[kRingT];
  uint8_t in[kInStage + 16];
  uint32_t crc_tab[256];
  uint32_t seg_crc[64];
  Huff lit, dist;
  uint16_t lens[352];  // code lengths: [0, 19) code-length code, [32, 348) decoded, then lit/len [0, 286) + dist [288, 318)
  int err;  // table build errors (any lane)
};

// RFC 1951 3.2.5 length and distance codes, computed (no table loads on the
// match path): length code s (symbol 257 + s) and distance code ds
__device__ __forceinline__ uint32_t len_ext(uint32_t s) { return s < 8 || s == 28 ? 0u : (s >> 2) - 1; }
__device__ __forceinline__ uint32_t len_base(uint32_t s, uint32_t ext) {
  return s < 8 ? s + 3 : s == 28 ? 258u : ((4 + (s & 3)) << ext) + 3;
}
__device__ __forceinline__ uint32_t dist_ext(uint32_t ds) { return ds < 4 ? 0u : (ds >> 1) - 1; }
__device__ __forceinline__ uint32_t dist_base(uint32_t ds, uint32_t ext) {
  return ds < 4 ? ds + 1 : ((2 + (ds & 1)) << ext) + 1;
}
__device__ const uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// a * b mod P over GF(2), reflected (bit 31 = x^0): zlib's multmodp,
// branch-free (32 fixed steps: the lanes of a CRC combine hold different a)
__host__ __device__ constexpr uint32_t multmodp(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#pragma unroll 4
  for (int i = 0; i < 32; i++) {
    p ^= b & (0u - ((a >> (31 - i)) & 1u));
    b = (b >> 1) ^ (kCrcPoly & (0u - (b & 1u)));
  }
  return p;
}
// x^(2^k) mod P, k = 0..31 (zlib's x2n_table; the period is 32)
struct X2n {
  uint32_t v[32];
};
constexpr X2n make_x2n() {
  X2n t{};
  uint32_t p = 1u << 30;  // x^1
  t.v[0] = p;
  for (int k = 1; k < 32; k++) t.v[k] = p = multmodp(p, p);
  return t;
}
__device__ const X2n kX2n = make_x2n();
// x^(8 n) mod P: one multiply per set bit of n (zlib's x2nmodp(n, 3))
__device__ __forceinline__ uint32_t x8nmodp(uint64_t n) {
  uint32_t p = 1u << 31;  // x^0
  for (int k = 3; n; k++, n >>= 1)
    if (n & 1) p = multmodp(kX2n.v[k & 31], p);
  return p;
}

}  // namespace


// One wave's inflater.  Every lane holds the same state (wave-uniform control
// flow); `lane` splits the byte-parallel steps.  kRingT: the LDS history ring.
// A ring smaller than the 32 KiB window (k_inflate_s: 8 KiB, so ~10 waves fit
// a CU instead of 4) flushes every kRingT / 2 decoded bytes, so a match
// reaching further back than the ring finds its bytes already stored in the
// page's output: they are read back from there (L2).  Such a byte at or past
// the output's capacity (a page decoding to more than its size) was never
// stored: the page goes to the 32 KiB-ring pass (kInflateRedo).
template <int kRingT, typename Ix>
struct Inflater {
  static constexpr int kFlushT = kRingT >= 32768 ? 16384 : kRingT / 2;  // decoded bytes flushed (and CRC'd) at a time
  static_assert(kFlushT + 258 + 64 <= kRingT, "unflushed bytes and a match must fit the ring");
  InflateShared<kRingT>* sh;
  gcu8 src;
  Ix n;            // compressed bytes
  Ix pos = 0;      // next byte for the bit buffer
  Ix in_base = -(Ix)kInStage * 4;  // stream offset of in[0]
  uint64_t bitbuf = 0;
  int bitcnt = 0;
  gu8 dst;              // decoded bytes (cap of them are stored)
  Ix cap;
  Ix d = 0;        // decoded bytes so far
  Ix flushed = 0;  // decoded bytes flushed (stored and CRC'd)
  Ix mstart = 0;   // first decoded byte of the current member
  uint32_t crc = 0;     // CRC-32 of the member's flushed bytes (conditioned)
  int lane;
#ifdef PQG_PROFILE
  // 0 literals, 1 matches, 2 far matches, 3 slow decodes, 4 slow-walk bits,
  // 5 flush cycles, 6 stage() refills, 7 match bytes, 8 lit_run cycles,
  // 9 lit_run calls, 10 cycles of the other symbols (decode, copy, flush)
  uint64_t f_cnt[11] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#endif

  __device__ __forceinline__ void stage(Ix at) {
    // 16-byte granules from the aligned address at or below `at`; granules
    // past the block re-read its last one (never used)
    PQG_CNT(6, 1);
    const uintptr_t a0 = (uintptr_t)(src + at) & ~(uintptr_t)15;
    in_base = at - (Ix)((uintptr_t)(src + at) - a0);
    const uintptr_t last = ((uintptr_t)(src + n) - 1) & ~(uintptr_t)15;
    const uintptr_t a = a0 + 16 * (uintptr_t)lane;
    const uint4 v = ldg16(a <= last ? a : last);
    __builtin_amdgcn_wave_barrier();
    sts16(lds_ptr(sh->in) + 16 * lane, v);
    __builtin_amdgcn_wave_barrier();
  }
  __device__ __forceinline__ int byte_at(Ix i) {
    if (i < in_base || i >= in_base + kInStage) stage(i);
    return lds_ptr(sh->in)[i - in_base];
  }
  // the 4 bytes at i (staged window; bytes past the block are never used)
  __device__ __forceinline__ uint32_t word_at(Ix i) {
    if (i < in_base || i + 4 > in_base + kInStage) stage(i);
    const uint32_t o = (uint32_t)(i - in_base);
    const PQG_L uint32_t* W = (const PQG_L uint32_t*)lds_ptr(sh->in);
    return __builtin_amdgcn_readfirstlane(__builtin_amdgcn_alignbit(W[(o >> 2) + 1], W[o >> 2], (o & 3) * 8));
  }
  // at least k (<= 32) bits in the buffer; false past the end of the block.
  // Whole bytes are taken up to 4 at a time (one LDS read per refill, not one
  // per byte): the buffer runs ahead of the decode, which only ever reads it.
  __device__ __forceinline__ bool need(int k) {
    while (bitcnt < k) {
      if (pos >= n) return false;
      int m = (64 - bitcnt) >> 3;
      m = m > 4 ? 4 : m;
      if ((Ix)m > n - pos) m = (int)(n - pos);
      const uint32_t x = word_at(pos);
      bitbuf |= (uint64_t)(m >= 4 ? x : (x & ((1u << (8 * m)) - 1))) << bitcnt;
      pos += m;
      bitcnt += 8 * m;
    }
    return true;
  }
  __device__ __forceinline__ bool bits(int k, uint32_t* v) {
    if (k == 0) { *v = 0; return true; }
    if (!need(k)) return false;
    *v = (uint32_t)bitbuf & ((1u << k) - 1);
    bitbuf >>= k;
    bitcnt -= k;
    return true;
  }
  // the bytes of the next whole byte boundary on (stored blocks, trailers)
  __device__ __forceinline__ void align_byte() {
    const int r = bitcnt & 7;
    bitbuf >>= r;
    bitcnt -= r;
  }
  __device__ __forceinline__ bool byte_aligned(uint32_t* v) { return bits(8, v); }

  // Canonical code from lengths[0..n) (RFC 1951 3.2.2): counts, symbols, and
  // the 9-bit fast table.  Returns the number of unused code points at the
  // longest length (< 0: over-subscribed, 0: complete, > 0: incomplete), as
  // puff's construct.  Counts and the symbol order come from ballots over 64
  // symbols at a time (nsym <= 288); lane l keeps the count and the running
  // offset of length l, so no per-length arrays sit in scalar registers.
  __device__ __forceinline__ int build(Huff& h, const uint16_t* lengths, int nsym) {
    PQG_L Huff* H = lds_ptr(&h);
    const uint64_t lt = (1ull << lane) - 1;  // the lanes below this one
    uint32_t my_cnt = 0;                     // lane l: symbols of length l
#pragma unroll 1
    for (int k = 0; k < nsym; k += 64) {
      const uint32_t L = k + lane < nsym ? (uint32_t)lds_ptr(lengths)[k + lane] : 16u;  // 16: no symbol
#pragma unroll
      for (int l = 0; l < 16; l++) {
        const uint32_t c = (uint32_t)__popcll(__ballot(L == (uint32_t)l));
        if (lane == l) my_cnt += c;
      }
    }
    // left = 2^15 - sum_l cnt[l] * 2^(15 - l), the unused code points
    int left = 1;
#pragma unroll
    for (int l = 1; l < 16; l++) left = 2 * left - (int)__builtin_amdgcn_readlane(my_cnt, l);
    if (lane < 16) H->count[lane] = (uint16_t)my_cnt;
    // my_off (lane l >= 1): the first slot of length l = the counts of lengths 1 .. l-1
    uint32_t my_off = 0;
#pragma unroll
    for (int l = 1; l < 15; l++) {
      const uint32_t c = __builtin_amdgcn_readlane(my_cnt, l);
      if (lane > l) my_off += c;
    }
    // symbols by length then value: symbol s of length L goes after every
    // shorter code and every smaller symbol of length L
#pragma unroll 1
    for (int k = 0; k < nsym; k += 64) {
      const uint32_t L = k + lane < nsym ? (uint32_t)lds_ptr(lengths)[k + lane] : 16u;
      const uint32_t base = (uint32_t)__shfl((int)my_off, (int)(L & 15), 64);
      uint32_t rank = 0;
#pragma unroll
      for (int l = 1; l < 16; l++) {
        const uint64_t m = __ballot(L == (uint32_t)l);
        if (L == (uint32_t)l) rank = (uint32_t)__popcll(m & lt);
        if (lane == l) my_off += (uint32_t)__popcll(m);
      }
      if (L - 1u < 15u) H->symbol[base + rank] = (uint16_t)(k + lane);
    }
    __builtin_amdgcn_wave_barrier();
    // fast table: entry x = the next 9 stream bits (LSB first)
    for (int x = lane; x < (1 << kFastBits); x += 64) {
      int code = 0, first = 0, index = 0;
      uint16_t e = 0;
      for (int l = 1; l <= kFastBits; l++) {
        code |= (x >> (l - 1)) & 1;
        const int c = (int)H->count[l];
        if (code - c < first) {
          const uint32_t sy = H->symbol[index + (code - first)];
          e = (uint16_t)((sy < 256 ? 0x8000u : 0u) | l << 9 | sy);
          break;
        }
        index += c;
        first += c;
        first <<= 1;
        code <<= 1;
      }
      H->fast[x] = e;
    }
    __builtin_amdgcn_wave_barrier();
    return left;
  }

  // next symbol of code h, or -1 (out of input, or no such code)
  __device__ __forceinline__ int decode(const Huff& h) {
    const PQG_L Huff* H = lds_ptr(&h);
    need(kFastBits);  // as many as the block holds
    if (bitcnt >= kFastBits || bitcnt > 0) {
      const uint32_t e = __builtin_amdgcn_readfirstlane(H->fast[(uint32_t)bitbuf & ((1u << kFastBits) - 1)]);
      const int l = (int)((e >> 9) & 15);
      if (e != 0 && l <= bitcnt) {
        bitbuf >>= l;
        bitcnt -= l;
        return (int)(e & 511);
      }
    }
    // the slow walk, bit by bit (codes longer than 9 bits, or the block's end)
    PQG_CNT(3, 1);
    int code = 0, first = 0, index = 0;
    for (int l = 1; l < 16; l++) {
      PQG_CNT(4, 1);
      uint32_t b;
      if (!bits(1, &b)) return -1;
      code |= (int)b;
      const int c = __builtin_amdgcn_readfirstlane(H->count[l]);
      if (code - c < first) return __builtin_amdgcn_readfirstlane(H->symbol[index + (code - first)]);
      index += c;
      first += c;
      first <<= 1;
      code <<= 1;
    }
    return -1;
  }

  // ---- output: the history ring, flushed to HBM (bytes below cap) and CRC'd
  __device__ __forceinline__ void flush_to(Ix upto) {
    PQG_L uint8_t* ring = lds_ptr(sh->ring);
    __builtin_amdgcn_wave_barrier();
    const Ix nb = upto - flushed;
    if (nb <= 0) return;
    PQG_T(tf0);
    // stores: bytes [flushed, upto) below cap, 16-byte granules of the output
    const Ix s_hi = upto < cap ? upto : cap;
    if (s_hi > flushed) {
      const Ix g0 = flushed & ~(Ix)15;
      for (Ix g = g0 + 16 * (Ix)lane; g < s_hi; g += 1024) {
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          uint32_t x = 0;
#pragma unroll
          for (int b = 0; b < 4; b++) x |= (uint32_t)ring[(g + 4 * k + b) & (kRingT - 1)] << (8 * b);
          w[k] = x;
        }
        if (g >= flushed && g + 16 <= s_hi && ((uintptr_t)(dst + g) & 15) == 0) {
          stg16((uintptr_t)(dst + g), make_uint4(w[0], w[1], w[2], w[3]));
        } else {
          for (int b = 0; b < 16; b++)
            if (g + b >= flushed && g + b < s_hi) dst[g + b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
        }
      }
    }
    // CRC-32 of [flushed, upto): lane slices, combined in a tree
    const Ix per = (nb + 63) / 64;
    const Ix lo = flushed + per * lane, hi = lo + per < upto ? lo + per : upto;
    uint32_t c = 0;  // raw (unconditioned) CRC register of the slice
    for (Ix i = lo; i < hi; i++) c = lds_ptr(sh->crc_tab)[(c ^ ring[i & (kRingT - 1)]) & 0xff] ^ (c >> 8);
    // combine: crc(A || B) = crc(A) * x^(8 |B|) ^ crc(B) for raw registers
    Ix len = hi > lo ? hi - lo : 0;
#pragma unroll 1
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t oc = (uint32_t)__shfl_down((int)c, o, 64);
      const Ix ol = __shfl_down(len, o, 64);
      if ((lane & (2 * o - 1)) == 0 && lane + o < 64) {
        c = multmodp(x8nmodp((uint64_t)ol), c) ^ oc;
        len += ol;
      }
    }
    const uint32_t slice = (uint32_t)__shfl((int)c, 0, 64);
    // the member's conditioned CRC: crc' = ~( (~crc) * x^(8 nb) ^ raw )
    crc = ~(multmodp(x8nmodp((uint64_t)nb), ~crc) ^ slice);
    flushed = upto;
#ifdef PQG_PROFILE
    PQG_T(tf1);
    PQG_CNT(5, tf1 - tf0);
#endif
    __builtin_amdgcn_wave_barrier();
  }
  // false: a 32-bit decoder is past 2^30 decoded bytes (the 64-bit pass takes the page)
  __device__ __forceinline__ bool maybe_flush() {
    if (d - flushed >= kFlushT) {
      if (sizeof(Ix) < 8 && d > (Ix)(1 << 30)) return false;
      flush_to(d);
    }
    return true;
  }
  __device__ __forceinline__ void put(uint32_t byte) {
    if (lane == 0) lds_ptr(sh->ring)[d & (kRingT - 1)] = (uint8_t)byte;
    d++;
  }
  // len bytes from dist back (dist <= bytes of this member so far); false: a
  // source byte is neither in the ring nor stored (the 32 KiB-ring pass takes the page)
  __device__ __forceinline__ bool copy(uint32_t dist, uint32_t len) {
    PQG_L uint8_t* ring = lds_ptr(sh->ring);
    __builtin_amdgcn_wave_barrier();
    uint32_t done = 0;
    if (kRingT < 32768 && dist > (uint32_t)(kRingT - 64)) {
      // older than the ring: flushed (flushed >= d - kFlushT - 258), read back
      // from the output after this wave's stores completed (L2-coherent loads)
      __builtin_amdgcn_s_waitcnt(0);
      while (done < len) {
        const uint32_t k = len - done < 64u ? len - done : 64u;
        const Ix sp = d + done - dist + lane;  // source byte
        if (__ballot((uint32_t)lane < k && sp >= cap)) return false;
        uint32_t v = 0;
        if ((uint32_t)lane < k) {
          const uintptr_t a = (uintptr_t)(dst + sp);
          const uint32_t wv = ld_l2_u32((const PQG_G uint32_t*)(a & ~(uintptr_t)3));
          v = (wv >> (8 * (a & 3))) & 0xff;
        }
        if ((uint32_t)lane < k) ring[(d + done + lane) & (kRingT - 1)] = (uint8_t)v;
        __builtin_amdgcn_wave_barrier();
        done += k;
      }
      d += len;
      return true;
    }
    while (done < len) {
      // a round of min(dist, 64) bytes never reads a byte written in the round
      const uint32_t step = dist < 64u ? dist : 64u;
      const uint32_t k = len - done < step ? len - done : step;
      uint8_t v = 0;
      if ((uint32_t)lane < k) v = ring[(d + done + lane - dist) & (kRingT - 1)];
      __builtin_amdgcn_wave_barrier();
      if ((uint32_t)lane < k) ring[(d + done + lane) & (kRingT - 1)] = v;
      __builtin_amdgcn_wave_barrier();
      done += k;
    }
    d += len;
    return true;
  }

  // ---- one DEFLATE stream (RFC 1951 3.2.3), kOK or kGZIP
  // Literals while the next code is a literal of the fast table: the bytes
  // collect in one VGPR (lane i: the batch's i-th literal) and go to the ring
  // 64 at a time, so a literal costs one table read and a few scalar ops
  // instead of decode() + put().  Exact: only real stream bits are consumed
  // (the 4-byte refills stop short of the end, where decode() takes over),
  // and any other symbol is left to decode(), which reads the same entry.
  // Returns with fewer than kFlushT + 64 bytes unflushed.
  __device__ __forceinline__ void lit_run(const Huff& lc) {
    const PQG_L uint16_t* F = lds_ptr(lc.fast);
    PQG_L uint8_t* ring = lds_ptr(sh->ring);
    int pend = 0;
    int np = 0;
    for (;;) {
      // two literals per step: >= 2 x 9 bits in the buffer
      if (bitcnt < 32) {
        if (pos + 4 <= n) {
          bitbuf |= (uint64_t)word_at(pos) << bitcnt;
          pos += 4;
          bitcnt += 32;
        } else if (bitcnt < 2 * kFastBits) {
          break;
        }
      }
      const uint32_t e = __builtin_amdgcn_readfirstlane(F[(uint32_t)bitbuf & ((1u << kFastBits) - 1)]);
      if (!(e & 0x8000u)) break;  // not a literal of the table (a longer code, or a length / end code)
      const uint32_t l = (e >> 9) & 15;
      bitbuf >>= l;
      bitcnt -= (int)l;
      PQG_CNT(0, 1);
      pend = lane == np ? (int)(e & 255) : pend;  // lane np takes the byte
      const uint32_t e2 = __builtin_amdgcn_readfirstlane(F[(uint32_t)bitbuf & ((1u << kFastBits) - 1)]);
      if (!(e2 & 0x8000u)) {
        np++;
        break;
      }
      const uint32_t l2 = (e2 >> 9) & 15;
      bitbuf >>= l2;
      bitcnt -= (int)l2;
      PQG_CNT(0, 1);
      pend = lane == np + 1 ? (int)(e2 & 255) : pend;
      np += 2;
      if (np == 64) {
        ring[(d + lane) & (kRingT - 1)] = (uint8_t)pend;
        d += 64;
        np = 0;
        if (d - flushed >= kFlushT) break;
      }
    }
    if (lane < np) ring[(d + lane) & (kRingT - 1)] = (uint8_t)pend;
    d += np;
    __builtin_amdgcn_wave_barrier();
  }
  __device__ __forceinline__ int codes(const Huff& lc, const Huff& dc) {
    for (;;) {
      PQG_T(tl0);
      lit_run(lc);
#ifdef PQG_PROFILE
      PQG_T(tl1);
      PQG_CNT(8, tl1 - tl0);
      PQG_CNT(9, 1);
#endif
      const int sym = decode(lc);
      if (sym < 0) return kGZIP;
      if (sym < 256) {
        PQG_CNT(0, 1);
        put((uint32_t)sym);
      } else if (sym == 256) {
        return kOK;
      } else {
        const int s = sym - 257;
        if (s >= 29) return kGZIP;
        uint32_t e;
        const uint32_t lx = len_ext((uint32_t)s);
        if (!bits(lx, &e)) return kGZIP;
        const uint32_t len = len_base((uint32_t)s, lx) + e;
        const int ds = decode(dc);
        if (ds < 0 || ds >= 30) return kGZIP;
        const uint32_t dx = dist_ext((uint32_t)ds);
        if (!bits(dx, &e)) return kGZIP;
        const uint32_t dist = dist_base((uint32_t)ds, dx) + e;
        if ((Ix)dist > d - mstart) return kGZIP;  // "invalid distance too far back"
        PQG_CNT(1, 1);
        PQG_CNT(2, dist > (uint32_t)(kRingT - 64) ? 1 : 0);
        PQG_CNT(7, len);
        if (!copy(dist, len)) return kInflateRedo;
      }
      if (!maybe_flush()) return kInflateRedo;
#ifdef PQG_PROFILE
      PQG_T(tl2);
      PQG_CNT(10, tl2 - tl1);
#endif
    }
  }
  __device__ __forceinline__ int stored() {
    align_byte();
    uint32_t a, b, c, e;
    if (!bits(8, &a) || !bits(8, &b) || !bits(8, &c) || !bits(8, &e)) return kGZIP;
    const uint32_t len = a | b << 8, nlen = c | e << 8;
    if (len != (~nlen & 0xffffu)) return kGZIP;
    for (uint32_t k = 0; k < len; k++) {
      uint32_t v;
      if (!bits(8, &v)) return kGZIP;
      put(v);
      if (((k & 255) == 255 || k + 1 == len) && !maybe_flush()) return kInflateRedo;
    }
    return kOK;
  }
  // the block's code tables (codes() then decodes its symbols: one inlined copy)
  __device__ __forceinline__ int fixed() {
    PQG_L uint16_t* L = lds_ptr(sh->lens);
    for (int s = lane; s < 288 + 30; s += 64)
      L[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : s < 288 ? 8 : 5;
    __builtin_amdgcn_wave_barrier();
    return tables(288, 30, false);
  }
  // the literal/length and distance codes from lens[0..nlen) and lens[288..):
  // one build site in a loop (not one inlined build per table).  check: a
  // dynamic block's codes must be complete, except that a code may be a
  // single code of length 1 (puff, zlib's inflate_table); the fixed distance
  // code (30 of 32 five-bit codes) is incomplete by definition.
  __device__ __forceinline__ int tables(uint32_t nlen, uint32_t ndist, bool check) {
#pragma unroll 1
    for (int t = 0; t < 2; t++) {
      Huff& h = t ? sh->dist : sh->lit;
      const int ns = (int)(t ? ndist : nlen);
      const int e = build(h, sh->lens + (t ? 288 : 0), ns);
      if (check && (e < 0 || (e > 0 && ns != (int)lds_ptr(h.count)[0] + (int)lds_ptr(h.count)[1]))) return kGZIP;
    }
    return kOK;
  }
  __device__ __forceinline__ int dynamic() {
    uint32_t nlen, ndist, ncode;
    if (!bits(5, &nlen) || !bits(5, &ndist) || !bits(4, &ncode)) return kGZIP;
    nlen += 257;
    ndist += 1;
    ncode += 4;
    if (nlen > 286 || ndist > 30) return kGZIP;
    PQG_L uint16_t* L = lds_ptr(sh->lens);
    for (int s = lane; s < 19; s += 64) L[s] = 0;
    __builtin_amdgcn_wave_barrier();
    for (uint32_t k = 0; k < ncode; k++) {
      uint32_t v;
      if (!bits(3, &v)) return kGZIP;
      if (lane == 0) L[kClOrder[k]] = (uint16_t)v;
    }
    __builtin_amdgcn_wave_barrier();
    if (build(sh->lit, sh->lens, 19) != 0) return kGZIP;  // the code-length code must be complete
    // literal/length and distance code lengths (into lens, after the first 19 are used up)
    uint32_t index = 0;
    const uint32_t total = nlen + ndist;
    // decoded lengths go to lens[32 ...] (lens[0..18] hold the code-length code's lengths)
    PQG_L uint16_t* O = L + 32;
    while (index < total) {
      const int sym = decode(sh->lit);
      if (sym < 0) return kGZIP;
      if (sym < 16) {
        if (lane == 0) O[index] = (uint16_t)sym;
        index++;
      } else {
        uint32_t len = 0, rep, e;
        if (sym == 16) {
          if (index == 0) return kGZIP;
          __builtin_amdgcn_wave_barrier();
          len = O[index - 1];
          if (!bits(2, &e)) return kGZIP;
          rep = 3 + e;
        } else if (sym == 17) {
          if (!bits(3, &e)) return kGZIP;
          rep = 3 + e;
        } else {
          if (!bits(7, &e)) return kGZIP;
          rep = 11 + e;
        }
        if (index + rep > total) return kGZIP;
        for (uint32_t k = lane; k < rep; k += 64) O[index + k] = (uint16_t)len;
        index += rep;
      }
      __builtin_amdgcn_wave_barrier();
    }
    __builtin_amdgcn_wave_barrier();
    if (O[256] == 0) return kGZIP;  // no end-of-block code
    // move the lengths down: lit/len at lens[0..nlen), distance at lens[288..)
    uint16_t v[5];
#pragma unroll
    for (int k = 0; k < 5; k++) {
      const uint32_t s = (uint32_t)lane + 64u * k;
      v[k] = s < total ? O[s] : (uint16_t)0;
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 5; k++) {
      const uint32_t s = (uint32_t)lane + 64u * k;
      if (s < nlen) L[s] = v[k];
      else if (s < total) L[288 + (s - nlen)] = v[k];
    }
    __builtin_amdgcn_wave_barrier();
    return tables(nlen, ndist, true);
  }
  __device__ __forceinline__ int deflate() {
    uint32_t last, type;
    do {
      if (!bits(1, &last) || !bits(2, &type)) return kGZIP;
      int e;
      if (type == 0) {
        e = stored();
      } else {
        e = type == 1 ? fixed() : type == 2 ? dynamic() : kGZIP;
        if (!e) e = codes(sh->lit, sh->dist);
      }
      if (e) return e;
    } while (!last);
    return kOK;
  }

  // ---- RFC 1952 members until the block ends (Go's multistream reader)
  __device__ __forceinline__ int run() {
    PQG_L uint32_t* T = lds_ptr(sh->crc_tab);
    for (int i = lane; i < 256; i += 64) {
      uint32_t c = (uint32_t)i;
#pragma unroll
      for (int k = 0; k < 8; k++) c = c & 1 ? (c >> 1) ^ kCrcPoly : c >> 1;
      T[i] = c;
    }
    __builtin_amdgcn_wave_barrier();
    if (n <= 0) return kGZIP;  // NewReader: io.EOF on an empty block
    while (pos < n || bitcnt >= 8) {
      // the header: ID1 ID2 CM FLG MTIME(4) XFL OS, then the optional fields
      uint32_t hcrc = 0xffffffffu;
      auto hbyte = [&](uint32_t* v) -> bool {
        if (!bits(8, v)) return false;
        hcrc = T[(hcrc ^ *v) & 0xff] ^ (hcrc >> 8);
        return true;
      };
      uint32_t b[10];
      for (int k = 0; k < 10; k++)
        if (!hbyte(&b[k])) return kGZIP;
      if (b[0] != 0x1f || b[1] != 0x8b || b[2] != 8 || (b[3] & 0xe0)) return kGZIP;
      const uint32_t flg = b[3];
      uint32_t v, w;
      if (flg & 4) {  // FEXTRA
        if (!hbyte(&v) || !hbyte(&w)) return kGZIP;
        const uint32_t xlen = v | w << 8;
        for (uint32_t k = 0; k < xlen; k++)
          if (!hbyte(&v)) return kGZIP;
      }
      // FNAME, FCOMMENT: Go's readString reads into a [512]byte buffer, so the
      // NUL must come within 512 bytes (ErrHeader otherwise)
      if (flg & 8) {  // FNAME
        uint32_t k = 0;
        do {
          if (k++ == 512 || !hbyte(&v)) return kGZIP;
        } while (v != 0);
      }
      if (flg & 16) {  // FCOMMENT
        uint32_t k = 0;
        do {
          if (k++ == 512 || !hbyte(&v)) return kGZIP;
        } while (v != 0);
      }
      if (flg & 2) {  // FHCRC: the low 16 bits of the header's CRC-32
        const uint32_t want = ~hcrc & 0xffff;
        if (!bits(8, &v) || !bits(8, &w)) return kGZIP;
        if ((v | w << 8) != want) return kGZIP;
      }
      mstart = d;
      crc = 0;
      int e = deflate();
      if (e) return e;
      flush_to(d);
      // the trailer: CRC-32 and ISIZE (little endian) at the next byte boundary
      align_byte();
      uint32_t t[8];
      for (int k = 0; k < 8; k++)
        if (!bits(8, &t[k])) return kGZIP;
      const uint32_t c32 = t[0] | t[1] << 8 | t[2] << 16 | t[3] << 24;
      const uint32_t isz = t[4] | t[5] << 8 | t[6] << 16 | t[7] << 24;
      if (c32 != crc || isz != (uint32_t)(d - mstart)) return kGZIP;
    }
    return kOK;
  }
};

// The serial snappy path's twin for GZIP pages: one wave per page, decoded
// into the page's scratch block (its uncompressed size, 16-rounded).
__device__ __forceinline__ void gzip_loc(const PageDev& pg, int64_t* src_off, int64_t* clen, int64_t* ulen) {
  // V2 pages keep their level bytes raw in front of the compressed values
  // (page_v2.go:110-123)
  int64_t lv = 0;
  if (pg.page_type == 3) lv = (int64_t)(uint32_t)pg.rep_len + (int64_t)(uint32_t)pg.def_len;
  *src_off = pg.payload_offset + lv;
  *clen = (int64_t)pg.csize - lv;
  *ulen = (int64_t)pg.usize - lv;
}

// mode 0: every GZIP page of the list; 1: only the pages k_inflate_s left
// (kPageInflateRedo).
template <int kRingT, typename Ix>
__device__ __forceinline__ void inflate_pages(JobDev* jobs, PageDev* pages, const int* list, const int* total,
                                              int* queue, uint8_t* scratch, int mode) {
  __shared__ __attribute__((aligned(16))) InflateShared<kRingT> sh;
  const int lane = lane_id();
  for (;;) {
    const int t = queue_next(queue);
    if (t >= *total) return;
    const int pidx = __builtin_amdgcn_readfirstlane(list[t]);
    const PageDev pg = pages[pidx];
    if (pg.read_status != kOK || pg.scratch_offset < 0) continue;
    if (mode == 1 && !(pg.flags & kPageInflateRedo)) continue;
    const JobDev job = jobs[pg.job];
    if (job.codec != kCodecGzip) continue;
    int64_t so, clen, ulen;
    gzip_loc(pg, &so, &clen, &ulen);
    Inflater<kRingT, Ix> f;
    f.sh = &sh;
    f.src = gconst(job.data) + so;
    f.n = clen;
    f.dst = gmut(scratch) + job.scratch_base + pg.scratch_offset;
    f.cap = ulen;
    f.lane = lane;
    PQG_T(tp0);
    int e = f.run();
#ifdef PQG_PROFILE
    PQG_T(tp1);
    if (kRingT < kRing) {
      PQG_ACC(8, tp0, tp1);
      PQG_ACC(9, 0, 1);
      for (int k = 0; k < 8; k++) PQG_ACC(k, 0, f.f_cnt[k]);
      for (int k = 8; k < 11; k++) PQG_ACC(k + 2, 0, f.f_cnt[k]);  // slots 10..12
    }
#endif
    if (e == kInflateRedo) {  // k_inflate (32 KiB ring) decodes it again
      if (lane == 0) pages[pidx].flags |= kPageInflateRedo;
      continue;
    }
    if (pg.flags & kPageBareBlock) {  // pqg_block_decompress: the decoded length, no size check
      if (lane == 0) pages[pidx].gz_len = f.d;
    } else if (e == kOK && f.d != ulen) {
      e = kSIZE;  // "decompressed data must be %d byte" (compress.go:117)
    }
    // V1: getValuesDecoder runs after the block is decompressed (page_v1.go:91-97)
    if (e == kOK && pg.page_type == 0 && !values_supported(job.type, job.type_length, pg.encoding)) e = kUNSUPPORTED;
    if (lane == 0 && e != kOK) pages[pidx].read_status = e;
  }
}

// the 32 KiB ring: pqg_block_decompress blocks (mode 0) and the pages
// k_inflate_s left (mode 1)
__global__ void __launch_bounds__(64) k_inflate(JobDev* jobs, PageDev* pages, const int* list, const int* total,
                                                int* queue, uint8_t* scratch, int mode) {
  inflate_pages<kRing, int64_t>(jobs, pages, list, total, queue, scratch, mode);
}
// the GZIP pages of a decode, kRingSmall-byte ring
#ifndef PQG_INFLATE_WPE
#define PQG_INFLATE_WPE 1
#endif
__global__ void __attribute__((amdgpu_flat_work_group_size(1, 64), amdgpu_waves_per_eu(PQG_INFLATE_WPE))) k_inflate_s(JobDev* jobs, PageDev* pages, const int* list, const int* total,
                                                  int* queue, uint8_t* scratch) {
  inflate_pages<kRingSmall, int32_t>(jobs, pages, list, total, queue, scratch, 0);
}

}  // namespace pqg
