// pqg_snappy.hip — K2: snappy block decompression (compress.go:90-122 →
// snappy.Decode, vendor/github.com/golang/snappy/decode.go:55-72,
// decode_other.go:14-101).
#include <hip/hip_runtime.h>

#include "pqg_common.h"
#include "pqg_device.h"

namespace pqg {

#ifdef PQG_PROFILE
// host reader of this translation unit's phase counters (see pqg_debug_counters)
int prof_read_snappy(unsigned long long* out) {
  unsigned long long z[64] = {0};
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pqg_prof), sizeof(z)) != hipSuccess) return -1;
  hipMemcpyToSymbol(HIP_SYMBOL(pqg_prof), z, sizeof(z));
  return 0;
}
#endif

// ============================================================================
// K2: one wave per compressed block, tags resolved a window at a time.
//
// 1. Parse.  Every tag's length is a function of the bytes at its own
//    position, so each lane parses a tag speculatively at two of the next
//    kPos = 128 byte positions (lane, 64 + lane), from a 4 KiB LDS window.
// 2. Chain.  The true tags are the chain 0 -> next(0) -> ...; a scalar loop
//    follows it with v_readlane (an SGPR lane index), a few cycles per tag,
//    and marks it in two 64-bit masks.  Tags stay in their parse lanes.
// 3. Offsets and checks.  A DPP prefix sum over the chain's output lengths
//    gives every tag its output offset; the reference's checks
//    (decode_other.go:52, 85) and the batch cut (<= kSpan output bytes,
//    literal bytes inside the window) are then lane-parallel.
// 4a. Dense windows (>= kDense tags): the batch's output is 64 lanes x one
//    16-byte output granule, resolved byte by byte: a literal byte's source
//    is a window byte; a copy byte's source is the output byte `offset`
//    before it.  Copies reading bytes of the same batch (the overlapping
//    run-length form included) are resolved by pointer doubling over a
//    per-byte source table in LDS (<= 10 rounds, usually 0-2); then every
//    byte reads its source once, from the window or the history ring.
// 4b. Sparse windows (long literals, few tags): the tags are moved one at a
//    time with the fields already parsed — a literal as 16-byte granules,
//    one per lane, a copy one byte per lane — and the following tags are
//    taken one at a time too (the next header read ahead of the current
//    tag's bytes) until a streak of short tags sends the wave back to 1-3.
// The output history is a 64 KiB LDS ring: every copy-1/copy-2 offset
// (< 64 KiB) reads it; older bytes (copy-4) come from the flushed output
// through L2.  The ring leaves for HBM in 16-byte granules with each window
// refill (whose load wait then also covers the stores) or every 16 KiB.  A
// literal longer than the window goes from HBM in 4 KiB pieces.
// ============================================================================
constexpr int kPos = 128;         // tag positions parsed per window (2 per lane)
#ifndef PQG_SNAPPY_DENSE
#define PQG_SNAPPY_DENSE 8
#endif
constexpr int kDense = PQG_SNAPPY_DENSE;  // tags in a window for the batched byte resolution
constexpr int kSnWin = 4096;      // compressed-stream window (LDS)
constexpr int kSnWinNeed = 2048;  // window bytes wanted ahead of the first tag
constexpr int kSpan = 1024;       // output bytes a batch covers: 64 lanes x one 16-byte granule
#ifndef PQG_SNAPPY_RING
#define PQG_SNAPPY_RING 4096  // 4 KiB + 12 KiB of tables: 12 waves per CU (8 KiB: 9; r04 session 10: C4 snappy
                              // 11.95 -> 10.00 ms, C3 1.20 -> 0.93 ms with <= 168 VGPRs)
#endif
constexpr int kRing = PQG_SNAPPY_RING;  // output history kept in LDS (a power of two)
// flush granularity (a wave's stores are waited for at the next loop head);
// unflushed bytes (< kSnFlush + a batch or literal piece) must stay inside the ring
constexpr int kSnFlush = kRing / 4 < 16384 ? kRing / 4 : 16384;
// (kSnFlush + two writes of <= kLongPiece / a batch must fit the ring)
static_assert((kRing & (kRing - 1)) == 0 && kRing >= 4096, "ring: a power of two >= 4 KiB");
constexpr int kLongPiece = kRing >= 8192 ? 4096 : 1024;  // literal piece read from HBM
constexpr int kWinLit = 1024;     // literals up to this many bytes (after the granule prefix) move from the window
#ifndef PQG_SNAPPY_WPE
#define PQG_SNAPPY_WPE 3  // waves per EU the decoder is compiled for (3: <= 168 VGPRs, no spills)
#endif
#ifndef PQG_SNAPPY_LL_UNCOND
#define PQG_SNAPPY_LL_UNCOND 0  // 1: unconditional long-literal piece loads (36 B of spills at 168 VGPRs; C4 snappy 9.9 -> 10.7 ms)
#endif
#ifndef PQG_SNAPPY_SERIAL_CHAIN
#define PQG_SNAPPY_SERIAL_CHAIN 0
#endif
#ifndef PQG_SNAPPY_BATCH_WIN
#define PQG_SNAPPY_BATCH_WIN 3
#endif
constexpr int kBatchWin = PQG_SNAPPY_BATCH_WIN;  // windows of kPos positions one batch may take
constexpr int kBatchTags = 256;   // tag entries of a batch (>= 64 kBatchWin; marks are 1 + entry in a byte)
constexpr int kBatchRoom = 192;   // a batch with fewer free output bytes takes no further window
static_assert(64 * kBatchWin < kBatchTags && kBatchTags <= 256, "batch tags: byte marks");

struct SnapShared {
  uint8_t ring[kRing];
  uint8_t in[kSnWin + 32];
  union {
    int32_t src[kSpan];  // per output byte: [pre, kSpan) same batch, >= kSpan window byte + kSpan, else history
    struct {             // (before the doubling, which is the only user of src)
      uint8_t tmap[kSpan];         // 1 + batch tag entry, at the tag's first output byte
      u32x2_t tent[kBatchTags];    // per batch tag: {output start (relative to the batch's first granule),
                                   //  literal: 0x80000000 | window offset of its bytes; copy: offset}
    };
  };
  uint8_t cflag[kPos];    // chain marks of the pointer-doubling walk
};
static_assert(kSpan + 8 * kBatchTags <= 4 * kSpan, "tmap + tent share src's bytes");

// ---- 64-lane DPP scans (row_shr 1/2/4/8, row_bcast 15/31)
__device__ __forceinline__ uint32_t dpp_incl_add(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
  return x;
}
__device__ __forceinline__ uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint32_t dpp_incl_max(uint32_t x) {
  x = umax(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true));
  x = umax(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true));
  x = umax(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true));
  x = umax(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true));
  x = umax(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));
  x = umax(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));
  return x;
}
// value of the previous lane (0 in lane 0): DPP wave_shr:1
__device__ __forceinline__ uint32_t dpp_prev(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ int64_t readlane64(int64_t v, int l) {
  return (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l) |
         ((int64_t)__builtin_amdgcn_readlane((int)(v >> 32), l) << 32);
}

// One speculative tag at stream position pos (bytes from the LDS window).
struct Tag {
  int64_t len;   // output bytes
  int64_t next;  // position of the following tag (relative to the window's first position)
  uint32_t info; // copy offset
  int hdr;
  bool lit, err;
};

// lo, hi: the bytes [pos, pos + 8) of the block (decode_other.go:21-80 reads
// at most 5 of them)
__device__ __forceinline__ Tag parse_tag_bytes(uint32_t lo, uint32_t hi, int64_t pos, int64_t slen, int rel) {
  const uint32_t tag = lo & 0xff;
  const uint32_t w4 = (lo >> 8) | (hi << 24);  // bytes 1..4
  Tag t;
  t.lit = (tag & 3) == 0;
  t.info = 0;
  if (t.lit) {
    const uint32_t x = tag >> 2;
    if (x < 60) {
      t.hdr = 1;
      t.len = (int64_t)x + 1;
    } else {
      const int nb = (int)x - 59;
      t.hdr = 1 + nb;
      t.len = (int64_t)(nb == 4 ? w4 : (w4 & ((1u << (8 * nb)) - 1))) + 1;
    }
  } else if ((tag & 3) == 1) {
    t.hdr = 2;
    t.len = 4 + ((tag >> 2) & 7);
    t.info = (tag & 0xe0) << 3 | (w4 & 0xff);
  } else if ((tag & 3) == 2) {
    t.hdr = 3;
    t.len = 1 + (tag >> 2);
    t.info = w4 & 0xffff;
  } else {
    t.hdr = 5;
    t.len = 1 + (tag >> 2);
    t.info = w4;
  }
  t.err = pos + t.hdr > slen;                            // s += n; if s > len(src)
  if (t.lit) t.err |= t.len > slen - (pos + t.hdr);      // length > len(src)-s
  t.next = rel + t.hdr + (t.lit ? t.len : 0);
  return t;
}

__device__ __forceinline__ Tag parse_tag(const PQG_L uint8_t* in, uint32_t wo, int64_t pos, int64_t slen, int rel) {
  const PQG_L uint32_t* q = (const PQG_L uint32_t*)(in + (wo & ~3u));
  const uint32_t a = q[0], b = q[1], c = q[2];
  const uint32_t sft = (wo & 3) * 8;
  return parse_tag_bytes(__builtin_amdgcn_alignbit(b, a, sft), __builtin_amdgcn_alignbit(c, b, sft), pos, slen, rel);
}

// bytes [p, p + 8) of a block in global memory; dwords holding no byte of
// [0, slen) read as 0 (a dword holding one is mapped)
__device__ __forceinline__ void ld8_block(gcu8 src, int64_t slen, int64_t p, uint32_t& lo, uint32_t& hi) {
  const uintptr_t a = (uintptr_t)(src + p), q = a & ~(uintptr_t)3, end = (uintptr_t)(src + slen);
  const uint32_t w0 = q < end ? *(const PQG_G uint32_t*)q : 0u;
  const uint32_t w1 = q + 4 < end ? *(const PQG_G uint32_t*)(q + 4) : 0u;
  const uint32_t w2 = q + 8 < end ? *(const PQG_G uint32_t*)(q + 8) : 0u;
  const uint32_t sft = (uint32_t)(a & 3) * 8;
  lo = __builtin_amdgcn_alignbit(w1, w0, sft);
  hi = __builtin_amdgcn_alignbit(w2, w1, sft);
}

__device__ __forceinline__ uint32_t sat_add(uint32_t a, uint32_t b) {  // a, b <= 2^31 - 1
  const uint32_t c = a + b;
  return c > 0x7fffffffu ? 0x7fffffffu : c;
}
__device__ __forceinline__ uint32_t bperm(uint32_t v, int from_lane) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(from_lane << 2, (int)v);
}

// The chain step of the tag at window position rel (lo, hw: its bytes 0..7),
// branch-free and in 32 bits: J = parse_tag_bytes' next saturated at
// 0x7fffffff, O = its len saturated at 2^30 (the chain walks' caps).  The
// branchy 64-bit parse costs the walk its exec-mask juggling per step.
__device__ __forceinline__ void tag_step32(uint32_t lo, uint32_t hw, uint32_t rel, uint32_t& J, uint32_t& O) {
  const uint32_t tag = lo & 0xff, ty = tag & 3, x = tag >> 2;
  const uint32_t w4 = (lo >> 8) | (hw << 24);  // bytes 1..4
  const uint32_t nb = x >= 60 ? x - 59 : 0u;    // literal: extra length bytes
  const uint32_t mask = nb >= 4 ? 0xffffffffu : (1u << (8 * nb)) - 1u;
  const uint32_t lm1 = x < 60 ? x : (w4 & mask);  // literal length - 1
  const uint32_t hdr = ty == 0 ? 1 + nb : ty == 1 ? 2u : ty == 2 ? 3u : 5u;
  const uint32_t s = rel + hdr + 1 + lm1;          // literal: the next tag (may wrap)
  const bool sat = s < lm1 || s > 0x7fffffffu;
  const uint32_t Jl = sat ? 0x7fffffffu : s, Ol = lm1 >= (1u << 30) - 1 ? (1u << 30) : lm1 + 1;
  J = ty == 0 ? Jl : rel + hdr;
  O = ty == 0 ? Ol : ty == 1 ? 4 + (x & 7) : 1 + x;
}

// ---------------------------------------------------------------------------
// Tag-chain walk by pointer doubling (the split of big blocks, see k_snap_seg).
// Every lane follows its own chain position x (a block offset) to the first
// chain position >= hi, adding the output bytes of the tags it passes to acc.
// Each step takes the 64 positions from the smallest x still below hi: every
// lane parses the tag at one of them (speculatively), and six ds_bpermute
// doubling rounds give each position its exit from those 64 (or the first
// position >= hi inside them, which points at itself) and the output bytes on
// the way, so every chain in the window advances past it at once.
// ---------------------------------------------------------------------------
// RD: the 8 bytes at block offset p -> (lo, hi) (global memory, or a segment
// staged in LDS by k_snap_seg)
template <class RD>
__device__ void chain_walk_rd(const RD& rd, int64_t slen, int64_t hi, int64_t& x, uint32_t& acc) {
  const int lane = lane_id();
  for (;;) {
    const bool act = x < hi;
    if (!__ballot(act)) break;
    uint32_t xm = act ? (uint32_t)x : 0xffffffffu;  // block offsets are < 2^31
    // wave minimum by DPP (row_shr 1/2/4/8, row_bcast 15/31; lanes without a
    // source keep the identity), read from lane 63: no LDS round trips
#define PQG_MIN_STEP(ctrl, rm)                                                                          \
    {                                                                                                   \
      const uint32_t y = (uint32_t)__builtin_amdgcn_update_dpp((int)0xffffffffu, (int)xm, ctrl, rm, 0xf, false); \
      xm = y < xm ? y : xm;                                                                             \
    }
    PQG_MIN_STEP(0x111, 0xf) PQG_MIN_STEP(0x112, 0xf) PQG_MIN_STEP(0x114, 0xf) PQG_MIN_STEP(0x118, 0xf)
    PQG_MIN_STEP(0x142, 0xa) PQG_MIN_STEP(0x143, 0xc)
#undef PQG_MIN_STEP
    const int64_t wb = (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)xm, 63);
    const int64_t p = wb + lane;
    uint32_t lo, hw;
    rd(p, lo, hw);
#ifndef PQG_SNAP_SEG_TWO
    uint32_t J, O;  // relative to wb
    tag_step32(lo, hw, (uint32_t)lane, J, O);
#else
    const Tag t = parse_tag_bytes(lo, hw, p, slen, lane);
    uint32_t J = t.next < 0x7fffffff ? (uint32_t)t.next : 0x7fffffffu;  // relative to wb
    uint32_t O = t.len < (1 << 30) ? (uint32_t)t.len : (1u << 30);
#endif
    if (p >= hi) {  // the walk ends at the first chain position >= hi: a fixed point
      J = (uint32_t)lane;
      O = 0;
    }
#ifndef PQG_SNAP_SEG_TWO
    // One dword per position for the doubling: a terminal position (its next
    // tag outside the window, or itself >= hi: a fixed point) points at
    // itself; any other at its next tag, with that tag's output bytes (< 64
    // bytes of header and literal to stay in the window, so <= 64 output
    // bytes) in the bits above 8.  A round is then one ds_bpermute,
    // V = V[ptr] + (V's own sum): ptr follows, sums add (<= 63 * 64 < 2^24);
    // the terminal's exit and output bytes are read once at the end.  Rounds
    // stop when every pointer has reached a terminal.
    const bool term = p >= hi || J >= 64;
    const uint64_t tm = __ballot(term);
    uint32_t V = term ? (uint32_t)lane : (J | (O << 8));
#pragma unroll
    for (int r = 0; r < 6; r++) {
      if (!__ballot(!((tm >> (V & 63)) & 1))) break;
      const uint32_t W = bperm(V, (int)(V & 63));
      V = W + (V & ~0xffu);
    }
    const int64_t rel = x - wb;
    const bool here = act && rel < 64;
    const uint32_t Vx = bperm(V, here ? (int)rel : lane);
    const int T = (int)(Vx & 63);
    const uint32_t Jx = bperm(J, T), Ox = bperm(O, T);
    if (here) {
      x = wb + (int64_t)Jx;
      acc = sat_add(acc, sat_add(Vx >> 8, Ox));
    }
#else
    // positions >= hi are fixed points: a lane is done once J leaves the
    // window or reaches one (short tags need all six rounds, long ones few)
    const uint32_t jfix = hi - wb < 64 ? (uint32_t)(hi - wb) : 64u;
#pragma unroll
    for (int r = 0; r < 6; r++) {
#ifndef PQG_SNAP_ALL_ROUNDS
      if (!__ballot(J < jfix)) break;
#endif
      const bool in = J < 64;
      const uint32_t Jn = bperm(J, in ? (int)J : lane), On = bperm(O, in ? (int)J : lane);
      if (in) {
        J = Jn;
        O = sat_add(O, On);
      }
    }
    const int64_t rel = x - wb;
    const bool here = act && rel < 64;
    const uint32_t Jx = bperm(J, here ? (int)rel : lane), Ox = bperm(O, here ? (int)rel : lane);
    if (here) {
      x = wb + (int64_t)Jx;
      acc = sat_add(acc, Ox);
    }
#endif
  }
}
struct GlobalRd8 {
  gcu8 src;
  int64_t slen;
  __device__ __forceinline__ void operator()(int64_t p, uint32_t& lo, uint32_t& hi) const { ld8_block(src, slen, p, lo, hi); }
};
// bytes of a segment staged in LDS from block offset st_lo (16-byte aligned in
// memory); every position the walk of [b, hi) reads, < hi + 72, is staged
struct LdsRd8 {
  const PQG_L uint8_t* st;
  int64_t st_lo;
  __device__ __forceinline__ void operator()(int64_t p, uint32_t& lo, uint32_t& hi) const {
    const uint32_t o = (uint32_t)(p - st_lo);
    const PQG_L uint32_t* q = (const PQG_L uint32_t*)(st + (o & ~3u));
    const uint32_t a = q[0], b = q[1], c = q[2], sft = (o & 3) * 8;
    lo = __builtin_amdgcn_alignbit(b, a, sft);
    hi = __builtin_amdgcn_alignbit(c, b, sft);
  }
};
__device__ void chain_walk(gcu8 src, int64_t slen, int64_t hi, int64_t& x, uint32_t& acc) {
  chain_walk_rd(GlobalRd8{src, slen}, slen, hi, x, acc);
}

// SnapBlock keeps 32-bit block offsets: blocks (compressed or not) longer
// than this are UNSUPPORTED (page sizes are int32 in the page header; this
// leaves 1 MiB of headroom for the window and batch arithmetic)
constexpr int64_t kSnMaxLen = 0x7ff00000;
constexpr int32_t kSnNoWindow = -(1 << 30);  // in_base before the first fill

struct SnapBlock {
  gcu8 src;
  int32_t slen;
  gu8 dst;
  int32_t dlen;
  SnapShared* sh;
  // Block offsets and lengths are 32-bit (both lengths <= kSnMaxLen, checked
  // by the kernels): the scalar bookkeeping of every tag is then one
  // instruction per operation instead of a 64-bit pair or a VALU compare.
  int32_t d = 0;        // output bytes produced
  int32_t flushed = 0;  // output bytes stored (16-aligned until the end)
  int32_t in_base = kSnNoWindow;
  // A sub-block decode (k_snap_decode) produces the output [base, dend) only
  // and may read no output before base; the whole block is base 0, dend dlen.
  // Any tag that cannot be decoded that way (corrupt, or a copy reaching
  // before base) fails the decode, and the page is decoded serially.
  int32_t base = 0;
  int32_t dend = -1;
#ifdef PQG_PROFILE
  uint64_t pacc[24] = {0};
#define PQG_ST(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define PQG_SA(k, x) pacc[k] += (x)
#else
#define PQG_ST(v)
#define PQG_SA(k, x)
#endif

  // window [in_base, in_base + kSnWin) over the compressed block, 16-aligned in memory
  __device__ void fill(int32_t at) {
    const int lane = lane_id();
    in_base = at - (int32_t)(((uintptr_t)(src + at)) & 15);
    uint4 v[kSnWin / 1024];
#pragma unroll
    for (int h = 0; h < kSnWin / 1024; h++) {
      const int32_t g = in_base + 1024 * h + 16 * lane;
      // a granule holding a byte of [0, slen) is mapped (these loads stay
      // guarded: unconditional ones push the decoder past its 168 VGPRs; the
      // refills are ~1 % of its time, r04 session 10 counters)
      v[h] = (g < slen && g + 16 > 0) ? ldg16((uintptr_t)(src + g)) : make_uint4(0, 0, 0, 0);
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int h = 0; h < kSnWin / 1024; h++) sts16(lds_ptr(sh->in) + 1024 * h + 16 * lane, v[h]);
    __builtin_amdgcn_wave_barrier();
  }

  // store ring granules [flushed, upto) to dst (upto 16-aligned, or the end)
  __device__ void flush(int32_t upto) {
    const int lane = lane_id();
    __builtin_amdgcn_wave_barrier();
    for (int32_t g = flushed + 16 * lane; g < upto; g += 16 * 64) {
      const u32x4_t v = *(const PQG_L u32x4_t*)(lds_ptr(sh->ring) + (g & (kRing - 1)));
      stg16((uintptr_t)(dst + g), make_uint4(v.x, v.y, v.z, v.w));
    }
    flushed = upto;
  }
  __device__ __forceinline__ void maybe_flush() {
    const int32_t a = d & ~15;
    if (a - flushed >= kSnFlush) flush(a);
  }

  // A literal too long for one batch (or whose bytes leave the window):
  // pieces of up to kLongPiece bytes straight from the compressed block.
  __device__ void long_literal(int32_t at, int32_t len) {
    const int lane = lane_id();
    constexpr int NG = kLongPiece / 1024;  // granules per lane
    while (len > 0) {
      const int32_t a0 = d & ~15;
      const int pre = (int)(d - a0);
      const int32_t piece = len < kLongPiece - pre ? len : kLongPiece - pre;
      const int32_t lim = pre + piece;  // piece bytes are [pre, lim) of the granules from a0
      uint4 x[NG], y[NG];
      uint32_t r[NG];
      bool nx[NG], ny[NG];
#pragma unroll
      for (int j = 0; j < NG; j++) {
        const int32_t i0 = 1024 * j + 16 * lane;  // granule's first byte (relative to a0)
        const int32_t s0 = at + i0 - pre;         // block offset of that byte
        const uintptr_t sa = (uintptr_t)(src + s0);
        r[j] = (uint32_t)(sa & 15);
        const int32_t gb0 = s0 - (int32_t)r[j];   // aligned granule holding s0
        // load an aligned granule only if it holds a byte of the piece
        const int32_t lo = at + (i0 > pre ? i0 - pre : 0), hi = at + (i0 + 16 < lim ? i0 + 16 : lim) - pre;
        const bool need = i0 < lim && i0 + 16 > pre;
        // unconditional loads (a load under a branch is waited for inside it):
        // a granule not needed re-reads the literal's first one, zeroed below
        nx[j] = need && gb0 + 16 > lo;
        ny[j] = need && r[j] != 0 && gb0 + 16 < hi;
#if PQG_SNAPPY_LL_UNCOND
        const uintptr_t safe = (uintptr_t)(src + at) & ~(uintptr_t)15;
        x[j] = ldg16(nx[j] ? sa & ~(uintptr_t)15 : safe);
        y[j] = ldg16(ny[j] ? (sa & ~(uintptr_t)15) + 16 : safe);
#else
        x[j] = nx[j] ? ldg16(sa & ~(uintptr_t)15) : make_uint4(0, 0, 0, 0);
        y[j] = ny[j] ? ldg16((sa & ~(uintptr_t)15) + 16) : make_uint4(0, 0, 0, 0);
#endif
      }
#if PQG_SNAPPY_LL_UNCOND
#pragma unroll
      for (int j = 0; j < NG; j++) {
        if (!nx[j]) x[j] = make_uint4(0, 0, 0, 0);
        if (!ny[j]) y[j] = make_uint4(0, 0, 0, 0);
      }
#endif
#pragma unroll
      for (int j = 0; j < NG; j++) {
        const int32_t i0 = 1024 * j + 16 * lane;
        // (no early exit for lanes past the piece: every load is consumed on
        // every path, or the wait analysis keeps it pending into the next
        // tags and waits for all stores in flight there)
        const uint32_t q[8] = {x[j].x, x[j].y, x[j].z, x[j].w, y[j].x, y[j].y, y[j].z, y[j].w};
        const uint32_t qd = r[j] >> 2, sft = (r[j] & 3) * 8;
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          uint32_t lo_w = q[k], hi_w = q[k + 1];
#pragma unroll
          for (int m = 1; m < 4; m++) {
            lo_w = qd == (uint32_t)m ? q[m + k] : lo_w;
            hi_w = qd == (uint32_t)m ? q[m + k + 1 < 8 ? m + k + 1 : 7] : hi_w;
          }
          w[k] = __builtin_amdgcn_alignbit(hi_w, lo_w, sft);
        }
        const uint32_t rp = (uint32_t)((a0 + i0) & (kRing - 1));
        if (i0 < pre) {  // the granule's bytes before d are history: keep them
          const u32x4_t old = *(const PQG_L u32x4_t*)(lds_ptr(sh->ring) + rp);
          const uint32_t ow[4] = {old.x, old.y, old.z, old.w};
#pragma unroll
          for (int k = 0; k < 4; k++) {
            uint32_t m = 0;
#pragma unroll
            for (int e = 0; e < 4; e++) m |= (4 * k + e < pre ? 0xffu : 0u) << (8 * e);
            w[k] = (ow[k] & m) | (w[k] & ~m);
          }
        }
        if (i0 < lim) sts16(lds_ptr(sh->ring) + rp, make_uint4(w[0], w[1], w[2], w[3]));
      }
      __builtin_amdgcn_wave_barrier();
      d += piece;
      at += piece;
      len -= piece;
      maybe_flush();
    }
  }

  // A literal of len bytes at window offset wo (len <= kWinLit, inside the window).
  __device__ __forceinline__ void window_literal(uint32_t wo, int32_t len) {
    const int lane = lane_id();
    const int32_t a0 = d & ~15;
    const int pre = (int)(d - a0);
    const int lim = pre + (int)len;
    // A ragged first granule (pre > 0) is written byte by byte by lanes
    // pre..15, one byte each, so that its history bytes before d are never
    // read back (a read-modify-write would put a second LDS round trip on
    // every literal of the tag-by-tag path); the other granules go whole.
    // Both sets of source reads are issued before either write.
    const int so = (int)wo - pre + 16 * lane;
    const bool whole = 16 * lane < lim && (lane > 0 || pre == 0);
    const bool head = pre > 0 && lane >= pre && lane < 16 && lane < lim;
    // (lane 0 of a ragged literal may start up to 15 bytes before the window:
    // those offsets are clamped, the bytes are not written)
    const int hso = (int)wo - pre + lane;
    const PQG_L uint32_t* q = (const PQG_L uint32_t*)(lds_ptr(sh->in) + ((whole ? so : 0) & ~3));
    const uint32_t sft = (uint32_t)(so & 3) * 8;
    const uint32_t x0 = q[0], x1 = q[1], x2 = q[2], x3 = q[3], x4 = q[4];
    const uint8_t hb = lds_ptr(sh->in)[head ? hso : 0];
    if (head) lds_ptr(sh->ring)[(uint32_t)(a0 + lane) & (kRing - 1)] = hb;
    if (whole) {
      const uint32_t w[4] = {__builtin_amdgcn_alignbit(x1, x0, sft), __builtin_amdgcn_alignbit(x2, x1, sft),
                             __builtin_amdgcn_alignbit(x3, x2, sft), __builtin_amdgcn_alignbit(x4, x3, sft)};
      sts16(lds_ptr(sh->ring) + ((a0 + 16 * lane) & (kRing - 1)), make_uint4(w[0], w[1], w[2], w[3]));
    }
    d += len;
  }

  // Copy of len (<= 64) bytes from offset back, one byte per lane.
  __device__ __forceinline__ void copy_bytes(uint32_t off, int len) {
    const int lane = lane_id();
    const int32_t ring_lo = ((d + 15) & ~15) - kRing;  // see below
    int j = lane;
    if (off < (uint32_t)len) j = lane % (int)off;  // overlapping: the period of `off` bytes before d
    const int32_t h = d - (int32_t)off + j;          // (off <= d - base: checked by the callers)
    if (d - (int32_t)off >= ring_lo) {
      const uint8_t b = lds_ptr(sh->ring)[(uint32_t)h & (kRing - 1)];
      if (lane < len) lds_ptr(sh->ring)[(uint32_t)(d + lane) & (kRing - 1)] = b;
    } else {
      // older than the ring (copy-4): the flushed output through L2, once the
      // flush stores have landed and this CU's L1 holds no stale line
      // (off > kRing - 16 > len: no overlap)
      flush(d & ~15);
      __builtin_amdgcn_s_waitcnt(0);  // this wave's flush stores have reached L2
      // every lane loads (h < d for all 64: off > 64), so that no load is
      // left pending on a path the compiler cannot rule out (it would then
      // wait for every store in flight at the next write of that register)
      const uintptr_t a = (uintptr_t)(dst + h);
      const uint32_t bw = ld_l2_u32((const PQG_G uint32_t*)(a & ~(uintptr_t)3)) >> ((a & 3) * 8);
      asm volatile("" ::"v"(bw));  // consumed here, on every path
      if (lane < len) lds_ptr(sh->ring)[(uint32_t)(d + lane) & (kRing - 1)] = (uint8_t)bw;
    }
    d += len;
  }

  // peek8 in two halves: the LDS loads, then (after other work has been
  // issued behind them) the funnel shift and the move to scalar registers
  struct Peek {
    uint32_t a, b, c, sft;
  };
  __device__ __forceinline__ Peek peek_issue(int32_t t) {
    const uint32_t o = (uint32_t)(t - in_base);
    const PQG_L uint32_t* q = (const PQG_L uint32_t*)(lds_ptr(sh->in) + (o & ~3u));
    return Peek{q[0], q[1], q[2], (o & 3) * 8};
  }
  __device__ __forceinline__ uint64_t peek_finish(const Peek& p) {
    const uint32_t lo = __builtin_amdgcn_alignbit(p.b, p.a, p.sft), hi = __builtin_amdgcn_alignbit(p.c, p.b, p.sft);
    return (uint64_t)__builtin_amdgcn_readfirstlane(lo) | (uint64_t)__builtin_amdgcn_readfirstlane(hi) << 32;
  }
  // 8 bytes at block offset t (inside the window): one broadcast LDS load
  __device__ __forceinline__ uint64_t peek8(int32_t t) {
    const uint32_t o = (uint32_t)(t - in_base);
    const PQG_L uint32_t* q = (const PQG_L uint32_t*)(lds_ptr(sh->in) + (o & ~3u));
    const uint32_t a = q[0], b = q[1], c = q[2];
    const uint32_t sft = (o & 3) * 8;
    const uint32_t lo = __builtin_amdgcn_alignbit(b, a, sft), hi = __builtin_amdgcn_alignbit(c, b, sft);
    return (uint64_t)__builtin_amdgcn_readfirstlane(lo) | (uint64_t)__builtin_amdgcn_readfirstlane(hi) << 32;
  }

  // Up to max tags one at a time (tag-sparse stretches: long literals), the
  // next tag's header read ahead of the current tag's bytes.  Returns to the
  // windowed resolution after a streak of short tags or at a window refill.
  // kOK, or kSNAPPY at a corrupt tag.
  __device__ int serial(int32_t& s, int max) {
    // loads the dense path issued under one branch and consumed under another
    // look pending here to the compiler's wait analysis, which would then wait
    // for all stores in flight at every write of their registers: one real
    // wait here instead
    __builtin_amdgcn_s_waitcnt(0);
    int short_streak = 0;
    uint64_t x8 = peek8(s);
    const bool lastsub = dend == dlen;
    for (int n = 0; n < max && s < slen && short_streak < 4 && (lastsub || d < dend); n++) {
      PQG_ST(q0);
      PQG_SA(21, 1);
      const uint32_t tag = (uint32_t)x8 & 0xff;
      int64_t length;  // (a literal's length field is 32 bits: up to 2^32)
      int32_t ns;
      uint32_t offset = 0;
      const bool lit = (tag & 3) == 0;
      int hdr;
      if (lit) {
        uint32_t x = tag >> 2;
        hdr = 1;
        if (x >= 60) {
          const int nb = (int)x - 59;  // 1..4 length bytes
          hdr = 1 + nb;
          if (s + hdr > slen) return kSNAPPY;
          x = (uint32_t)(x8 >> 8) & (nb == 4 ? 0xffffffffu : ((1u << (8 * nb)) - 1));
        }
        length = (int64_t)x + 1;
        if (length > dend - d || length > slen - (s + hdr)) return kSNAPPY;
        ns = s + hdr + (int32_t)length;
      } else {
        hdr = (tag & 3) == 1 ? 2 : (tag & 3) == 2 ? 3 : 5;
        if (s + hdr > slen) return kSNAPPY;
        if ((tag & 3) == 1) {
          length = 4 + ((tag >> 2) & 7);
          offset = (tag & 0xe0) << 3 | ((uint32_t)(x8 >> 8) & 0xff);
        } else if ((tag & 3) == 2) {
          length = 1 + (tag >> 2);
          offset = (uint32_t)(x8 >> 8) & 0xffff;
        } else {
          length = 1 + (tag >> 2);
          offset = (uint32_t)(x8 >> 8);
        }
        if (offset == 0 || (int64_t)offset > d - base || length > dend - d) return kSNAPPY;
        ns = s + hdr;
      }
      short_streak = length < 16 ? short_streak + 1 : 0;
      const bool next_in = ns < slen && ns >= in_base && ns + kSnWinNeed <= in_base + kSnWin;
      // the next header's loads go out ahead of this tag's bytes and are
      // waited for after them (one LDS round trip per tag, not two)
      const Peek nx = peek_issue(next_in ? ns : in_base);
      PQG_ST(q1);
      PQG_SA(16, q1 - q0);
      if (lit) {
        const int32_t at = s + hdr;
        if ((d & 15) + length <= kWinLit && at + length <= in_base + kSnWin) window_literal((uint32_t)(at - in_base), (int32_t)length);
        else long_literal(at, (int32_t)length);
      } else {
        copy_bytes(offset, (int)length);
      }
      PQG_ST(q2);
      PQG_SA(lit ? 17 : 18, q2 - q1);
      maybe_flush();  // keeps the unflushed tail inside the ring
      PQG_ST(q3);
      PQG_SA(19, q3 - q2);
      s = ns;
      if (!next_in) break;
      x8 = peek_finish(nx);
      PQG_ST(q4);
      PQG_SA(20, q4 - q3);
    }
    if ((d & ~15) - flushed >= kSnFlush) flush(d & ~15);
    return kOK;
  }

  // decode_other.go:14-101 from tag position s (after the length varint).
  // The ring holds output [ring_lo, d), ring_lo = roundup16(d) - kRing: a
  // ragged last granule overwrites the slots of the kRing-older bytes just
  // above d.
  __device__ int run(int32_t s) {
    const int lane = lane_id();
    PQG_ST(t_run0);
    const PQG_L uint8_t* IN = lds_ptr(sh->in);
    int serial_next = 0;  // tags to take one at a time before the next windowed resolution
    if (dend < 0) dend = dlen;
    const bool lastsub = dend == dlen;  // the block's last sub-block: every tag up to slen is its own
    while (s < slen && (lastsub || d < dend)) {
      PQG_ST(ta);
      PQG_SA(8, 1);
      if (s < in_base || s + kSnWinNeed > in_base + kSnWin) {
        // pending output goes out with the window loads: one wait covers both
        if ((d & ~15) - flushed >= 2048) flush(d & ~15);
        fill(s);
      }
      PQG_ST(tb);
      PQG_SA(0, tb - ta);
      if (serial_next > 0) {
        const int e = serial(s, serial_next);
        PQG_ST(tsx);
        PQG_SA(7, tsx - tb);
        if (e) return e;
        serial_next = 0;
        continue;
      }
      // A batch: up to kBatchWin windows of kPos positions whose chain tags
      // fill <= kSpan output bytes, resolved together (step 4a).
      const int32_t a0 = d & ~15;
      const int pre = (int)(d - a0);
      int filled = pre;  // batch bytes [0, filled) from a0: history prefix + the tags so far
      int ntag = 0, nwin = 0;
      bool sparse_done = false;
      PQG_L uint8_t* TM = lds_ptr(sh->tmap);
      PQG_L u32x2_t* TE = lds_ptr(sh->tent);
      for (;;) {
        PQG_ST(tw);
        // ---- 1. speculative tags at positions lane and 64 + lane
        const uint32_t wo = (uint32_t)(s - in_base) + lane;
        const Tag t0 = parse_tag(IN, wo, s + lane, slen, lane);
        const Tag t1 = parse_tag(IN, wo + 64, s + 64 + lane, slen, 64 + lane);
        const int n0 = (t0.err || t0.next >= kPos) ? kPos : (int)t0.next;
        const int n1 = (t1.err || t1.next >= kPos) ? kPos : (int)t1.next;
        // ---- 2. the chain (pointer doubling, pqg_device.h); tags start before
        // the end of the block
        uint64_t cm0, cm1;
#if PQG_SNAPPY_SERIAL_CHAIN
        {  // A/B: the chain by a scalar v_readlane walk
          cm0 = cm1 = 0;
          int q = 0;
          while (q < kPos) {
            if (q < 64) {
              cm0 |= 1ull << q;
              q = __builtin_amdgcn_readlane(n0, q);
            } else {
              cm1 |= 1ull << (q - 64);
              q = __builtin_amdgcn_readlane(n1, q - 64);
            }
          }
        }
#else
        chain_marks128(n0, n1, lds_ptr(sh->cflag), cm0, cm1);
#endif
        const int32_t lim64 = slen - s;
        const int lim = lim64 < kPos ? (int)lim64 : kPos;
        if (lim < 64) {
          cm0 &= (1ull << lim) - 1;
          cm1 = 0;
        } else if (lim < kPos) {
          cm1 &= (1ull << (lim - 64)) - 1;
        }
        const int last = cm1 ? 127 - __builtin_clzll(cm1) : 63 - __builtin_clzll(cm0);
        const bool on0 = (cm0 >> lane) & 1, on1 = (cm1 >> lane) & 1;
        PQG_ST(tc);
        PQG_SA(1, tc - tw);
        // ---- 3. output offsets (from the batch's current end) and the reference's checks
        const uint32_t o0 = on0 ? (uint32_t)(t0.len < (1 << 30) ? t0.len : (1 << 30)) : 0u;
        const uint32_t o1 = on1 ? (uint32_t)(t1.len < (1 << 30) ? t1.len : (1 << 30)) : 0u;
        const uint32_t i0 = dpp_incl_add(o0);
        const uint32_t tot0 = (uint32_t)__builtin_amdgcn_readlane((int)i0, 63);
        const uint32_t i1 = dpp_incl_add(o1) + tot0;
        const int64_t st0 = (int64_t)(i0 - o0), st1 = (int64_t)(i1 - o1);  // output offsets (relative to a0 + filled)
        const int64_t dcur = a0 + filled;
        auto check = [&](const Tag& t, int64_t st, int64_t pos, bool& cut) {
          const int64_t dt = dcur + st;
          const bool past = !lastsub && dt >= dend;                       // the next sub-block's tag
          bool e = !past && (t.err || t.len > dend - dt);                 // length > len(dst)-d
          if (!t.lit) e |= !past && (t.info == 0 || (int64_t)t.info > dt - base);  // offset <= 0 || d < offset
          cut = past || filled + st + t.len > kSpan || (t.lit && pos + t.hdr + t.len > in_base + kSnWin);
          return e;
        };
        bool c0, c1;
        const bool e0 = check(t0, st0, s + lane, c0), e1 = check(t1, st1, s + 64 + lane, c1);
        if (__ballot(on0 && e0) | __ballot(on1 && e1)) return kSNAPPY;
        const uint64_t cb0 = __ballot(on0 && c0), cb1 = __ballot(on1 && c1);
        const int cutpos = cb0 ? __ffsll((long long)cb0) - 1 : cb1 ? 64 + __ffsll((long long)cb1) - 1 : kPos;
        if (cutpos == 0) {
          if (nwin > 0) break;  // the batch so far is resolved first
          // tag 0 alone is too long for a batch: a literal (copies are <= 64 bytes)
          const int32_t l0 = (int32_t)readlane64(t0.len, 0);  // (checked: <= dend - d)
          const int32_t at0 = s + __builtin_amdgcn_readlane(t0.hdr, 0);
          long_literal(at0, l0);
          s = at0 + l0;
          serial_next = 64;
          sparse_done = true;
          break;
        }
        // ---- the chain's tags before cutpos; output [dcur, dcur + out)
        const bool b0 = on0 && lane < cutpos, b1 = on1 && 64 + lane < cutpos;
        const uint64_t bm0 = __ballot(b0), bm1 = __ballot(b1);
        int32_t out, s1;  // (the chain's tags passed the checks: out <= kSpan)
        if (cutpos < kPos) {
          const int l = cutpos & 63;
          out = cutpos < 64 ? __builtin_amdgcn_readlane((int)(i0 - o0), l) : __builtin_amdgcn_readlane((int)(i1 - o1), l);
          s1 = s + cutpos;
        } else {
          out = __builtin_amdgcn_readlane((int)i1, 63);
          s1 = s + (int32_t)readlane64(last < 64 ? t0.next : t1.next, last & 63);
        }
        PQG_ST(td);
        PQG_SA(2, td - tc);
        const int cnt = __popcll(bm0) + __popcll(bm1);
        if (nwin == 0 && cnt < kDense) {
          PQG_SA(10, 1);
          // ---- 4b. sparse: tag by tag, with the fields already parsed
          uint64_t m0 = bm0, m1 = bm1;
          while (m0 | m1) {
            const bool hi = m0 == 0;
            const int l = __ffsll((long long)(hi ? m1 : m0)) - 1;
            if (hi) m1 &= m1 - 1;
            else m0 &= m0 - 1;
            const int32_t len = (int32_t)readlane64(hi ? t1.len : t0.len, l);
            const bool lit = __builtin_amdgcn_readlane((int)(hi ? t1.lit : t0.lit), l) != 0;
            if (lit) {
              const int32_t at = s + (hi ? 64 : 0) + l + __builtin_amdgcn_readlane(hi ? t1.hdr : t0.hdr, l);
              if ((d & 15) + len <= kWinLit) window_literal((uint32_t)(at - in_base), len);
              else long_literal(at, len);
            } else {
              copy_bytes((uint32_t)__builtin_amdgcn_readlane((int)(hi ? t1.info : t0.info), l), (int)len);
            }
            maybe_flush();
          }
          s = s1;
          if ((d & ~15) - flushed >= kSnFlush) flush(d & ~15);
          serial_next = 64;  // a tag-sparse stretch: continue tag by tag
          PQG_ST(tsp);
          PQG_SA(3, tsp - td);
          sparse_done = true;
          break;
        }
        if (nwin == 0) {
          *(PQG_L u32x4_t*)(TM + 16 * lane) = u32x4_t{0u, 0u, 0u, 0u};
          __builtin_amdgcn_wave_barrier();
        }
        // this window's tags: entries ntag.. in chain order (marks 1 + entry at
        // the tag's first output byte)
        const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
        const int r0 = ntag + __popcll(bm0 & below), r1 = ntag + __popcll(bm0) + __popcll(bm1 & below);
        if (b0) {
          TE[r0] = u32x2_t{(uint32_t)(filled + (int)st0),
                           t0.lit ? (0x80000000u | (uint32_t)(s + lane + t0.hdr - in_base)) : t0.info};
          TM[filled + st0] = (uint8_t)(r0 + 1);
        }
        if (b1) {
          TE[r1] = u32x2_t{(uint32_t)(filled + (int)st1),
                           t1.lit ? (0x80000000u | (uint32_t)(s + 64 + lane + t1.hdr - in_base)) : t1.info};
          TM[filled + st1] = (uint8_t)(r1 + 1);
        }
        ntag += cnt;
        filled += (int)out;
        s = s1;
        nwin++;
        // another window into the same batch: the whole window was taken, room
        // is left, and its positions (and most literals) are in the LDS window
        if (cutpos < kPos || nwin >= kBatchWin || filled > kSpan - kBatchRoom || s >= slen ||
            s + kSnWinNeed / 2 > in_base + kSnWin || (!lastsub && a0 + filled >= dend))
          break;
      }
      if (sparse_done) continue;
      PQG_ST(td);
      PQG_SA(9, 1);
      PQG_SA(12, ntag);
      // ---- 4a. dense: per-byte sources for the granules from a0
      const int end = filled;  // batch bytes [pre, end)
      const int32_t d1 = a0 + filled;
      __builtin_amdgcn_wave_barrier();
      // tag of each of this lane's 16 bytes: running max of the marks, then
      // the exclusive max over the lanes before
      const u32x4_t mk = *(const PQG_L u32x4_t*)(TM + 16 * lane);
      const uint32_t mw[4] = {mk.x, mk.y, mk.z, mk.w};
      uint32_t tix[16];
      uint32_t run_max = 0;
#pragma unroll
      for (int k = 0; k < 16; k++) {
        const uint32_t m = (mw[k >> 2] >> (8 * (k & 3))) & 0xff;
        run_max = m > run_max ? m : run_max;
        tix[k] = run_max;
      }
      const uint32_t before = dpp_prev(dpp_incl_max(run_max));
      int32_t own[16];
#pragma unroll
      for (int k = 0; k < 16; k++) {
        const int idx = 16 * lane + k;
        const uint32_t t = (tix[k] > before ? tix[k] : before) - 1;
        const u32x2_t te = TE[t & (kBatchTags - 1)];  // one load for both fields: no load under a branch
        const int32_t st = (int32_t)te.x;
        const uint32_t inf = te.y;
        const int32_t v = (inf & 0x80000000u) ? kSpan + (int32_t)(inf & 0x7fffffffu) + (idx - st) : idx - (int32_t)inf;
        // history bytes before d stay as they are; bytes past the batch read any terminal
        own[k] = idx < pre ? idx : idx >= end ? kSpan : v;
      }
      PQG_ST(te);
      PQG_SA(4, te - td);
      // Sources older than the ring (copy offsets past kRing, ~20 % of C4's
      // copies): the flushed output through L2 (sc1 loads bypass this CU's L1,
      // whose lines may predate later stores), issued now so that their
      // latency runs under the pointer doubling.  Only this wave's flush
      // stores need to have landed; the previous batch's went out a batch ago,
      // and this batch's pending output is flushed after these loads.
      const int32_t ring_lo = ((d + 15) & ~15) - kRing;
      uint32_t fm = 0;  // bytes whose (terminal) source is far
#pragma unroll
      for (int k = 0; k < 16; k++) fm |= (own[k] < pre && a0 + own[k] < ring_lo) ? 1u << k : 0u;
      uint32_t fw[16];
      const bool any_far = __ballot(fm != 0) != 0;
      if (any_far) {
        PQG_SA(14, 1);
        __builtin_amdgcn_s_waitcnt(0);
#pragma unroll
        for (int k = 0; k < 16; k++) {  // unconditional loads (non-far bytes read the output's first dword)
          const int32_t h = (fm >> k) & 1 ? a0 + own[k] : 0;
          fw[k] = ld_l2_u32((const PQG_G uint32_t*)((uintptr_t)(dst + h) & ~(uintptr_t)3));
        }
      }
      maybe_flush();  // the output before this batch
      PQG_ST(te2);
      PQG_SA(11, te2 - te);
      // same-batch copy sources: pointer doubling over src[]
      bool chase = false;
#pragma unroll
      for (int k = 0; k < 16; k++) chase |= own[k] >= pre && own[k] < kSpan;
      if (__ballot(chase)) {
        // byte x's source at S[(x % 16) * 64 + x / 16]: lane L's byte k at
        // k * 64 + L, so each store instruction writes 64 consecutive dwords,
        // and a gather of a nearby byte (copy offsets are mostly short) by
        // consecutive lanes reads consecutive dwords: no bank conflicts
        // (byte-major, lane stride 16 dwords, every gather of the doubling
        // was a 16-way conflict)
        PQG_L int32_t* S = lds_ptr(sh->src);
        for (int r = 0; r < 11; r++) {
#pragma unroll
          for (int k = 0; k < 16; k++) S[64 * k + lane] = own[k];
          __builtin_amdgcn_wave_barrier();
          chase = false;
#pragma unroll
          for (int k = 0; k < 16; k++) {
            // unconditional loads (a guarded load would wait on its own)
            const bool in = own[k] >= pre && own[k] < kSpan;
            const int32_t x = in ? own[k] : 0;
            const int32_t nv = S[((x & 15) << 6) | (x >> 4)];
            own[k] = in ? nv : own[k];
            chase |= own[k] >= pre && own[k] < kSpan;
          }
          __builtin_amdgcn_wave_barrier();
          PQG_SA(13, 1);
          if (!__ballot(chase)) break;
        }
      }
      PQG_ST(tf);
      PQG_SA(5, tf - te2);
      // every byte reads its source once: the window or the ring (one LDS
      // byte load at a computed address), or, older than the ring, L2
      const PQG_L uint8_t* shb = (const PQG_L uint8_t*)lds_ptr(sh->ring);  // the ring is at offset 0
      const uint32_t in_off = (uint32_t)(IN - shb);
      uint32_t bt[16];
      uint32_t fm2 = 0;  // far sources found by the doubling (a copy of a far copy in this batch)
#pragma unroll
      for (int k = 0; k < 16; k++) {
        const int32_t v = own[k];
        const int32_t h = a0 + v;
        const uint32_t off = v >= kSpan ? in_off + (uint32_t)(v - kSpan) : (uint32_t)(h & (kRing - 1));
        fm2 |= (v < kSpan && h < ring_lo && !((fm >> k) & 1)) ? 1u << k : 0u;
        bt[k] = shb[off];
      }
      if (any_far) {
#pragma unroll
        for (int k = 0; k < 16; k++)
          if ((fm >> k) & 1) bt[k] = (fw[k] >> (((uintptr_t)(dst + a0 + own[k]) & 3) * 8)) & 0xff;
      }
      if (__ballot(fm2 != 0)) {
        __builtin_amdgcn_s_waitcnt(0);
#pragma unroll
        for (int k = 0; k < 16; k++) {
          const int32_t h = (fm2 >> k) & 1 ? a0 + own[k] : 0;
          fw[k] = ld_l2_u32((const PQG_G uint32_t*)((uintptr_t)(dst + h) & ~(uintptr_t)3));
        }
#pragma unroll
        for (int k = 0; k < 16; k++)
          if ((fm2 >> k) & 1) bt[k] = (fw[k] >> (((uintptr_t)(dst + a0 + own[k]) & 3) * 8)) & 0xff;
      }
      __builtin_amdgcn_wave_barrier();
      if (16 * lane < end) {
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; k++) w[k] = bt[4 * k] | bt[4 * k + 1] << 8 | bt[4 * k + 2] << 16 | bt[4 * k + 3] << 24;
        sts16(lds_ptr(sh->ring) + ((a0 + 16 * lane) & (kRing - 1)), make_uint4(w[0], w[1], w[2], w[3]));
      }
      __builtin_amdgcn_wave_barrier();
      d = d1;  // flushed by the next batch (after its far loads) or the next path
      PQG_ST(tg);
      PQG_SA(6, tg - tf);
    }
    PQG_ST(t_run1);
    PQG_SA(15, t_run1 - t_run0);
    if (d != dend) return kSNAPPY;
    flush((dend + 15) & ~15);
    return kOK;
  }

  // Follow the tag chain from s (output d) to the tag whose output starts at
  // `target`, without producing output: the start of a sub-block found from a
  // chain tag before it.  kSNAPPY if a tag straddles target or the chain
  // leaves the block.
  __device__ int skip_to(int32_t& s, int32_t target) {
    const int lane = lane_id();
    const PQG_L uint8_t* IN = lds_ptr(sh->in);
    while (d < target) {
      if (s >= slen) return kSNAPPY;
      if (s < in_base || s + kSnWinNeed > in_base + kSnWin) fill(s);
      const uint32_t wo = (uint32_t)(s - in_base) + lane;
      const Tag t0 = parse_tag(IN, wo, s + lane, slen, lane);
      const Tag t1 = parse_tag(IN, wo + 64, s + 64 + lane, slen, 64 + lane);
      const uint32_t n0 = (uint32_t)(t0.next < kPos ? t0.next : kPos), n1 = (uint32_t)(t1.next < kPos ? t1.next : kPos);
      const uint32_t l0 = (uint32_t)(t0.len < (1 << 30) ? t0.len : (1 << 30)),
                     l1 = (uint32_t)(t1.len < (1 << 30) ? t1.len : (1 << 30));
      const int32_t lim64 = slen - s;
      const int lim = lim64 < kPos ? (int)lim64 : kPos;
      int p = 0;
      while (p < lim && d < target) {
        const bool h = p >= 64;
        const int l = p & 63;
        const uint32_t len = (uint32_t)__builtin_amdgcn_readlane((int)(h ? l1 : l0), l);
        const bool er = __builtin_amdgcn_readlane((int)(h ? t1.err : t0.err), l) != 0;
        if (er || d + (int64_t)len > target) return kSNAPPY;
        d += len;
        const int np = __builtin_amdgcn_readlane((int)(h ? n1 : n0), l);
        if (np >= kPos) {  // the tag's bytes run past the parsed positions
          s += h ? readlane64(t1.next, l) : readlane64(t0.next, l);
          p = -1;
          break;
        }
        p = np;
      }
      if (p >= 0) s += p;
    }
    return d == target ? kOK : kSNAPPY;
  }
};

// The compressed block of a page: V2 pages keep their level bytes raw in
// front of it (page_v2.go:110-123).
struct SnapLoc {
  int64_t src_off, clen, ulen;
};
__device__ __forceinline__ SnapLoc snap_loc(const PageDev& pg) {
  SnapLoc L{pg.payload_offset, pg.csize, pg.usize};
  if (pg.page_type == 3) {
    int32_t levels = (int32_t)((uint32_t)pg.rep_len + (uint32_t)pg.def_len);
    if (levels > 0) L.src_off += levels;
    L.clen = (int32_t)((uint32_t)pg.csize - (uint32_t)levels);
    L.ulen = (int32_t)((uint32_t)pg.usize - (uint32_t)levels);
  }
  return L;
}

// decodedLen: binary.Uvarint over the block (decode.go:32-43); kOK, kSNAPPY or
// kSIZE (a length other than the page's uncompressed size)
template <class RD>
__device__ __forceinline__ int snappy_header(RD byte_at, int64_t clen, int64_t ulen, int* hl) {
  uint64_t v = 0;
  int e = kOK;
  unsigned sft = 0;
  *hl = 0;
  for (int i = 0;; i++) {
    if (i >= clen) return kSNAPPY;
    const int b = byte_at(i);
    if (b < 0x80) {
      if (i > 9 || (i == 9 && b > 1)) e = kSNAPPY;
      else v |= (sft < 64 ? (uint64_t)b << sft : 0);
      *hl = i + 1;
      break;
    }
    if (sft < 64) v |= (uint64_t)(b & 0x7f) << sft;
    sft += 7;
  }
  if (e == kOK && v > 0xffffffffull) e = kSNAPPY;
  if (e == kOK && (int64_t)v != ulen) e = kSIZE;
  return e;
}

// ============================================================================
// K2 split: every compressed page is decoded as 64 KiB output sub-blocks, one
// wave each.  golang/snappy's Encode — the reference writer's snappyCompressor
// (compress.go:42-44, vendor/github.com/golang/snappy/encode.go:18-41) — and
// the C++ snappy behind other writers encode independent 64 KiB blocks, so a
// sub-block's copies stay inside it and its first tag starts exactly at
// j * 64 KiB of output.  Where a stream does not have that shape (or is
// corrupt) a sub-block decode fails and the page is decoded serially from the
// start by k_snappy, which also reports the reference's error.
//   k_snap_plan   per page: length varint, sub-block and segment table slots
//   k_snap_seg    per 4 KiB segment of a big block: the chain exit and output
//                 bytes from each of the segment's first 64 positions
//   k_snap_link   per big page: chain the segment exits -> a chain tag at or
//                 before every sub-block start
//   k_snap_decode per sub-block: skip to its start, decode it (SnapBlock)
//   k_snappy      pages whose split failed: the whole block on one wave
// ============================================================================
__global__ void __launch_bounds__(256) k_snap_plan(const JobDev* jobs, PageDev* pages, const int* list,
                                                   const int* total, int* ctr, SnapSub* subs, int sub_cap,
                                                   int* seg_page, int seg_cap) {
  __shared__ int64_t part[5];
  __shared__ int s_base[2];
  const int n = *total;
  for (int b0 = blockIdx.x * 256; b0 < n; b0 += gridDim.x * 256) {
    const int t = b0 + (int)threadIdx.x;
    int nsub = 0, nseg = 0, hdr = 0, fb = 0;
    int pidx = -1;
    bool split = false;
    if (t < n) {
      pidx = list[t];
      PageDev& pg = pages[pidx];
      // snappy pages only (GZIP pages: k_inflate); every other page leaves here
      // with an empty split (nsub = nseg = 0, no fallback)
      if (pg.read_status == kOK && pg.scratch_offset >= 0 && jobs[pg.job].codec == kCodecSnappy) {
        const JobDev& job = jobs[pg.job];
        const SnapLoc L = snap_loc(pg);
        const PQG_G uint8_t* src = gconst(job.data) + L.src_off;
        const int e = snappy_header([&](int i) { return (int)src[i]; }, L.clen, L.ulen, &hdr);
        if (e != kOK) {
          pg.read_status = e;
        } else if (pg.page_type == 0 && !values_supported(job.type, job.type_length, pg.encoding)) {
          fb = 1;  // V1: the values decoder is chosen after decompression (page_v1.go:91-97)
        } else {
          split = true;
          nsub = L.ulen > 0 ? (int)((L.ulen + kSnapSub - 1) / kSnapSub) : 1;
          nseg = nsub > 1 ? (int)((L.clen - hdr + kSnapSeg - 1) / kSnapSeg) : 0;
        }
      }
    }
    int64_t tsub, tseg;
    const int64_t esub = block_excl_scan<256>(nsub, &tsub, part);
    const int64_t eseg = block_excl_scan<256>(nseg, &tseg, part);
    if (threadIdx.x == 0) {
      s_base[0] = tsub ? atomicAdd(ctr, (int)tsub) : 0;
      s_base[1] = tseg ? atomicAdd(ctr + 1, (int)tseg) : 0;
    }
    __syncthreads();
    if (t < n) {
      PageDev& pg = pages[pidx];
      const int64_t sb = s_base[0] + esub, gb = s_base[1] + eseg;
      if (split && (sb + nsub > sub_cap || gb + nseg > seg_cap)) {
        split = false;
        fb = 1;  // tables full: the serial path
        // the slots this page was given that exist: marked empty, so that
        // k_snap_decode (which reads every slot < min(total, cap)) skips them
        for (int j = 0; j < nsub && sb + j < sub_cap; j++) subs[sb + j] = SnapSub{pidx, j, -1, 0};
      }
      if (split) {
        for (int j = 0; j < nsub; j++) subs[sb + j] = SnapSub{pidx, j, j == 0 ? hdr : -1, 0};
        for (int k = 0; k < nseg; k++) seg_page[gb + k] = pidx;
      }
      pg.sn_hdr = hdr;
      pg.sn_nsub = split ? nsub : 0;
      pg.sn_sub_base = (int32_t)sb;
      pg.sn_nseg = split ? nseg : 0;
      pg.sn_seg_base = (int32_t)gb;
      pg.sn_fallback = fb;
    }
    __syncthreads();
  }
}

// One wave per segment [b, b + 4 KiB) of a big block: from each entry b + lane
// the chain position where the tag chain leaves the segment, and the output
// bytes of the tags on the way.  The true chain enters a segment within its
// first 64 bytes unless a literal longer than that ends inside it.
__global__ void __launch_bounds__(64) k_snap_seg(const JobDev* jobs, const PageDev* pages, const int* seg_page,
                                                 const int* seg_total, int seg_cap, uint2* F) {
  constexpr int kStG = (kSnapSeg + 16 + 72 + 1023) / 1024;  // staged KiB: the segment, its alignment, the read-ahead
  __shared__ __attribute__((aligned(16))) uint8_t st[kStG * 1024 + 16];
  const int lane = lane_id();
  const int n = min(*seg_total, seg_cap);
  for (int g = blockIdx.x; g < n; g += gridDim.x) {
    const int pidx = __builtin_amdgcn_readfirstlane(seg_page[g]);
    const PageDev pg = pages[pidx];
    const JobDev job = jobs[pg.job];
    const SnapLoc L = snap_loc(pg);
    const int64_t b = pg.sn_hdr + (int64_t)(g - pg.sn_seg_base) * kSnapSeg;
    const int64_t hi = b + kSnapSeg < L.clen ? b + kSnapSeg : L.clen;
    const gcu8 src = gconst(job.data) + L.src_off;
    // the segment in LDS with one round of loads (granules holding a block
    // byte are mapped; the others read as zero)
    const int64_t st_lo = b - (int64_t)(((uintptr_t)(src + b)) & 15);
    uint4 v[kStG];
    const uintptr_t safe = (uintptr_t)src & ~(uintptr_t)15;  // unconditional loads (see SnapBlock::fill)
#pragma unroll
    for (int k = 0; k < kStG; k++) {
      const int64_t o = st_lo + 16 * (int64_t)(lane + 64 * k);
      v[k] = ldg16((o < L.clen && o + 16 > 0) ? (uintptr_t)(src + o) : safe);
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < kStG; k++) {
      const int64_t o = st_lo + 16 * (int64_t)(lane + 64 * k);
      sts16(lds_ptr(st) + 16 * (lane + 64 * k), (o < L.clen && o + 16 > 0) ? v[k] : make_uint4(0u, 0u, 0u, 0u));
    }
    __builtin_amdgcn_wave_barrier();
    int64_t x = b + lane;
    uint32_t acc = 0;
    chain_walk_rd(LdsRd8{lds_ptr(st), st_lo}, L.clen, hi, x, acc);
    F[(int64_t)g * 64 + lane] = make_uint2(x < 0x7fffffff ? (uint32_t)x : 0x7fffffffu, acc);
    __builtin_amdgcn_wave_barrier();
  }
}

// One wave per big page: the tag chain from the first tag, hopping a segment
// at a time through the exits of k_snap_seg (an entry past a segment's first
// 64 bytes — after a long literal — walks that segment here), recording for
// each sub-block the last chain tag at or before its first output byte.  A
// chain that does not end exactly at the block's end with the page's
// uncompressed size sends the page to the serial path.
__global__ void __launch_bounds__(64) k_snap_link(const JobDev* jobs, PageDev* pages, const int* list,
                                                  const int* total, SnapSub* subs, const uint2* F) {
  const int lane = lane_id();
  const int n = *total;
  for (int t = blockIdx.x; t < n; t += gridDim.x) {
    const int pidx = __builtin_amdgcn_readfirstlane(list[t]);
    const PageDev pg = pages[pidx];
    if (pg.read_status != kOK || pg.scratch_offset < 0 || pg.sn_fallback || pg.sn_nsub <= 1) continue;
    const JobDev job = jobs[pg.job];
    const SnapLoc L = snap_loc(pg);
    gcu8 src = gconst(job.data) + L.src_off;
    const int nseg = pg.sn_nseg, nsub = pg.sn_nsub;
    const int64_t hdr = pg.sn_hdr;
    const uint2* Fp = F + (int64_t)pg.sn_seg_base * 64;
    int64_t e = hdr, o = 0;
    int j = 1;  // sub-block 0 starts at the first tag (k_snap_plan)
    int why = 0;  // sn_fallback reason (diagnostics: pqg_page_info.flags >> 8)
    // rows of 8 segments at a time (lane = entry), the next 8 loaded ahead
    int kb = 0;
    uint2 ra[8], rb[8];
#pragma unroll
    for (int r = 0; r < 8; r++) {
      ra[r] = r < nseg ? Fp[(int64_t)r * 64 + lane] : make_uint2(0, 0);
      rb[r] = 8 + r < nseg ? Fp[(int64_t)(8 + r) * 64 + lane] : make_uint2(0, 0);
    }
    while (e < L.clen) {
      const int k = (int)((e - hdr) / kSnapSeg);
      if (k >= nseg) {
        why = 4;
        break;
      }
      const int64_t b = hdr + (int64_t)k * kSnapSeg;
      const int rel = (int)(e - b);
      int64_t x;
      uint32_t out;
      if (rel < 64) {
        if (k >= kb + 16 || k < kb) {  // a jump (long literal): reload both row sets
          kb = k;
#pragma unroll
          for (int r = 0; r < 8; r++) {
            ra[r] = kb + r < nseg ? Fp[(int64_t)(kb + r) * 64 + lane] : make_uint2(0, 0);
            rb[r] = kb + 8 + r < nseg ? Fp[(int64_t)(kb + 8 + r) * 64 + lane] : make_uint2(0, 0);
          }
        } else if (k >= kb + 8) {  // advance by 8: the prefetched set becomes current
          kb += 8;
#pragma unroll
          for (int r = 0; r < 8; r++) {
            ra[r] = rb[r];
            rb[r] = kb + 8 + r < nseg ? Fp[(int64_t)(kb + 8 + r) * 64 + lane] : make_uint2(0, 0);
          }
        }
        uint2 row = ra[0];
#pragma unroll
        for (int r = 1; r < 8; r++) row = k - kb == r ? ra[r] : row;
        x = (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)row.x, rel);
        out = (uint32_t)__builtin_amdgcn_readlane((int)row.y, rel);
      } else {
        x = e;
        out = 0;
        chain_walk(src, L.clen, b + kSnapSeg < L.clen ? b + kSnapSeg : L.clen, x, out);
        x = (int64_t)__builtin_amdgcn_readfirstlane((int)x);
        out = (uint32_t)__builtin_amdgcn_readfirstlane((int)out);
      }
      while (j < nsub && (int64_t)j * kSnapSub < o + (int64_t)out) {
        if (lane == 0) subs[pg.sn_sub_base + j] = SnapSub{pidx, j, (int32_t)e, (int32_t)o};
        j++;
      }
      if (x <= e || out >= 0x7fffffffu) {
        why = 8;
        break;
      }
      e = x;
      o += out;
      if (o > L.ulen) {
        why = 16;
        break;
      }
    }
    if (!why && (e != L.clen || o != L.ulen || j != nsub)) why = 32;
    if (why && lane == 0) pages[pidx].sn_fallback = why;
  }
}

__global__ void __launch_bounds__(64, PQG_SNAPPY_WPE) k_snap_decode(const JobDev* jobs, PageDev* pages, const SnapSub* subs,
                                                    const int* sub_total, int sub_cap, int* queue, uint8_t* scratch) {
  __shared__ __attribute__((aligned(16))) SnapShared sh;
  const int lane = lane_id();
  const int n = min(*sub_total, sub_cap);
  for (;;) {
    const int t = queue_next(queue);
    if (t >= n) return;
    const SnapSub sb = subs[t];
    const PageDev pg = pages[sb.page];
    if (pg.sn_fallback || sb.pos < 0) continue;
    const JobDev job = jobs[pg.job];
    const SnapLoc L = snap_loc(pg);
    if (L.clen > kSnMaxLen || L.ulen > kSnMaxLen) {  // the serial path reports it
      if (lane == 0) atomicOr(&pages[sb.page].sn_fallback, 64);
      continue;
    }
    SnapBlock blk{gconst(job.data) + L.src_off, (int32_t)L.clen, gmut(scratch) + job.scratch_base + pg.scratch_offset,
                  (int32_t)L.ulen, &sh};
    blk.base = sb.j * kSnapSub;
    blk.dend = (int64_t)blk.base + kSnapSub < L.ulen ? blk.base + kSnapSub : (int32_t)L.ulen;
    int32_t s = sb.pos;
    blk.d = sb.out;
    int e = blk.d < blk.base ? blk.skip_to(s, blk.base) : (blk.d == blk.base ? kOK : kSNAPPY);
    int why = e != kOK ? 64 : 0;
    blk.d = blk.flushed = blk.base;
    if (e == kOK) {
      e = blk.run(s);
      if (e != kOK) why = 128;
    }
#ifdef PQG_PROFILE
    for (int k = 0; k < 24; k++) PQG_ACC(k, 0, blk.pacc[k]);
#endif
    if (why && lane == 0) atomicOr(&pages[sb.page].sn_fallback, why);
  }
}

// The serial path: pages whose split decode failed (k_snap_plan / k_snap_link
// / k_snap_decode set sn_fallback), decoded from the start on one wave.
__global__ void __launch_bounds__(64, PQG_SNAPPY_WPE) k_snappy(JobDev* jobs, PageDev* pages, const int* list, const int* total,
                                               int* queue, uint8_t* scratch) {
  __shared__ __attribute__((aligned(16))) SnapShared sh;
  const int lane = lane_id();
  for (;;) {
    const int t = queue_next(queue);
    if (t >= *total) return;
    const int pidx = __builtin_amdgcn_readfirstlane(list[t]);
    const PageDev pg = pages[pidx];  // locals via scalar loads (see k_levels_expand)
    if (pg.read_status != kOK || pg.scratch_offset < 0 || !pg.sn_fallback) continue;
    const SnapLoc L = snap_loc(pg);
    const JobDev job = jobs[pg.job];
    if (job.codec != kCodecSnappy) continue;
    if (L.clen > kSnMaxLen || L.ulen > kSnMaxLen) {  // beyond SnapBlock's 32-bit offsets
      if (lane == 0) pages[pidx].read_status = kUNSUPPORTED;
      continue;
    }
    SnapBlock blk{gconst(job.data) + L.src_off, (int32_t)L.clen, gmut(scratch) + job.scratch_base + pg.scratch_offset,
                  (int32_t)L.ulen, &sh};
    int hl = 0;
    blk.fill(0);
    int e = snappy_header([&](int i) { return (int)lds_ptr(sh.in)[i - blk.in_base]; }, L.clen, L.ulen, &hl);
    if (e == kOK) e = blk.run(hl);
#ifdef PQG_PROFILE
    for (int k = 0; k < 24; k++) PQG_ACC(k, 0, blk.pacc[k]);
#endif
    // V1: getValuesDecoder runs after the block is decompressed (page_v1.go:91-97)
    if (e == kOK && pg.page_type == 0 && !values_supported(job.type, job.type_length, pg.encoding)) e = kUNSUPPORTED;
    if (lane == 0 && e != kOK) pages[pidx].read_status = e;
  }
}

}  // namespace pqg
