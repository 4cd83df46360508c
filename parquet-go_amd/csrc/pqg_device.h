// pqg_device.h — wave-level building blocks of the gfx950 decoder.
#pragma once
#include <hip/hip_runtime.h>

#include "pqg_common.h"

// Address-space typed pointers.  Pointers loaded from memory (JobDev.data,
// HStream.p, ...) are generic to the compiler, and generic accesses become
// FLAT instructions, which count in both vmcnt and lgkmcnt: every LDS wait then
// also waits for all outstanding global loads and stores.  Hot code therefore
// converts them to global (address space 1) once, at the load of the pointer.
#define PQG_G __attribute__((address_space(1)))
#define PQG_L __attribute__((address_space(3)))

namespace pqg {

typedef const PQG_G uint8_t* gcu8;
typedef PQG_G uint8_t* gu8;
template <class T>
__device__ __forceinline__ const PQG_G T* gconst(const T* p) { return (const PQG_G T*)p; }
template <class T>
__device__ __forceinline__ PQG_G T* gmut(T* p) { return (PQG_G T*)p; }
template <class T>
__device__ __forceinline__ PQG_L T* lds_ptr(T* p) { return (PQG_L T*)p; }

// 16 / 8-byte global and LDS accesses (HIP's uint4 class does not copy out of
// an address-space-qualified lvalue, a clang vector type does).
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 ldg16(uintptr_t a) {
  const u32x4_t v = *(const PQG_G u32x4_t*)a;
  return make_uint4(v.x, v.y, v.z, v.w);
}
// streaming read (non-temporal): data read once, kept out of the L2's way
__device__ __forceinline__ uint4 ldg16_nt(uintptr_t a) {
  const u32x4_t v = __builtin_nontemporal_load((const PQG_G u32x4_t*)a);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void stg16(uintptr_t a, uint4 x) {
  const u32x4_t v = {x.x, x.y, x.z, x.w};
  *(PQG_G u32x4_t*)a = v;
}
// Decoded-output stores: the outputs are not read again by the pipeline, so
// they are stored non-temporally (PQG_NT_OUT, default on: the L2 keeps what
// later kernels re-read -- dictionaries, run tables, pages; C2 3.31 -> 3.25 ms
// with k_dict4's stores, r04 session 15).
#ifndef PQG_NT_OUT
#define PQG_NT_OUT 1
#endif
__device__ __forceinline__ void stg16o(uintptr_t a, uint4 x) {
#if PQG_NT_OUT
  const u32x4_t v = {x.x, x.y, x.z, x.w};
  __builtin_nontemporal_store(v, (PQG_G u32x4_t*)a);
#else
  stg16(a, x);
#endif
}
__device__ __forceinline__ void stg8(uintptr_t a, uint32_t lo, uint32_t hi) {
  const u32x2_t v = {lo, hi};
  *(PQG_G u32x2_t*)a = v;
}
__device__ __forceinline__ void sts16(PQG_L void* a, uint4 x) {
  const u32x4_t v = {x.x, x.y, x.z, x.w};
  *(PQG_L u32x4_t*)a = v;
}

// Agent-scope relaxed load: `global_load_dword … sc1`, served by L2 and never
// by this CU's L1 (MI355X_MICROARCH.md, fence table).  Reading bytes this wave
// stored earlier needs only its own `s_waitcnt vmcnt(0)` before it — no
// acquire fence, which would invalidate the whole CU's L1 (≈1.7 µs).
__device__ __forceinline__ uint32_t ld_l2_u32(const PQG_G uint32_t* p) {
  return __hip_atomic_load((PQG_G uint32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

__device__ __forceinline__ int bits_len(uint32_t v) { return v ? 32 - __builtin_clz(v) : 0; }

// getValuesDecoder chunk_reader.go:143-196
__device__ __forceinline__ int values_supported(int type, int type_length, int enc) {
  switch (type) {
    case 0: return enc == 0 || enc == 3 || enc == 8;
    case 6: return enc == 0 || enc == 8 || enc == 6 || enc == 7;  // + DELTA_LENGTH_BYTE_ARRAY / DELTA_BYTE_ARRAY
    case 7: return type_length >= 0 && (enc == 0 || enc == 8 || enc == 7);  // chunk_reader.go:86-97
    case 3: case 4: case 5: return enc == 0 || enc == 8;
    case 1: case 2: return enc == 0 || enc == 5 || enc == 8;
  }
  return 0;
}

template <class P>
__device__ __forceinline__ uint32_t rd_u32(P p) {
  return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

// One lane's byte reader over [p, p+n): 16-byte granules cached in registers
// (a granule holding a byte < n lies in mapped memory).  -1 past the end.
struct LaneBytes {
  gcu8 p;
  int64_t n;
  uintptr_t gaddr;
  uint4 g;
  __device__ __forceinline__ void init(const uint8_t* p_, int64_t n_) {
    p = gconst(p_);
    n = n_;
    gaddr = 0;
  }
  __device__ __forceinline__ int get(int64_t i) {
    if (i < 0 || i >= n) return -1;
    const uintptr_t a = (uintptr_t)(p + i);
    const uintptr_t ga = a & ~(uintptr_t)15;
    if (ga != gaddr) {
      g = ldg16(ga);
      gaddr = ga;
    }
    const int w = (int)((a >> 2) & 3);
    const uint32_t d = w == 0 ? g.x : w == 1 ? g.y : w == 2 ? g.z : g.w;
    return (int)((d >> (8 * (a & 3))) & 0xff);
  }
};

// Bounds-checked byte read of a device buffer.
template <class P>
__device__ __forceinline__ int get_byte(P p, int64_t n, int64_t i) {
  return (i >= 0 && i < n) ? (int)p[i] : -1;
}

// Read 8 bytes little endian starting at byte i of [p, p+n); bytes at or
// beyond `valid` read as 0 (Q5 zero padding), bytes beyond n are never touched.
// Fast path: the aligned dwords covering [i, i+8) all contain a readable byte,
// so they lie on pages that are mapped.
template <class P>
__device__ __forceinline__ uint64_t load_u64_masked(P p, int64_t n, int64_t i, int64_t valid) {
  int64_t lim = valid < n ? valid : n;
  if (i >= 0 && i + 8 <= lim) {
    uintptr_t a = (uintptr_t)(p + i);
    const PQG_G uint32_t* q = (const PQG_G uint32_t*)(a & ~(uintptr_t)3);
    int sh = (int)(a & 3) * 8;
    uint64_t lo = (uint64_t)q[0] | ((uint64_t)q[1] << 32);
    if (sh == 0) return lo;
    uint64_t hi = (uint64_t)q[2];
    return (lo >> sh) | (hi << (64 - sh));
  }
  uint64_t v = 0;
  for (int k = 0; k < 8; k++) {
    int64_t j = i + k;
    if (j >= 0 && j < lim) v |= (uint64_t)p[j] << (8 * k);
  }
  return v;
}

// Extract `w` (<= 32) bits at bit offset `bit` of stream [p, p+valid).
template <class P>
__device__ __forceinline__ uint32_t extract_bits32(P p, int64_t n, int64_t valid, int64_t bit, int w) {
  if (w == 0) return 0;
  uint64_t x = load_u64_masked(p, n, bit >> 3, valid);
  x >>= (bit & 7);
  return (uint32_t)(x & ((w == 32) ? 0xffffffffull : ((1ull << w) - 1)));
}

// Extract `w` (<= 64) bits.
template <class P>
__device__ __forceinline__ uint64_t extract_bits64(P p, int64_t n, int64_t valid, int64_t bit, int w) {
  if (w == 0) return 0;
  int64_t byte = bit >> 3;
  int sh = (int)(bit & 7);
  uint64_t lo = load_u64_masked(p, n, byte, valid);
  uint64_t v = lo >> sh;
  if (sh + w > 64) {
    uint64_t hi = load_u64_masked(p, n, byte + 8, valid);
    v |= hi << (64 - sh);
  }
  return w == 64 ? v : (v & ((1ull << w) - 1));
}

// ---------------------------------------------------------------------------
// Lane-contiguous output runs as aligned 16-byte stores: lane L's D dwords go
// to base + 4 (D L + i), i < nv (nv = D except at the ragged end; base is
// 4-byte aligned).  The run starts s dwords before a 16-byte boundary, so lane
// L stores dwords [D L + s, D L + s + D) — its own from s on and the first s
// of lane L + 1 (DPP wave_shl:1) — as aligned granules; lane 0 stores the
// first s dwords and ragged lanes store per dword.  All 64 lanes must be
// active.
// ---------------------------------------------------------------------------
template <int D, bool NT = false>
__device__ __forceinline__ void store_run_aligned(uintptr_t base, const uint32_t (&d)[D], int nv) {
  static_assert(D % 4 == 0, "whole granules per lane");
  const int lane = lane_id();
  const int s = __builtin_amdgcn_readfirstlane((int)(((16 - (base & 15)) & 15) >> 2));
  uint32_t nx[3];
#pragma unroll
  for (int q = 0; q < 3; q++) nx[q] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)d[q], 0x130, 0xf, 0xf, true);
  const int nxv = __builtin_amdgcn_update_dpp(0, nv, 0x130, 0xf, 0xf, true);
  uint32_t w[D];
#pragma unroll
  for (int q = 0; q < D; q++) {
    const uint32_t a1 = q + 1 < D ? d[q + 1] : nx[q + 1 - D];
    const uint32_t a2 = q + 2 < D ? d[q + 2] : nx[q + 2 - D];
    const uint32_t a3 = q + 3 < D ? d[q + 3] : nx[q + 3 - D];
    w[q] = s == 0 ? d[q] : s == 1 ? a1 : s == 2 ? a2 : a3;
  }
  const uintptr_t o = base + 4 * ((uintptr_t)D * lane + s);
  if (nv == D && nxv >= s) {
#pragma unroll
    for (int g = 0; g < D / 4; g++) {
      if (NT) {
        const u32x4_t v = {w[4 * g], w[4 * g + 1], w[4 * g + 2], w[4 * g + 3]};
        __builtin_nontemporal_store(v, (PQG_G u32x4_t*)(o + 16 * g));
      } else if (D >= 8) {
        // each instruction writes every other granule of the wave's span:
        // write-back stores, so the L2 merges the halves of each line (the
        // non-temporal ones went out as half lines, see store_run64)
        stg16(o + 16 * g, make_uint4(w[4 * g], w[4 * g + 1], w[4 * g + 2], w[4 * g + 3]));
      } else {
        stg16o(o + 16 * g, make_uint4(w[4 * g], w[4 * g + 1], w[4 * g + 2], w[4 * g + 3]));
      }
    }
  } else {
#pragma unroll
    for (int q = 0; q < D; q++) {
      const int r = s + q;
      if (r < D ? r < nv : r - D < nxv) *(PQG_G uint32_t*)(o + 4 * q) = w[q];
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int q = 0; q < 3; q++)
      if (q < s && q < nv) *(PQG_G uint32_t*)(base + 4 * q) = d[q];
  }
}

// ---------------------------------------------------------------------------
// Wave-cooperative byte copy, any alignment on either side: 16-byte aligned
// destination granules (one dwordx4 store per lane), each funnel-shifted out of
// two aligned 16-byte source granules; ragged head and tail bytewise.  Only
// granules holding a source byte are read (mapped memory).
// ---------------------------------------------------------------------------
// Four granules per lane per step, every load issued before the first store
// (one memory round trip per 4 KiB per wave instead of per 1 KiB).
template <int Q>
__device__ __forceinline__ void wave_copy_body(PQG_G uint8_t* db, uintptr_t sbase, uint32_t r, int64_t body) {
  const int lane = lane_id();
  constexpr int U = 4;
  for (int64_t g0 = (int64_t)lane * 16; g0 < body; g0 += 64 * 16 * U) {
    uint4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t g = g0 + (int64_t)u * 64 * 16;
      const uintptr_t at = g < body ? sbase + g : sbase;  // sbase holds a source byte
      a[u] = ldg16(at);
      b[u] = (Q != 0 || r != 0) ? ldg16(g < body ? at + 16 : sbase) : a[u];
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t g = g0 + (int64_t)u * 64 * 16;
      if (g >= body) break;
      const uint32_t w[8] = {a[u].x, a[u].y, a[u].z, a[u].w, b[u].x, b[u].y, b[u].z, b[u].w};
      uint4 o;
      o.x = __builtin_amdgcn_alignbit(w[Q + 1], w[Q], r);
      o.y = __builtin_amdgcn_alignbit(w[Q + 2], w[Q + 1], r);
      o.z = __builtin_amdgcn_alignbit(w[Q + 3], w[Q + 2], r);
      o.w = __builtin_amdgcn_alignbit(w[Q + 4 < 8 ? Q + 4 : 7], w[Q + 3], r);
      stg16o((uintptr_t)(db + g), o);
    }
  }
}

__device__ __forceinline__ void wave_copy(PQG_G uint8_t* dst, const PQG_G uint8_t* src, int64_t nbytes) {
  if (nbytes <= 0) return;
  const int lane = lane_id();
  int64_t head = (int64_t)((16 - ((uintptr_t)dst & 15)) & 15);
  if (head > nbytes) head = nbytes;
  if (lane < head) dst[lane] = src[lane];
  const int64_t body = (nbytes - head) & ~(int64_t)15;
  PQG_G uint8_t* db = dst + head;
  const uintptr_t sa = (uintptr_t)(src + head);
  const uintptr_t sbase = sa & ~(uintptr_t)15;
  const uint32_t q = (uint32_t)(sa >> 2) & 3, r = (uint32_t)(sa & 3) * 8;
  switch (q) {
    case 0: wave_copy_body<0>(db, sbase, r, body); break;
    case 1: wave_copy_body<1>(db, sbase, r, body); break;
    case 2: wave_copy_body<2>(db, sbase, r, body); break;
    default: wave_copy_body<3>(db, sbase, r, body); break;
  }
  const int64_t t0 = head + body;
  if (t0 + lane < nbytes) dst[t0 + lane] = src[t0 + lane];
}

// In-kernel phase timing (diagnostic builds only: -DPQG_PROFILE).  Lane 0
// adds s_memtime deltas into pqg_prof[slot]; pqg_debug_counters reads them.
#ifdef PQG_PROFILE
static __device__ unsigned long long pqg_prof[64];  // one per translation unit (no -fgpu-rdc)
#define PQG_T(var) const uint64_t var = __builtin_amdgcn_s_memtime()
#define PQG_ACC(slot, a, b) \
  do { if (lane_id() == 0) atomicAdd(&pqg_prof[slot], (unsigned long long)((b) - (a))); } while (0)
#else
#define PQG_T(var)
#define PQG_ACC(slot, a, b) do { } while (0)
#endif

// Work queues are sharded over the 8 XCDs: one device-scope atomic word
// saturates near 88 dequeues/us (MI355X_MICROARCH.md, dequeue row), i.e.
// ~0.4 ms for 35 000 pages.  Blocks are dealt round-robin over the XCDs, so
// shard = blockIdx & 7 keeps each head on one XCD; shard s hands out items
// s, s + 8, s + 16, ...  A queue is kQShards heads kQStride ints apart (one
// 128-byte line each), zeroed before the launch.
__device__ __forceinline__ int queue_pull(int* queue) {
  const int shard = (int)(blockIdx.x & (kQShards - 1));
  return atomicAdd(queue + shard * kQStride, 1) * kQShards + shard;
}
// Next item, wave-uniform (in an SGPR): struct loads indexed by it become
// scalar loads, which do not queue behind vector loads and stores (vmcnt) the
// way vector loads of the same fields would.
__device__ __forceinline__ int queue_next(int* queue) {
  // the first active lane pulls: should a compiler ever make the caller's loop
  // divergent, the active lanes still agree on t (no lane re-reads a stale 0)
  const int leader = __builtin_amdgcn_readfirstlane(lane_id());
  int t = 0;
  if (lane_id() == leader) t = queue_pull(queue);
  return __builtin_amdgcn_readfirstlane(t);
}

// ---------------------------------------------------------------------------
// Wave-wide reductions / scans (64 lanes).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int64_t wave_sum(int64_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int64_t wave_min(int64_t v) {
  for (int o = 32; o > 0; o >>= 1) {
    int64_t t = __shfl_xor(v, o, 64);
    v = t < v ? t : v;
  }
  return v;
}
// ---------------------------------------------------------------------------
// The chain 0 -> next(0) -> ... among 128 speculative positions (next0 /
// next1: the successor of positions lane / 64 + lane, 128 when it leaves the
// positions or the item there fails), as two 64-bit masks, by pointer doubling
// instead of a serial readlane walk: J_k = next^(2^k) by ds_bpermute, then the
// marks {next^m(0) : m < 64} in six scatter rounds through 128 LDS flag bytes
// F (k = 5..0).  Items are >= 2 positions long, so the chain has <= 64 of them.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void chain_marks128(int next0, int next1, PQG_L uint8_t* F, uint64_t& cm0, uint64_t& cm1) {
  const int lane = lane_id();
  uint32_t j0[6], j1[6];
  j0[0] = (uint32_t)next0;
  j1[0] = (uint32_t)next1;
#pragma unroll
  for (int k = 1; k < 6; k++) {
    const uint32_t q0 = j0[k - 1], q1 = j1[k - 1];
    const uint32_t a0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((q0 & 63) * 4), (int)j0[k - 1]);
    const uint32_t b0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((q0 & 63) * 4), (int)j1[k - 1]);
    const uint32_t a1 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((q1 & 63) * 4), (int)j0[k - 1]);
    const uint32_t b1 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((q1 & 63) * 4), (int)j1[k - 1]);
    j0[k] = q0 < 64 ? a0 : q0 < 128u ? b0 : 128u;
    j1[k] = q1 < 64 ? a1 : q1 < 128u ? b1 : 128u;
  }
  F[lane] = lane == 0 ? 1 : 0;
  F[64 + lane] = 0;
  cm0 = 1;
  cm1 = 0;
#pragma unroll
  for (int k = 5; k >= 0; k--) {
    if (((cm0 >> lane) & 1) && j0[k] < 128u) F[j0[k]] = 1;
    if (((cm1 >> lane) & 1) && j1[k] < 128u) F[j1[k]] = 1;
    __builtin_amdgcn_wave_barrier();
    cm0 = __ballot(F[lane] != 0);
    cm1 = __ballot(F[64 + lane] != 0);
  }
}

// inclusive scan of uint64 (wrapping): DPP row_shr 1/2/4/8 then row_bcast
// 15/31 on both halves, one 64-bit add per step (no LDS round trips)
__device__ __forceinline__ uint64_t wave_incl_scan_u64(uint64_t v) {
#define PQG_SCAN64_STEP(ctrl, rm, bc)                                                             \
  {                                                                                               \
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, ctrl, rm, 0xf, bc);  \
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), ctrl, rm, 0xf, bc); \
    v += (uint64_t)hi << 32 | lo;                                                                 \
  }
  PQG_SCAN64_STEP(0x111, 0xf, true) PQG_SCAN64_STEP(0x112, 0xf, true) PQG_SCAN64_STEP(0x114, 0xf, true)
  PQG_SCAN64_STEP(0x118, 0xf, true) PQG_SCAN64_STEP(0x142, 0xa, false) PQG_SCAN64_STEP(0x143, 0xc, false)
#undef PQG_SCAN64_STEP
  return v;
}
__device__ __forceinline__ int64_t wave_excl_scan_i64(int64_t v, int64_t* total) {
  const uint64_t x = wave_incl_scan_u64((uint64_t)v);  // DPP, wrapping = two's complement
  *total = (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, 63) |
                     (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), 63) << 32);
  return (int64_t)x - v;
}

// Block-wide exclusive scan (NT threads, NT/64 waves); `part` holds NT/64+1
// entries of LDS.  Every thread of the block must call it.
template <int NT>
__device__ __forceinline__ int64_t block_excl_scan(int64_t v, int64_t* total, int64_t* part) {
  constexpr int NW = NT / 64;
  const int lane = lane_id(), wid = (int)(threadIdx.x >> 6);
  int64_t wt;
  const int64_t ex = wave_excl_scan_i64(v, &wt);
  if (lane == 0) part[wid] = wt;
  __syncthreads();
  if (wid == 0) {
    int64_t x = lane < NW ? part[lane] : 0, t;
    int64_t e = wave_excl_scan_i64(x, &t);
    __builtin_amdgcn_wave_barrier();
    if (lane < NW) part[lane] = e;
    if (lane == 0) part[NW] = t;
  }
  __syncthreads();
  const int64_t r = ex + part[wid];
  *total = part[NW];
  __syncthreads();
  return r;
}

// ---------------------------------------------------------------------------
// LDS byte window over a device stream, refilled cooperatively by the wave.
// All lanes call get() with the same position (wave-uniform control flow).
// ---------------------------------------------------------------------------
constexpr int kWin = 1024;
constexpr int64_t kFarAway = -((int64_t)1 << 62);

struct Window {
  gcu8 p;
  int64_t n;        // readable bytes of the stream
  int64_t base;     // stream offset of window[0]
  PQG_L uint8_t* lds;  // kWin bytes (16-byte aligned)

  __device__ void fill(int64_t at) {
    // align the window to 16 bytes of absolute address so each lane moves one
    // dwordx4; window covers [base, base + kWin) with base in (at - 16, at].
    uintptr_t abs = (uintptr_t)(p + at);
    uintptr_t ab = abs & ~(uintptr_t)15;
    base = at - (int64_t)(abs - ab);
    int l = lane_id();
    int64_t off = base + l * 16;
    uint4 v;
    if (off >= 0 && off + 16 <= n) {
      v = ldg16((uintptr_t)(p + off));
    } else {
      uint32_t w[4] = {0, 0, 0, 0};
      for (int k = 0; k < 16; k++) {
        int64_t j = off + k;
        if (j >= 0 && j < n) w[k >> 2] |= (uint32_t)p[j] << (8 * (k & 3));
      }
      v = make_uint4(w[0], w[1], w[2], w[3]);
    }
    sts16(lds + l * 16, v);
    __builtin_amdgcn_wave_barrier();
  }
  // byte at stream offset i, or -1 past the end
  __device__ __forceinline__ int get(int64_t i) {
    if (i < 0 || i >= n) return -1;
    if (i < base || i >= base + kWin) fill(i);
    return lds[i - base];
  }
};

// ---- varints of DELTA_BINARY_PACKED headers (helpers.go:149-183 via
// binary.ReadUvarint / ReadVarint), through a Window, with the oracle's error
// classes
__device__ __forceinline__ int read_uvarint64(Window& w, int64_t& pos, uint64_t* out) {
  uint64_t x = 0;
  unsigned s = 0;
  for (int i = 0;; i++) {
    int b = w.get(pos);
    if (b < 0) return kEOF;
    pos++;
    if (b < 0x80) {
      if (i > 9 || (i == 9 && b > 1)) return kRLE;
      *out = x | (s < 64 ? (uint64_t)b << s : 0);
      return kOK;
    }
    if (s < 64) x |= (uint64_t)(b & 0x7f) << s;
    s += 7;
  }
}
// readVariant32 / readVariant64 with the oracle's error classes
__device__ __forceinline__ int read_signed(Window& w, int64_t& pos, bool is64, uint64_t* out) {
  uint64_t ux;
  int e = read_uvarint64(w, pos, &ux);
  if (e) return e == kEOF ? kEOF : kDELTA;
  int64_t x = (int64_t)(ux >> 1);
  if (ux & 1) x = ~x;
  if (!is64 && (x > 2147483647LL || x < -2147483648LL)) return kDELTA;
  *out = (uint64_t)x;
  return kOK;
}
__device__ __forceinline__ int read_u32var_delta(Window& w, int64_t& pos, int32_t* out) {
  uint64_t v;
  int e = read_uvarint64(w, pos, &v);
  if (e) return e == kEOF ? kEOF : kDELTA;
  if (v > 0x7fffffffull) return kDELTA;
  *out = (int32_t)v;
  return kOK;
}

}  // namespace pqg
