// pqg_assemble.hip — K8: Dremel levels → validity bitmap, spaced values and
// record/list offsets for one decoded column chunk.
//
// What it replaces: the per-slot walk of ColumnStore.get (data_store.go:158-203)
// and Column.getData (schema.go:235-264).  There a slot with dLevel < maxD is a
// null that advances the level cursor but not the value cursor; a slot with
// rLevel < maxR ends the current repeated object.  Here the same two
// predicates are evaluated for every slot at once:
//   valid(i)    = def[i] == max_def                (def == NULL → all valid)
//   boundary(i) = rep[i] <= boundary_level         (rep == NULL → every slot)
// and the dense value cursor becomes rank(i) = #valid slots before i, so
//   validity bit i      = valid(i)                 (LSB-first, Arrow layout)
//   spaced[i]           = valid(i) ? dense[rank(i)] : 0
//   offsets[#b before i]= i for every boundary slot, offsets[num_rows] = n.
// boundary_level 0 gives record (row) starts (rep==0 → new row); maxR-1 gives
// the objects ColumnStore.get returns (`rl < maxR` ends one).
//
// Three launches, all HBM-streaming integer work:
//   k_asm_count  one wave per 4096-slot segment: ballot + popcount of both
//                predicates (reads the level bytes once)
//   k_asm_scan   one block: exclusive scan of the per-segment counts
//   k_asm_write  one wave per segment again: 64 slots per ballot, the bitmap
//                word is the ballot itself, ranks are popcount(mask & lt);
//                value copies and stores are contiguous across the wave.
#include <hip/hip_runtime.h>

#include "pqgpu.h"
#include "pqg_common.h"
#include "pqg_device.h"

namespace pqg {

constexpr int kAsmSeg = 4096;  // slots per wave segment (64 ballots)

__device__ __forceinline__ uint64_t ballot64(bool p) { return __ballot(p); }
__device__ __forceinline__ int lane64() { return __lane_id(); }

__device__ __forceinline__ bool slot_valid(const PQG_G uint8_t* def, int64_t i, int max_def) {
  return def == nullptr || def[i] == (uint8_t)max_def;
}
__device__ __forceinline__ bool slot_boundary(const PQG_G uint8_t* rep, int64_t i, int level) {
  return rep == nullptr || (int)rep[i] <= level;
}

__global__ void __launch_bounds__(256) k_asm_count(const uint8_t* def_, const uint8_t* rep_, int64_t n, int max_def,
                                                   int level, int64_t nseg, int64_t* seg_cnt) {
  const PQG_G uint8_t* def = gconst(def_);
  const PQG_G uint8_t* rep = gconst(rep_);
  const int64_t seg = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (seg >= nseg) return;
  const int lane = lane64();
  const int64_t s0 = seg * kAsmSeg, s1 = s0 + kAsmSeg < n ? s0 + kAsmSeg : n;
  int64_t nv = 0, nb = 0;
  for (int64_t b = s0; b < s1; b += 64) {
    const int64_t i = b + lane;
    const bool in = i < s1;
    nv += __popcll(ballot64(in && slot_valid(def, i, max_def)));
    nb += __popcll(ballot64(in && slot_boundary(rep, i, level)));
  }
  if (lane == 0) {
    PQG_G int64_t* o = gmut(seg_cnt) + 2 * seg;
    o[0] = nv;
    o[1] = nb;
  }
}

// Exclusive scan of (valid, boundary) pairs in place; tot[0..1] = totals.
// Writes offsets[num_rows] = n (the closing offset).  Each thread owns 4
// consecutive segments, so one block-wide pass covers 4096 segments (16 M slots).
__global__ void __launch_bounds__(1024) k_asm_scan(int64_t* seg_cnt, int64_t nseg, int64_t n, int64_t* tot,
                                                   int64_t* offsets) {
  __shared__ int64_t sv[1024], sb[1024];
  __shared__ int64_t carry[2];
  const int t = threadIdx.x;
  if (t == 0) carry[0] = carry[1] = 0;
  __syncthreads();
  for (int64_t base = 0; base < nseg; base += 4096) {
    const int64_t k0 = base + 4 * (int64_t)t;
    int64_t v[4], b[4], lv = 0, lb = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const bool in = k0 + j < nseg;
      v[j] = in ? seg_cnt[2 * (k0 + j)] : 0;
      b[j] = in ? seg_cnt[2 * (k0 + j) + 1] : 0;
      lv += v[j];
      lb += b[j];
    }
    sv[t] = lv;
    sb[t] = lb;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {  // Hillis–Steele inclusive scan of the per-thread sums
      const int64_t av = t >= d ? sv[t - d] : 0, ab = t >= d ? sb[t - d] : 0;
      __syncthreads();
      sv[t] += av;
      sb[t] += ab;
      __syncthreads();
    }
    int64_t ev = carry[0] + sv[t] - lv, eb = carry[1] + sb[t] - lb;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (k0 + j < nseg) {
        seg_cnt[2 * (k0 + j)] = ev;
        seg_cnt[2 * (k0 + j) + 1] = eb;
      }
      ev += v[j];
      eb += b[j];
    }
    __syncthreads();
    if (t == 1023) {
      carry[0] += sv[t];
      carry[1] += sb[t];
    }
    __syncthreads();
  }
  if (t == 0) {
    tot[0] = carry[0];
    tot[1] = carry[1];
    if (offsets) offsets[carry[1]] = n;
  }
}

template <int W>
__device__ __forceinline__ void copy_value(PQG_G uint8_t* dst, const PQG_G uint8_t* src, bool valid, int w) {
  if constexpr (W == 4) {
    *(PQG_G uint32_t*)dst = valid ? *(const PQG_G uint32_t*)src : 0u;
  } else if constexpr (W == 8) {
    *(PQG_G uint64_t*)dst = valid ? *(const PQG_G uint64_t*)src : 0ull;
  } else if constexpr (W == 1) {
    *dst = valid ? *src : (uint8_t)0;
  } else {
    for (int k = 0; k < w; k++) dst[k] = valid ? src[k] : (uint8_t)0;
  }
}

template <int W>
__global__ void __launch_bounds__(256) k_asm_write(const uint8_t* def_, const uint8_t* rep_, const uint8_t* values_,
                                                   int64_t n, int max_def, int level, int w, int64_t nseg,
                                                   const int64_t* seg_cnt, uint8_t* validity_, uint8_t* spaced_,
                                                   int64_t* offsets_) {
  const PQG_G uint8_t* def = gconst(def_);
  const PQG_G uint8_t* rep = gconst(rep_);
  const PQG_G uint8_t* values = gconst(values_);
  PQG_G uint8_t* validity = gmut(validity_);
  PQG_G uint8_t* spaced = gmut(spaced_);
  PQG_G int64_t* offsets = gmut(offsets_);
  const int64_t seg = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (seg >= nseg) return;
  const int lane = lane64();
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  const int64_t s0 = seg * kAsmSeg, s1 = s0 + kAsmSeg < n ? s0 + kAsmSeg : n;
  const int64_t nbytes = (n + 7) >> 3;
  int64_t rv = gconst(seg_cnt)[2 * seg], rb = gconst(seg_cnt)[2 * seg + 1];
  for (int64_t b = s0; b < s1; b += 64) {
    const int64_t i = b + lane;
    const bool in = i < s1;
    const bool v = in && slot_valid(def, i, max_def);
    const bool bd = in && slot_boundary(rep, i, level);
    const uint64_t mv = ballot64(v), mb = ballot64(bd);
    if (validity && lane < 8 && (b >> 3) + lane < nbytes) validity[(b >> 3) + lane] = (uint8_t)(mv >> (8 * lane));
    if (spaced && in) copy_value<W>(spaced + i * w, values + (rv + __popcll(mv & lt)) * w, v, w);
    if (offsets && bd) offsets[rb + __popcll(mb & lt)] = i;
    rv += __popcll(mv);
    rb += __popcll(mb);
  }
}

// ---------------------------------------------------------------------------
// List export (pqg_assemble_list): Arrow LIST layout of a repeated leaf.
// Three predicates per slot — row start (rep == 0), element (def >= elem_def),
// valid element (def == max_def) — give three ranks per slot, all popcounts of
// ballots plus the segment bases from the scan.  Row and element validity bits
// are not slot-aligned: the wave compresses each ballot's bits to rank order
// with one ds_permute (lane l pushes its bit to lane rank(l)) and ORs the
// packed word into the bitmap at the running bit offset.
// ---------------------------------------------------------------------------
struct ListPred {
  bool row, elem, valid, list_ok;
};
__device__ __forceinline__ ListPred list_pred(const PQG_G uint8_t* def, const PQG_G uint8_t* rep, int64_t i, bool in,
                                              int max_def, int list_def, int elem_def) {
  ListPred p;
  const int d = in ? (int)def[i] : -1;
  p.row = in && (rep == nullptr || rep[i] == 0);
  p.elem = in && d >= elem_def;
  p.valid = in && d == max_def;
  p.list_ok = p.row && d >= list_def;
  return p;
}

__global__ void __launch_bounds__(256) k_list_count(const uint8_t* def_, const uint8_t* rep_, int64_t n, int max_def,
                                                    int list_def, int elem_def, int64_t nseg, int64_t* seg_cnt) {
  const PQG_G uint8_t* def = gconst(def_);
  const PQG_G uint8_t* rep = gconst(rep_);
  const int64_t seg = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (seg >= nseg) return;
  const int lane = lane64();
  const int64_t s0 = seg * kAsmSeg, s1 = s0 + kAsmSeg < n ? s0 + kAsmSeg : n;
  int64_t nr = 0, ne = 0, nv = 0, nl = 0;
  for (int64_t b = s0; b < s1; b += 64) {
    const ListPred p = list_pred(def, rep, b + lane, b + lane < s1, max_def, list_def, elem_def);
    nr += __popcll(ballot64(p.row));
    ne += __popcll(ballot64(p.elem));
    nv += __popcll(ballot64(p.valid));
    nl += __popcll(ballot64(p.row && !p.list_ok));
  }
  if (lane == 0) {
    PQG_G int64_t* o = gmut(seg_cnt) + 4 * seg;
    o[0] = nr;
    o[1] = ne;
    o[2] = nv;
    o[3] = nl;
  }
}

// Exclusive scan of the 4 per-segment counters in place; tot[0..3] = totals;
// list_offsets[rows] = elements.
__global__ void __launch_bounds__(1024) k_list_scan(int64_t* seg_cnt, int64_t nseg, int64_t* tot,
                                                    int32_t* list_offsets) {
  __shared__ int64_t sc[4][1024];
  __shared__ int64_t carry[4];
  const int t = threadIdx.x;
  if (t < 4) carry[t] = 0;
  __syncthreads();
  for (int64_t base = 0; base < nseg; base += 1024) {
    const int64_t k = base + t;
    int64_t v[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      v[j] = k < nseg ? seg_cnt[4 * k + j] : 0;
      sc[j][t] = v[j];
    }
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
      int64_t a[4];
#pragma unroll
      for (int j = 0; j < 4; j++) a[j] = t >= d ? sc[j][t - d] : 0;
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 4; j++) sc[j][t] += a[j];
      __syncthreads();
    }
    if (k < nseg) {
#pragma unroll
      for (int j = 0; j < 4; j++) seg_cnt[4 * k + j] = carry[j] + sc[j][t] - v[j];
    }
    __syncthreads();
    if (t < 4) carry[t] += sc[t][1023];
    __syncthreads();
  }
  if (t == 0) {
    for (int j = 0; j < 4; j++) tot[j] = carry[j];
    // more elements than int32 offsets hold: the host reports PQG_ERR_INVALID_ARG
    // before any output is written (pqg_assemble_list)
    if (list_offsets && carry[1] <= INT32_MAX) list_offsets[carry[0]] = (int32_t)carry[1];
  }
}

// bits of `m` (ballot order) packed to rank order under mask `sel`: bit k of
// the result = m's bit at the k-th set lane of sel
__device__ __forceinline__ uint64_t compress_ballot(bool bit, bool in_sel, uint64_t sel, uint64_t lt) {
  const int rank = in_sel ? __popcll(sel & lt) : __popcll(sel) + __popcll(~sel & lt);
  const int got = __builtin_amdgcn_ds_permute(rank << 2, (int)bit);
  return ballot64(lane64() < __popcll(sel) && got != 0);
}

// OR packed bits into a bitmap at bit offset `at` (atomic: neighbouring
// waves share the boundary words); the bits span at most three dwords
__device__ __forceinline__ void or_bits(uint32_t* bm, int64_t at, uint64_t bits) {
  if (bits == 0) return;
  uint32_t* w = bm + (at >> 5);
  const int sh = (int)(at & 31);
  const uint32_t q0 = (uint32_t)(bits << sh);
  const uint32_t q1 = (uint32_t)(bits >> (32 - sh));  // sh = 0: bits >> 32
  const uint32_t q2 = sh ? (uint32_t)(bits >> (64 - sh)) : 0u;
  if (q0) atomicOr(w, q0);
  if (q1) atomicOr(w + 1, q1);
  if (q2) atomicOr(w + 2, q2);
}

template <int W>
__global__ void __launch_bounds__(256) k_list_write(const uint8_t* def_, const uint8_t* rep_, const uint8_t* values_,
                                                    int64_t n, int max_def, int list_def, int elem_def, int w,
                                                    int64_t nseg, const int64_t* seg_cnt, uint8_t* list_validity_,
                                                    int32_t* list_offsets_, uint8_t* elem_validity_,
                                                    uint8_t* elem_values_) {
  const PQG_G uint8_t* def = gconst(def_);
  const PQG_G uint8_t* rep = gconst(rep_);
  const PQG_G uint8_t* values = gconst(values_);
  PQG_G int32_t* list_offsets = gmut(list_offsets_);
  PQG_G uint8_t* elem_values = gmut(elem_values_);
  uint32_t* lval = (uint32_t*)list_validity_;
  uint32_t* evalid = (uint32_t*)elem_validity_;
  const int64_t seg = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (seg >= nseg) return;
  const int lane = lane64();
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  const int64_t s0 = seg * kAsmSeg, s1 = s0 + kAsmSeg < n ? s0 + kAsmSeg : n;
  const PQG_G int64_t* sc = gconst(seg_cnt) + 4 * seg;
  int64_t rb = sc[0], eb = sc[1], vb = sc[2];
  for (int64_t b = s0; b < s1; b += 64) {
    const int64_t i = b + lane;
    const ListPred p = list_pred(def, rep, i, i < s1, max_def, list_def, elem_def);
    const uint64_t mr = ballot64(p.row), me = ballot64(p.elem), mv = ballot64(p.valid);
    const int64_t e = eb + __popcll(me & lt);
    if (p.row && list_offsets) list_offsets[rb + __popcll(mr & lt)] = (int32_t)e;
    if (p.elem && elem_values)
      copy_value<W>(elem_values + e * w, values + (vb + __popcll(mv & lt)) * w, p.valid, w);
    if (list_validity_) {
      const uint64_t bits = compress_ballot(p.list_ok, p.row, mr, lt);
      if (lane == 0) or_bits(lval, rb, bits);
    }
    if (elem_validity_) {
      const uint64_t bits = compress_ballot(p.valid, p.elem, me, lt);
      if (lane == 0) or_bits(evalid, eb, bits);
    }
    rb += __popcll(mr);
    eb += __popcll(me);
    vb += __popcll(mv);
  }
}

// Count + scan of the list export; tot[0..3] = rows, elements, valid elements,
// null lists.  Writes no output but list_offsets[rows] (and that only when the
// element count fits int32).
int list_count_launch(hipStream_t s, const pqg_list_args* a, int64_t* seg_scratch, int64_t* tot) {
  const int64_t n = a->num_slots;
  const int64_t nseg = (n + kAsmSeg - 1) / kAsmSeg;
  const unsigned blocks = (unsigned)((nseg + 3) / 4);
  if (nseg > 0)
    hipLaunchKernelGGL(k_list_count, dim3(blocks), dim3(256), 0, s, a->def_levels, a->rep_levels, n, a->max_def,
                       a->list_def, a->elem_def, nseg, seg_scratch);
  hipLaunchKernelGGL(k_list_scan, dim3(1), dim3(1024), 0, s, seg_scratch, nseg, tot, a->list_offsets);
  return hipGetLastError() == hipSuccess ? PQG_OK : PQG_ERR_HIP;
}

// The outputs, after list_count_launch's totals were checked by the host.
int list_write_launch(hipStream_t s, const pqg_list_args* a, int64_t* seg_scratch) {
  const int64_t n = a->num_slots;
  const int64_t nseg = (n + kAsmSeg - 1) / kAsmSeg;
  const unsigned blocks = (unsigned)((nseg + 3) / 4);
  const int w = a->elem_values ? a->value_width : 0;
  const size_t bm_bytes = (size_t)((n + 31) / 32) * 4;  // whole dwords (see pqgpu.h)
  if (a->list_validity && bm_bytes) hipMemsetAsync(a->list_validity, 0, bm_bytes, s);
  if (a->elem_validity && bm_bytes) hipMemsetAsync(a->elem_validity, 0, bm_bytes, s);
  if (nseg == 0) return hipGetLastError() == hipSuccess ? PQG_OK : PQG_ERR_HIP;
#define PQG_LST(WW)                                                                                                  \
  hipLaunchKernelGGL(k_list_write<WW>, dim3(blocks), dim3(256), 0, s, a->def_levels, a->rep_levels, a->values, n,   \
                     a->max_def, a->list_def, a->elem_def, w, nseg, (const int64_t*)seg_scratch, a->list_validity,  \
                     a->list_offsets, a->elem_validity, a->elem_values)
  switch (w) {
    case 1: PQG_LST(1); break;
    case 4: PQG_LST(4); break;
    case 8: PQG_LST(8); break;
    default: PQG_LST(0); break;
  }
#undef PQG_LST
  return hipGetLastError() == hipSuccess ? PQG_OK : PQG_ERR_HIP;
}

// ---------------------------------------------------------------------------
// ColumnStore refill: levels -> packedArray bytes (packed_array.go:34-101).
// One lane per group of 8 levels: one 8-byte load, the 8 w-bit fields OR-ed
// into a 64-bit word (bw <= 8 for u8 levels), bw byte stores.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_pack_levels(const uint8_t* levels_, int64_t n, int bw, uint8_t* packed_) {
  const PQG_G uint8_t* levels = gconst(levels_);
  PQG_G uint8_t* packed = gmut(packed_);
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t groups = (n + 7) / 8;
  if (g >= groups) return;
  uint64_t bits = 0;
  const uint64_t mask = (1ull << bw) - 1;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const int64_t i = g * 8 + k;
    const uint64_t v = i < n ? levels[i] : 0;
    bits |= (v & mask) << (k * bw);
  }
  for (int b = 0; b < bw; b++) packed[g * bw + b] = (uint8_t)(bits >> (8 * b));
}

int pack_levels_launch(hipStream_t s, const uint8_t* levels, int64_t n, int bw, uint8_t* packed) {
  const int64_t groups = (n + 7) / 8;
  if (groups > 0 && bw > 0)
    hipLaunchKernelGGL(k_pack_levels, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, s, levels, n, bw, packed);
  return hipGetLastError() == hipSuccess ? PQG_OK : PQG_ERR_HIP;
}

// Host launcher (called from pqg_assemble in pqg_runtime.hip).  seg_scratch
// holds 2 × nseg int64; tot 2 int64 (device).
int assemble_launch(hipStream_t s, const pqg_assemble_args* a, int64_t* seg_scratch, int64_t* tot) {
  const int64_t n = a->num_slots;
  const int64_t nseg = (n + kAsmSeg - 1) / kAsmSeg;
  const unsigned blocks = (unsigned)((nseg + 3) / 4);
  const int w = a->values_spaced ? a->value_width : 0;
  if (nseg > 0)
    hipLaunchKernelGGL(k_asm_count, dim3(blocks), dim3(256), 0, s, a->def_levels, a->rep_levels, n, a->max_def,
                       a->boundary_level, nseg, seg_scratch);
  hipLaunchKernelGGL(k_asm_scan, dim3(1), dim3(1024), 0, s, seg_scratch, nseg, n, tot, a->offsets);
  if (nseg == 0) return hipGetLastError() == hipSuccess ? PQG_OK : PQG_ERR_HIP;
#define PQG_ASM(WW)                                                                                                  \
  hipLaunchKernelGGL(k_asm_write<WW>, dim3(blocks), dim3(256), 0, s, a->def_levels, a->rep_levels, a->values, n,    \
                     a->max_def, a->boundary_level, w, nseg, (const int64_t*)seg_scratch, a->validity,              \
                     a->values_spaced, a->offsets)
  switch (w) {
    case 1: PQG_ASM(1); break;
    case 4: PQG_ASM(4); break;
    case 8: PQG_ASM(8); break;
    default: PQG_ASM(0); break;
  }
#undef PQG_ASM
  return hipGetLastError() == hipSuccess ? PQG_OK : PQG_ERR_HIP;
}

}  // namespace pqg
