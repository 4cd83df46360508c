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
// K2: one wave per compressed block.
//
// The tag stream is serial (each tag's length decides where the next one
// starts), so the wave decodes it tag by tag, wave-uniformly; the bytes of a
// literal or a copy are moved by all lanes at once.  The output is produced in
// an LDS ring that holds the last RING bytes: every back-reference with
// offset <= RING reads the ring (snappy's copy-1/copy-2 offsets are < 64 KiB),
// so no tag waits on HBM.  The ring is flushed to the page's scratch block in
// 4 KiB pieces with 16-byte stores.  The compressed bytes are read through a
// 1 KiB LDS window (8 bytes per tag read, one broadcast LDS load).  Copies
// reaching further back than the ring (copy-4 offsets >= RING) read the
// already flushed output from L2 after the flush stores have completed.
//
// Two instances: RING = 32 KiB for blocks of at most 32 KiB (every offset is
// inside the ring; 4 waves per CU), RING = 64 KiB for larger blocks.
// ============================================================================
constexpr int kFlush = 4096;
constexpr int kSmallRing = 32768;  // blocks up to this size go to the 32 KiB-ring instance

template <int RING>
struct SnapShared {
  uint8_t ring[RING];
  uint8_t win[kWin];
};

__device__ __forceinline__ uint32_t l2_load_u32(const PQG_G uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The compressed stream through the LDS window (refilled 16-byte aligned so
// each lane moves one dwordx4).
struct SnapIn {
  gcu8 p;
  int64_t n;
  int64_t base;
  PQG_L uint8_t* lds;
  __device__ void fill(int64_t at) {
    const uintptr_t abs = (uintptr_t)(p + at);
    base = at - (int64_t)(abs & 15);
    const int l = lane_id();
    const int64_t off = base + l * 16;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (off >= 0 && off + 16 <= n) {
      v = ldg16((uintptr_t)(p + off));
    } else {
      uint32_t w[4] = {0, 0, 0, 0};
      for (int k = 0; k < 16; k++) {
        const int64_t j = off + k;
        if (j >= 0 && j < n) w[k >> 2] |= (uint32_t)p[j] << (8 * (k & 3));
      }
      v = make_uint4(w[0], w[1], w[2], w[3]);
    }
    __builtin_amdgcn_wave_barrier();
    sts16(lds + l * 16, v);
    __builtin_amdgcn_wave_barrier();
  }
  // 8 bytes at s (bytes past n read as 0): one broadcast LDS load
  __device__ __forceinline__ uint64_t peek8(int64_t s) {
    if (s < base || s + 8 > base + kWin) fill(s);
    const uint32_t o = (uint32_t)(s - base);
    const PQG_L uint32_t* q = (const PQG_L uint32_t*)(lds + (o & ~3u));
    const uint32_t a = q[0], b = q[1], c = q[2];
    const uint32_t sh = (o & 3) * 8;
    const uint32_t lo = __builtin_amdgcn_alignbit(b, a, sh), hi = __builtin_amdgcn_alignbit(c, b, sh);
    return (uint64_t)__builtin_amdgcn_readfirstlane(lo) | (uint64_t)__builtin_amdgcn_readfirstlane(hi) << 32;
  }
};

template <int RING>
struct SnapOut {
  PQG_L uint8_t* ring;
  gu8 dst;
  int64_t dlen;
  int64_t d = 0;        // output bytes produced
  int64_t flushed = 0;  // output bytes stored to dst
  static constexpr uint32_t M = RING - 1;

  // store [flushed, upto) from the ring: 16-byte granules of dst (16-aligned);
  // a ragged tail is stored bytewise and stored again by the next flush, so
  // `flushed` stays 16-byte aligned
  __device__ void flush(int64_t upto) {
    const int lane = lane_id();
    __builtin_amdgcn_wave_barrier();
    for (int64_t g = flushed + 16 * lane; g < upto; g += 16 * 64) {
      if (g + 16 <= upto) {
        const u32x4_t v = *(const PQG_L u32x4_t*)(ring + (g & M));
        stg16((uintptr_t)(dst + g), make_uint4(v.x, v.y, v.z, v.w));
      } else {
        for (int64_t k = g; k < upto; k++) dst[k] = ring[k & M];
      }
    }
    flushed = upto & ~(int64_t)15;
  }
  __device__ __forceinline__ void maybe_flush() {
    if (d - flushed >= kFlush) flush(flushed + kFlush * ((d - flushed) / kFlush));
  }
};

// Literal of `len` bytes at compressed offset s (len <= dlen - d, s + len <= slen).
template <int RING>
__device__ __forceinline__ void snap_literal(SnapIn& in, SnapOut<RING>& out, int64_t s, int64_t len) {
  const int lane = lane_id();
  constexpr uint32_t M = RING - 1;
  int64_t done = 0;
  while (done < len) {
    out.maybe_flush();
    // a piece inside the current window, at most 1 KiB
    const int64_t at = s + done;
    if (at < in.base || at >= in.base + kWin) in.fill(at);
    int64_t piece = in.base + kWin - at;
    if (piece > len - done) piece = len - done;
    if (piece > 1024) piece = 1024;
    const uint32_t wo = (uint32_t)(at - in.base);
    const int64_t d0 = out.d;
    for (int64_t j = lane; j < piece; j += 64) out.ring[(uint32_t)(d0 + j) & M] = in.lds[wo + j];
    out.d += piece;
    done += piece;
  }
}

// Copy of `len` bytes from `off` back (validated: 0 < off <= d, len <= dlen - d).
template <int RING>
__device__ __forceinline__ void snap_copy(SnapOut<RING>& out, int64_t off, int64_t len) {
  const int lane = lane_id();
  constexpr uint32_t M = RING - 1;
  out.maybe_flush();
  const int64_t d0 = out.d;
  if (off <= RING) {
    // forward copy with overlap == periodic copy of the `off` bytes before d;
    // the ring still holds positions [d - RING, d)
    for (int64_t j = lane; j < len; j += 64) {
      const int64_t from = d0 - off + (off >= len ? j : j % off);
      out.ring[(uint32_t)(d0 + j) & M] = out.ring[(uint32_t)from & M];
    }
  } else {
    // older than the ring (copy-4 offsets): the flushed output, read from L2
    // once the flush stores have completed (off > RING >= 64 > len: no overlap)
    out.flush(d0);
    __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) expcnt(0) lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    for (int64_t j = lane; j < len; j += 64) {
      const uintptr_t a = (uintptr_t)(out.dst + (d0 - off + j));
      out.ring[(uint32_t)(d0 + j) & M] =
          (uint8_t)(l2_load_u32((const PQG_G uint32_t*)(a & ~(uintptr_t)3)) >> ((a & 3) * 8));
    }
  }
  out.d += len;
}

// decode_other.go:14-101 over [s, slen) into dlen bytes
template <int RING>
__device__ int snappy_body(SnapIn& in, int64_t s, int64_t slen, SnapOut<RING>& out) {
  const int64_t dlen = out.dlen;
#ifdef PQG_PROFILE
  uint64_t n_lit = 0, n_copy = 0, c_lit = 0, c_copy = 0, c_parse = 0;
#endif
  while (s < slen) {
    PQG_T(ta);
    const uint64_t x8 = in.peek8(s);
#ifdef PQG_PROFILE
    PQG_T(tb);
    c_parse += tb - ta;
#endif
    const uint32_t tag = (uint32_t)x8 & 0xff;
    int64_t length, offset;
    switch (tag & 3) {
      case 0: {
        uint32_t x = tag >> 2;
        if (x < 60) {
          s += 1;
        } else {
          const int nb = (int)x - 59;  // 1..4 length bytes
          s += 1 + nb;
          if ((uint64_t)s > (uint64_t)slen) return kSNAPPY;
          x = (uint32_t)(x8 >> 8) & (nb == 4 ? 0xffffffffu : ((1u << (8 * nb)) - 1));
        }
        length = (int64_t)x + 1;
        if (length > dlen - out.d || length > slen - s) return kSNAPPY;
        snap_literal(in, out, s, length);
#ifdef PQG_PROFILE
        {
          PQG_T(tc);
          c_lit += tc - tb;
          n_lit++;
        }
#endif
        s += length;
        continue;
      }
      case 1:
        s += 2;
        if ((uint64_t)s > (uint64_t)slen) return kSNAPPY;
        length = 4 + ((tag >> 2) & 7);
        offset = (int64_t)((tag & 0xe0) << 3 | ((uint32_t)(x8 >> 8) & 0xff));
        break;
      case 2:
        s += 3;
        if ((uint64_t)s > (uint64_t)slen) return kSNAPPY;
        length = 1 + (tag >> 2);
        offset = (int64_t)((uint32_t)(x8 >> 8) & 0xffff);
        break;
      default:
        s += 5;
        if ((uint64_t)s > (uint64_t)slen) return kSNAPPY;
        length = 1 + (tag >> 2);
        offset = (int64_t)(uint32_t)(x8 >> 8);
        break;
    }
    if (offset <= 0 || out.d < offset || length > dlen - out.d) return kSNAPPY;
    snap_copy(out, offset, length);
#ifdef PQG_PROFILE
    {
      PQG_T(tc);
      c_copy += tc - tb;
      n_copy++;
    }
#endif
  }
#ifdef PQG_PROFILE
  PQG_ACC(16, 0, n_lit);
  PQG_ACC(17, 0, n_copy);
  PQG_ACC(18, 0, c_lit);
  PQG_ACC(19, 0, c_copy);
  PQG_ACC(20, 0, c_parse);
  PQG_ACC(21, 0, slen);
  PQG_ACC(22, 0, dlen);
#endif
  if (out.d != dlen) return kSNAPPY;
  out.flush(dlen);
  return kOK;
}

// kind 0: blocks of at most kSmallRing bytes; kind 1: larger ones
template <int RING, int KIND>
__global__ void __launch_bounds__(64) k_snappy(JobDev* jobs, PageDev* pages, const int* list, const int* total,
                                               int* queue, uint8_t* scratch) {
  __shared__ __attribute__((aligned(16))) SnapShared<RING> sh;
  const int lane = lane_id();
  for (;;) {
    const int t = queue_next(queue);
    if (t >= *total) return;
    const int pidx = __builtin_amdgcn_readfirstlane(list[t]);
    const PageDev pg = pages[pidx];  // locals via scalar loads (see k_levels_expand)
    if (pg.read_status != kOK || pg.scratch_offset < 0) continue;
    // compressed block location (V2: after the raw level bytes)
    int64_t src_off = pg.payload_offset;
    int64_t clen = pg.csize, ulen = pg.usize;
    if (pg.page_type == 3) {
      int32_t levels = (int32_t)((uint32_t)pg.rep_len + (uint32_t)pg.def_len);
      if (levels > 0) src_off += levels;
      clen = (int32_t)((uint32_t)pg.csize - (uint32_t)levels);
      ulen = (int32_t)((uint32_t)pg.usize - (uint32_t)levels);
    }
    if ((KIND == 0) != (ulen <= kSmallRing)) continue;  // the other instance's block
    const JobDev job = jobs[pg.job];
    SnapIn in{gconst(job.data) + src_off, clen, kFarAway, lds_ptr(sh.win)};
    // decodedLen: binary.Uvarint over the block (decode.go:32-43)
    uint64_t v = 0;
    int hl = 0;
    int e = kOK;
    {
      unsigned sft = 0;
      for (int i = 0;; i++) {
        if (i >= clen) { e = kSNAPPY; break; }
        const int b = (int)(in.peek8(i) & 0xff);
        if (b < 0x80) {
          if (i > 9 || (i == 9 && b > 1)) e = kSNAPPY;
          else v |= (sft < 64 ? (uint64_t)b << sft : 0);
          hl = i + 1;
          break;
        }
        if (sft < 64) v |= (uint64_t)(b & 0x7f) << sft;
        sft += 7;
      }
    }
    if (e == kOK && v > 0xffffffffull) e = kSNAPPY;
    if (e == kOK && (int64_t)v != ulen) e = kSIZE;
    if (e == kOK) {
      SnapOut<RING> out{lds_ptr(sh.ring), gmut(scratch) + job.scratch_base + pg.scratch_offset, ulen};
      e = snappy_body(in, hl, clen, out);
    }
    // V1: getValuesDecoder runs after the block is decompressed (page_v1.go:91-97)
    if (e == kOK && pg.page_type == 0 && !values_supported(job.type, job.type_length, pg.encoding)) e = kUNSUPPORTED;
    if (lane == 0 && e != kOK) pages[pidx].read_status = e;
  }
}

template __global__ void k_snappy<32768, 0>(JobDev*, PageDev*, const int*, const int*, int*, uint8_t*);
template __global__ void k_snappy<65536, 1>(JobDev*, PageDev*, const int*, const int*, int*, uint8_t*);

}  // namespace pqg
