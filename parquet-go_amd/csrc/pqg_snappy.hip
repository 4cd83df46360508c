// pqg_snappy.hip — K2: snappy block decompression (compress.go:90-122 →
// snappy.Decode, vendor/github.com/golang/snappy/decode.go:55-72,
// decode_other.go:14-101).
#include <hip/hip_runtime.h>

#include "pqg_common.h"
#include "pqg_device.h"

namespace pqg {

// ============================================================================
// K2: snappy block decompression — one wave per compressed block.
// Token parse is wave-uniform over an LDS window of the compressed bytes; the
// copies are lane parallel.  Output is staged in LDS when it fits (forward
// copies with overlap read only bytes written by earlier tokens), otherwise
// written to HBM with L2-coherent (sc1) reads of earlier output.
// ============================================================================
constexpr int kSnapLds = 32768;

struct SnapShared {
  uint8_t win[kWin];
  uint8_t out[kSnapLds];
};

__device__ __forceinline__ uint32_t l2_load_u32(const PQG_G uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool kLds>
__device__ int snappy_body(Window& win, int64_t s, int64_t slen, gu8 dst_g, PQG_L uint8_t* dst_l, int64_t dlen) {
  const int lane = lane_id();
  int64_t d = 0;
  while (s < slen) {
    int tag = win.get(s);
    int64_t length = 0, offset = 0;
    if ((tag & 3) == 0) {
      uint32_t x = (uint32_t)tag >> 2;
      if (x < 60) {
        s += 1;
      } else {
        int nb = (int)x - 59;  // 1..4 length bytes
        s += 1 + nb;
        if ((uint64_t)s > (uint64_t)slen) return kSNAPPY;
        x = 0;
        for (int k = 0; k < nb; k++) x |= (uint32_t)win.get(s - nb + k) << (8 * k);
      }
      length = (int64_t)x + 1;
      if (length > dlen - d || length > slen - s) return kSNAPPY;
      // literal copy: source bytes from the compressed block (window source)
      const gcu8 src = win.p + s;
      for (int64_t i = lane; i < length; i += 64) {
        uint8_t b = src[i];
        if (kLds) dst_l[d + i] = b; else dst_g[d + i] = b;
      }
      d += length;
      s += length;
      if (kLds) __builtin_amdgcn_wave_barrier();
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      continue;
    }
    if ((tag & 3) == 1) {
      s += 2;
      if ((uint64_t)s > (uint64_t)slen) return kSNAPPY;
      length = 4 + ((tag >> 2) & 7);
      offset = (int64_t)(((uint32_t)tag & 0xe0) << 3 | (uint32_t)win.get(s - 1));
    } else if ((tag & 3) == 2) {
      s += 3;
      if ((uint64_t)s > (uint64_t)slen) return kSNAPPY;
      length = 1 + (tag >> 2);
      offset = (int64_t)((uint32_t)win.get(s - 2) | (uint32_t)win.get(s - 1) << 8);
    } else {
      s += 5;
      if ((uint64_t)s > (uint64_t)slen) return kSNAPPY;
      length = 1 + (tag >> 2);
      offset = (int64_t)((uint32_t)win.get(s - 4) | (uint32_t)win.get(s - 3) << 8 | (uint32_t)win.get(s - 2) << 16 |
                         (uint32_t)win.get(s - 1) << 24);
    }
    if (offset <= 0 || d < offset || length > dlen - d) return kSNAPPY;
    // forward copy with overlap == periodic copy of the `offset` bytes before d
    for (int64_t i = lane; i < length; i += 64) {
      int64_t from = d - offset + (i % offset);
      uint8_t b;
      if (kLds) {
        b = dst_l[from];
      } else {
        uintptr_t a = (uintptr_t)(dst_g + from);
        uint32_t wv = l2_load_u32((const PQG_G uint32_t*)(a & ~(uintptr_t)3));
        b = (uint8_t)(wv >> ((a & 3) * 8));
      }
      if (kLds) dst_l[d + i] = b; else dst_g[d + i] = b;
    }
    d += length;
    if (kLds) __builtin_amdgcn_wave_barrier();
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (d != dlen) return kSNAPPY;
  return kOK;
}

__global__ void __launch_bounds__(64) k_snappy(JobDev* jobs, PageDev* pages, const int* list, const int* total,
                                               int* queue, uint8_t* scratch) {
  __shared__ __attribute__((aligned(16))) SnapShared sh;
  const int lane = lane_id();
  for (;;) {
    const int t = queue_next(queue);
    if (t >= *total) return;
    const int pidx = __builtin_amdgcn_readfirstlane(list[t]);
    const PageDev pg = pages[pidx];  // locals via scalar loads (see k_levels_expand)
    if (pg.read_status != kOK || pg.scratch_offset < 0) continue;
    const JobDev job = jobs[pg.job];
    // compressed block location (V2: after the raw level bytes)
    int64_t src_off = pg.payload_offset;
    int64_t clen = pg.csize, ulen = pg.usize;
    if (pg.page_type == 3) {
      int32_t levels = (int32_t)((uint32_t)pg.rep_len + (uint32_t)pg.def_len);
      if (levels > 0) src_off += levels;
      clen = (int32_t)((uint32_t)pg.csize - (uint32_t)levels);
      ulen = (int32_t)((uint32_t)pg.usize - (uint32_t)levels);
    }
    Window win{gconst(job.data) + src_off, clen, kFarAway, lds_ptr(sh.win)};
    // decodedLen: binary.Uvarint over the block (decode.go:32-43)
    uint64_t v = 0;
    int hl = 0;
    int e = kOK;
    {
      unsigned sft = 0;
      int i = 0;
      for (;; i++) {
        int b = win.get(i);
        if (b < 0) { e = kSNAPPY; break; }
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
    const gu8 dst = gmut(scratch) + job.scratch_base + pg.scratch_offset;
    if (e == kOK) {
      if (ulen <= kSnapLds) {
        e = snappy_body<true>(win, hl, clen, nullptr, lds_ptr(sh.out), ulen);
        if (e == kOK)
          for (int64_t i = lane; i < ulen; i += 64) dst[i] = sh.out[i];
      } else {
        e = snappy_body<false>(win, hl, clen, dst, nullptr, ulen);
      }
    }
    // V1: getValuesDecoder runs after the block is decompressed (page_v1.go:91-97)
    if (e == kOK && pg.page_type == 0 && !values_supported(job.type, job.type_length, pg.encoding)) e = kUNSUPPORTED;
    if (lane == 0 && e != kOK) pages[pidx].read_status = e;
  }
}

}  // namespace pqg
