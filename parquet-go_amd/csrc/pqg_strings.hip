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
//   K7a k_str_dict   one wave per chunk with a byte-array dictionary: walks the
//                    dictionary page's length chain into the record-start table
//                    doffs[count + 1], then publishes the dictionary
//   K7b k_str_count  one wave per byte-array data page: PLAIN pages walk the
//                    length chain (page-relative value ends, written into the
//                    chunk's offsets); dictionary pages sum the entry lengths
//                    of their keys.  -> page.chars
//   K7c k_char_scan  one block per chunk: exclusive scan of page.chars
//   K7d k_str_write  one wave per byte-array data page: final offsets + chars
//
// The length chain is the one serial dependency of the format.  It is walked
// by the scalar unit over a 1 KiB window held in the wave's VGPRs (64 lanes x 4
// dwords): a hop is two v_readlane of the dwords under the position, an
// alignbit and the bounds checks, all wave-uniform, so no LDS round trip sits
// on the chain.  64 consecutive value ends are collected one per lane and
// stored by one coalesced wave store.
#include <hip/hip_runtime.h>

#include "pqg_common.h"
#include "pqg_device.h"
#include "pqg_hybrid.h"

namespace pqg {

// 1 KiB of a byte stream in VGPRs: window dword k lives in d[k >> 6] of lane k & 63.
struct RegWindow {
  gcu8 p;        // stream start
  int64_t n;     // stream bytes
  int64_t base;  // stream offset of window byte 0 (4-byte aligned address)
  uint32_t d[4];

  __device__ __forceinline__ void init(gcu8 p_, int64_t n_) {
    p = p_;
    n = n_;
    base = kFarAway;
  }
  __device__ void fill(int64_t at) {
    const uintptr_t a = (uintptr_t)(p + at);
    base = at - (int64_t)(a & 3);
    const int l = lane_id();
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int64_t off = base + 4 * (int64_t)(j * 64 + l);
      // the dword holds a stream byte < n: it lies in the stream's allocation
      d[j] = (off + 4 > 0 && off < n) ? *(const PQG_G uint32_t*)(p + off) : 0u;
    }
  }
  __device__ __forceinline__ uint32_t dword(uint32_t k) {
    const uint32_t j = k >> 6;
    const uint32_t v = j == 0 ? d[0] : j == 1 ? d[1] : j == 2 ? d[2] : d[3];
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)(k & 63));
  }
  // u32 at stream offset pos (caller checked pos + 4 <= n)
  __device__ __forceinline__ uint32_t u32(int64_t pos) {
    int64_t off = pos - base;
    if (off < 0 || off + 8 > 1024) {
      fill(pos);
      off = pos - base;
    }
    const uint32_t k = (uint32_t)off >> 2, sh = ((uint32_t)off & 3) * 8;
    const uint32_t lo = dword(k), hi = dword(k + 1);
    return __builtin_amdgcn_alignbit(hi, lo, sh);
  }
};

// byteArrayPlainDecoder.next for values [0, count): a failing value ends the
// walk with its status.  `sink(i, pos_after, chars_after)` sees every value.
template <class F>
__device__ __forceinline__ int walk_lengths(RegWindow& win, int64_t count, int64_t* consumed, int64_t* chars, F&& sink) {
  int64_t pos = 0, cum = 0;
  int st = kOK;
  const int64_t n = win.n;
  for (int64_t i = 0; i < count; i++) {
    if (n - pos < 4) { st = kEOF; break; }
    const int32_t l = (int32_t)win.u32(pos);
    if (l < 0) { st = kBYTE_ARRAY; break; }
    if (n - pos - 4 < (int64_t)l) { st = kEOF; break; }
    pos += 4 + (int64_t)l;
    cum += l;
    sink(i, pos, cum);
  }
  *consumed = pos;
  *chars = cum;
  return st;
}

// Collects one int64 per value in lane (i & 63) and stores each full batch of 64.
struct LaneBatch {
  PQG_G int64_t* out;
  uint32_t lo, hi;
  __device__ __forceinline__ void put(int64_t i, int64_t v) {
    const int l = (int)(i & 63);
    const bool mine = lane_id() == l;  // v_cmp + two v_cndmask: the value lands in lane l
    lo = mine ? (uint32_t)v : lo;
    hi = mine ? (uint32_t)((uint64_t)v >> 32) : hi;
    if (l == 63) flush(i - 63, 64);
  }
  __device__ __forceinline__ void flush(int64_t i0, int cnt) {
    const int lane = lane_id();
    if (lane < cnt) stg8((uintptr_t)(out + i0 + lane), lo, hi);
  }
};

// ---- K7a ---------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_str_dict(JobDev* jobs, PageDev* pages, int64_t* doffs_arena) {
  JobDev& job = jobs[blockIdx.x];
  if (job.status == kCAPACITY || !(job.flags & 2) || job.dict_page < 0) return;
  PageDev& dp = pages[job.page_base + job.dict_page];
  if (dp.read_status != kOK) return;
  const int64_t cnt = dp.num_values;
  PQG_G int64_t* doffs = gmut(doffs_arena) + job.doffs_base;
  RegWindow win;
  win.init(gconst(job.dict_data), job.dict_len);
  LaneBatch lb{doffs + 1, 0u, 0u};
  int64_t used, chars;
  const int st = walk_lengths(win, cnt, &used, &chars, [&](int64_t i, int64_t pos, int64_t) { lb.put(i, pos); });
  const int64_t done = st == kOK ? cnt : 0;
  if (st == kOK) lb.flush(cnt & ~(int64_t)63, (int)(cnt & 63));
  __builtin_amdgcn_wave_barrier();
  if (lane_id() == 0) {
    if (st == kOK) {
      doffs[0] = 0;
      job.dict_offs = (const int64_t*)doffs;
      job.dict_count = done;
    } else {
      dp.read_status = st;  // dictPageReader.read: any error is fatal (page_dict.go:50-56)
    }
  }
}

// ---- dictionary sinks (type_dict.go:39-59 over variable-length entries) ------
struct StrDictCount {
  const PQG_G int64_t* doffs;
  int64_t count;
  int64_t bad;   // first value index with an invalid key
  int64_t sum;   // lane's chars
  __device__ __forceinline__ void group(const uint32_t (&v)[kGroup][8], const uint32_t (&i0)[kGroup],
                                        const int (&cnt)[kGroup]) {
#pragma unroll
    for (int b = 0; b < kGroup; b++)
      for (int q = 0; q < cnt[b]; q++) {
        const uint32_t key = v[b][q];
        if ((int64_t)key < count) sum += doffs[key + 1] - doffs[key] - 4;
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

struct StrDictWrite {
  gu8 chars;                 // chunk chars + the page's char offset
  PQG_G int64_t* ends;       // chunk offsets + value_offset + 1
  int64_t base;              // the page's char offset in the chunk
  gcu8 dict;                 // dictionary page block
  const PQG_G int64_t* doffs;
  int64_t count;
  int64_t carry;             // page chars written before this group (wave-uniform)
  __device__ __forceinline__ void group(const uint32_t (&v)[kGroup][8], const uint32_t (&i0)[kGroup],
                                        const int (&cnt)[kGroup]) {
#pragma unroll
    for (int b = 0; b < kGroup; b++) {
      int64_t src[8];
      int32_t len[8];
      int64_t s = 0;
#pragma unroll
      for (int q = 0; q < 8; q++) {
        len[q] = 0;
        src[q] = 0;
        if (q < cnt[b] && (int64_t)v[b][q] < count) {
          const int64_t a = doffs[v[b][q]];
          len[q] = (int32_t)(doffs[v[b][q] + 1] - a - 4);
          src[q] = a + 4;
        }
        s += len[q];
      }
      int64_t tot;
      int64_t pos = carry + wave_excl_scan_i64(s, &tot);
      for (int q = 0; q < cnt[b]; q++) {
        copy_bytes(chars + pos, dict + src[q], len[q]);
        pos += len[q];
        ends[i0[b] + q] = base + pos;
      }
      carry += tot;
    }
  }
};

// ---- K7b ---------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_str_count(JobDev* jobs, PageDev* pages, const int* list, const int* total,
                                                  int* queue, int64_t* offs_arena, const HStream* streams,
                                                  const RunEnt* runs, const BlockDesc* blks) {
  __shared__ __attribute__((aligned(16))) ExpandShared sh;
  const int lane = lane_id();
  for (;;) {
    const int t = queue_next(queue);
    if (t >= *total) return;
    const int pidx = __builtin_amdgcn_readfirstlane(list[t]);
    const PageDev pg = pages[pidx];
    if (pg.read_status != kOK || (pg.page_type != 0 && pg.page_type != 3)) continue;
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
      RegWindow win;
      win.init(val, vn);
      LaneBatch lb{gmut(offs_arena) + job.offs_base + pg.value_offset + 1, 0u, 0u};
      int64_t used;
      de = walk_lengths(win, nn, &used, &chars, [&](int64_t i, int64_t, int64_t cum) { lb.put(i, cum); });
      if (de == kOK) lb.flush(nn & ~(int64_t)63, (int)(nn & 63));
    } else if (enc == 8) {
      const int64_t dcount = job.dict_offs ? job.dict_count : 0;
      const int dw = pg.dict_width;
      if (dw == 0) {
        // zero-width indices: key 0 forever (hybrid_decoder.go:84-86)
        if (dcount < 1) de = kDICT_INDEX;
        else chars = nn * (gconst(job.dict_offs)[1] - 4);
      } else {
        const HStream S = streams[pg.hs_val];
        const int serr = (S.status != kOK && S.produced < nn) ? S.status : kOK;
        StrDictCount sk{gconst(job.dict_offs ? job.dict_offs : (const int64_t*)offs_arena), dcount, nn, 0};
        hybrid_expand(S, runs, blks, nn, sh, sk);
        const int64_t bad = wave_min(sk.bad);
        chars = wave_sum(sk.sum);
        if (bad < nn && (serr == kOK || bad < S.produced)) de = kDICT_INDEX;
        else de = serr;
      }
    } else {
      de = kUNSUPPORTED;
    }
    if (lane == 0) {
      PageDev& o = pages[pidx];
      o.chars = chars;
      if (de != kOK) o.decode_status = de;
    }
  }
}

// ---- K7c ---------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_char_scan(JobDev* jobs, PageDev* pages, int64_t* offs_arena) {
  __shared__ int64_t part[5];
  JobDev& job = jobs[blockIdx.x];
  if (job.value_width != 0 || job.status == kCAPACITY) return;
  const int np = job.num_pages < job.page_cap ? job.num_pages : job.page_cap;
  int64_t carry = 0;
  for (int b = 0; b < np; b += 256) {
    const int i = b + threadIdx.x;
    int64_t v = 0;
    if (i < np) {
      const PageDev& pg = pages[job.page_base + i];
      if ((pg.page_type == 0 || pg.page_type == 3) && pg.read_status == kOK && pg.decode_status == kOK) v = pg.chars;
    }
    int64_t tot;
    const int64_t ex = block_excl_scan<256>(v, &tot, part);
    if (i < np) pages[job.page_base + i].char_offset = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) {
    job.values_bytes = carry;
    if (carry > job.value_cap) job.status = kCAPACITY;
    offs_arena[job.offs_base] = 0;
  }
}

// ---- K7d ---------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_str_write(JobDev* jobs, PageDev* pages, const int* list, const int* total,
                                                  int* queue, uint8_t* value_arena, int64_t* offs_arena,
                                                  const HStream* streams, const RunEnt* runs, const BlockDesc* blks) {
  __shared__ __attribute__((aligned(16))) ExpandShared sh;
  const int lane = lane_id();
  for (;;) {
    const int t = queue_next(queue);
    if (t >= *total) return;
    const int pidx = __builtin_amdgcn_readfirstlane(list[t]);
    const PageDev pg = pages[pidx];
    if (pg.read_status != kOK || pg.decode_status != kOK || (pg.page_type != 0 && pg.page_type != 3)) continue;
    const JobDev job = jobs[pg.job];
    if (job.status == kCAPACITY) continue;
    const int64_t nn = pg.not_null;
    if (nn == 0) continue;
    const gu8 chars = gmut(value_arena) + job.value_base + pg.char_offset;
    PQG_G int64_t* ends = gmut(offs_arena) + job.offs_base + pg.value_offset + 1;
    const int64_t base = pg.char_offset;
    if (pg.encoding == 0) {
      // PLAIN: value i's record starts at (its chars' start) + 4 (i + 1) - 4
      const gcu8 val = gconst(pg.val);
      int64_t prev = 0;  // page-relative end of the value before the batch
      for (int64_t i0 = 0; i0 < nn; i0 += 64) {
        const int64_t i = i0 + lane;
        int64_t e = 0;
        if (i < nn) e = ends[i];
        int64_t s = __shfl_up(e, 1, 64);
        if (lane == 0) s = prev;
        if (i < nn) {
          copy_bytes(chars + s, val + s + 4 * (i + 1), e - s);
          ends[i] = base + e;
        }
        prev = __shfl(e, 63, 64);
      }
    } else {
      const gcu8 dict = gconst(job.dict_data);
      const PQG_G int64_t* doffs = gconst(job.dict_offs);
      if (pg.dict_width == 0) {
        const int64_t l = doffs[1] - 4;
        for (int64_t i = lane; i < nn; i += 64) {
          copy_bytes(chars + i * l, dict + 4, l);
          ends[i] = base + (i + 1) * l;
        }
      } else {
        const HStream S = streams[pg.hs_val];
        StrDictWrite sk{chars, ends, base, dict, doffs, job.dict_count, 0};
        hybrid_expand(S, runs, blks, nn, sh, sk);
      }
    }
  }
}

}  // namespace pqg
