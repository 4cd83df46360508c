// pqg_kernels.hip — gfx950 kernels of the Parquet column-chunk decoder.
//
// Pipeline per batch of chunk jobs (one HIP stream, see pqg_runtime.hip):
//   K1  k_scan_pages      page-header walk per chunk (readPages, chunk_reader.go:206-284)
//   K1b k_page_list       compact list of all pages + per-job counters
//   K2  k_snappy          snappy block decompression (compress.go:90-122, snappy decode.go)
//   K3a k_levels          level streams: V1 initSize / V2 raw, hybrid RLE/bit-pack decode
//                         (hybrid_decoder.go:57-166, decodePackedArray helpers.go:131-147)
//   K3s k_nn_scan         per-chunk prefix of notNull → value offsets (readPageData :380-402)
//   K4  k_values          values[:nn] per page: PLAIN / RLE_DICTIONARY gather /
//                         DELTA_BINARY_PACKED / boolean (type_*.go, type_dict.go:39-59,
//                         deltabp_decoder.go:114-334)
//   K5  k_finalize        chunk status in reference order
// All kernels are integer / byte work (HBM-bound; no MFMA).  Work is dealt to
// 64-lane wavefronts from an atomic page queue, one wave per page.
#include <hip/hip_runtime.h>

#include "pqg_common.h"
#include "pqg_device.h"
#include "pqg_thrift.h"

namespace pqg {

// Byte source over the LDS window, for the thrift reader.
struct WinSrc {
  Window* w;
  __device__ int get(int64_t i) { return w->get(i); }
};

__device__ __forceinline__ int bits_len(uint32_t v) { return v ? 32 - __builtin_clz(v) : 0; }

// getValuesDecoder chunk_reader.go:143-196 (DELTA_*_BYTE_ARRAY are outside this build)
__device__ __forceinline__ int values_supported(int type, int type_length, int enc) {
  switch (type) {
    case 0: return enc == 0 || enc == 3 || enc == 8;
    case 6: return enc == 0 || enc == 8;
    case 7: return type_length >= 0 && (enc == 0 || enc == 8);
    case 3: case 4: case 5: return enc == 0 || enc == 8;
    case 1: case 2: return enc == 0 || enc == 5 || enc == 8;
  }
  return 0;
}

// ============================================================================
// K1: page-header walk — one wave per chunk.
// ============================================================================
struct ScanShared {
  uint8_t win[kWin];
  SkipFrame frames[kMaxFrames];
  int16_t last[kMaxLast];
};

__global__ void __launch_bounds__(64) k_scan_pages(JobDev* jobs, PageDev* pages, int n_jobs) {
  __shared__ __attribute__((aligned(16))) ScanShared sh;
  int j = blockIdx.x;
  if (j >= n_jobs) return;
  JobDev& job = jobs[j];
  Window win{job.data, job.data_len, kFarAway, sh.win};
  int64_t pos = 0;
  int np = 0;
  int status = kOK;
  bool dict_seen = false;
  int dict_page = -1;
  int64_t scratch = 0;
  int64_t slots = 0;
  const int lane = lane_id();
  const int64_t tcs = job.tcs;
  while (tcs - pos > 0) {
    Compact<WinSrc> c;
    c.src.w = &win;
    c.pos = pos;
    c.frames = sh.frames;
    c.last = sh.last;
    c.nlast = 0;
    c.last_id = 0;
    c.bool_set = false;
    c.bool_val = false;
    PageHdr h;
    int e = c.read_page_header(&h);
    PageDev pg;
    pg.header_offset = pos;
    pg.payload_offset = c.pos;
    pg.slot_offset = slots;
    pg.value_offset = 0;
    pg.scratch_offset = -1;
    pg.block = nullptr;
    pg.block_len = 0;
    pg.rep = pg.def = pg.val = nullptr;
    pg.rep_n = pg.def_n = pg.val_n = 0;
    pg.page_type = h.type;
    pg.encoding = h.encoding;
    pg.num_values = 0;
    pg.csize = h.csize;
    pg.usize = h.usize;
    pg.def_len = h.v2_def_len;
    pg.rep_len = h.v2_rep_len;
    pg.def_enc = h.def_enc;
    pg.rep_enc = h.rep_enc;
    pg.job = j;
    pg.read_status = kOK;
    pg.decode_status = kOK;
    pg.not_null = 0;
    pg.flags = 0;
    pg.dict_width = 0;
    pg.pad = 0;
    int64_t next = pos;
    if (e == kOK) {
      const int64_t payload = c.pos;
      if (h.type == 2) {  // DICTIONARY_PAGE (page_dict.go:30-64, chunk_reader.go:221-251)
        pg.num_values = h.has_dict ? h.num_values : 0;
        if (dict_seen) {
          e = kDICT_PAGE;
        } else if (job.type == 0 || (job.type == 7 && job.type_length < 0)) {
          e = kUNSUPPORTED;
        } else if (!h.has_dict || h.num_values < 0) {
          e = kPAGE_HEADER;
        } else if (h.encoding != 0 && h.encoding != 2) {
          e = kUNSUPPORTED;
        } else if (h.csize < 0 || h.usize < 0) {
          e = kPAGE_HEADER;
        } else if (job.data_len - payload < (int64_t)h.csize) {
          e = kSIZE;
        } else if (job.codec == 0) {
          if (h.csize != h.usize) e = kSIZE;
        } else if (job.codec == 1) {
          pg.scratch_offset = scratch;
          scratch += ((int64_t)h.usize + 15) & ~(int64_t)15;
        } else {
          e = kUNSUPPORTED;
        }
        next = payload + h.csize;
        if (e == kOK) {
          dict_seen = true;
          dict_page = np;
          if (job.has_dict_off) next = job.data_page_offset;
        }
      } else if (h.type == 0) {  // DATA_PAGE (page_v1.go:57-108)
        pg.num_values = h.has_dph ? h.num_values : 0;
        int wr = bits_len((uint32_t)job.max_rep), wd = bits_len((uint32_t)job.max_def);
        int enc = h.encoding == 2 ? 8 : h.encoding;
        pg.encoding = enc;
        if (!h.has_dph) e = kPAGE_HEADER;
        else if (job.max_rep > 0 && h.rep_enc != 3) e = kUNSUPPORTED;
        else if (job.max_def > 0 && h.def_enc != 3) e = kUNSUPPORTED;
        else if (h.num_values < 0) e = kPAGE_HEADER;
        else if (h.csize < 0 || h.usize < 0) e = kPAGE_HEADER;
        else if (job.data_len - payload < (int64_t)h.csize) e = kSIZE;
        else if (job.codec == 0 && h.csize != h.usize) e = kSIZE;
        else if (job.codec != 0 && job.codec != 1) e = kUNSUPPORTED;
        else if (job.codec == 0 && !values_supported(job.type, job.type_length, enc)) e = kUNSUPPORTED;
        (void)wr;
        (void)wd;
        if (e == kOK && job.codec == 1) {
          pg.scratch_offset = scratch;
          scratch += ((int64_t)h.usize + 15) & ~(int64_t)15;
        }
        next = payload + h.csize;
      } else if (h.type == 3) {  // DATA_PAGE_V2 (page_v2.go:56-129)
        pg.num_values = h.has_v2 ? h.num_values : 0;
        int enc = h.encoding == 2 ? 8 : h.encoding;
        pg.encoding = enc;
        int32_t levels = (int32_t)((uint32_t)h.v2_rep_len + (uint32_t)h.v2_def_len);
        int32_t cs = (int32_t)((uint32_t)h.csize - (uint32_t)levels);
        int32_t us = (int32_t)((uint32_t)h.usize - (uint32_t)levels);
        int64_t body = payload + (levels > 0 ? levels : 0);
        if (!h.has_v2) e = kPAGE_HEADER;
        else if (h.num_values < 0 || h.v2_rep_len < 0 || h.v2_def_len < 0) e = kPAGE_HEADER;
        else if (!values_supported(job.type, job.type_length, enc)) e = kUNSUPPORTED;
        else if (levels > 0 && job.data_len - payload < (int64_t)levels) e = kEOF;
        else if (cs < 0 || us < 0) e = kPAGE_HEADER;
        else if (job.data_len - body < (int64_t)cs) e = kSIZE;
        else if (job.codec == 0 && cs != us) e = kSIZE;
        else if (job.codec != 0 && job.codec != 1) e = kUNSUPPORTED;
        if (e == kOK && job.codec == 1) {
          pg.scratch_offset = scratch;
          scratch += ((int64_t)us + 15) & ~(int64_t)15;
        }
        next = body + cs;
      } else {
        e = kUNSUPPORTED;  // "DATA_PAGE or DATA_PAGE_V2 type supported"
      }
    }
    pg.read_status = e;
    if (np < job.page_cap && lane == 0) pages[job.page_base + np] = pg;
    if (h.type == 0 || h.type == 3) slots += (e == kOK) ? pg.num_values : 0;
    np++;
    if (e != kOK) {
      status = e;
      break;
    }
    pos = next;
  }
  if (lane == 0) {
    job.num_pages = np;
    job.dict_page = dict_page;
    job.scan_status = status;
    job.need_scratch = scratch;
    job.num_slots = slots;
    job.dict_data = nullptr;
    job.dict_count = 0;
    job.dict_len = 0;
    job.dict_offs = nullptr;
    job.status = kOK;
    job.error_page = -1;
    job.flags = 0;
    if (np > job.page_cap || slots > job.slot_cap || scratch > job.scratch_cap) job.status = kCAPACITY;
  }
}

// ============================================================================
// K1b: compact list of page indices over all jobs.
// ============================================================================
__global__ void k_page_list(JobDev* jobs, int n_jobs, int* list, int list_cap, int* total, int* queues) {
  int off = 0;
  for (int j = 0; j < n_jobs; j++) {
    int n = jobs[j].num_pages;
    if (n > jobs[j].page_cap) n = jobs[j].page_cap;
    if (jobs[j].status == kCAPACITY) n = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x)
      if (off + i < list_cap) list[off + i] = (int)(jobs[j].page_base + i);
    off += n;
  }
  if (threadIdx.x == 0) {
    *total = off < list_cap ? off : list_cap;
    for (int q = 0; q < 8; q++) queues[q] = 0;
  }
}

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

__device__ __forceinline__ uint32_t l2_load_u32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool kLds>
__device__ int snappy_body(Window& win, int64_t s, int64_t slen, uint8_t* dst_g, uint8_t* dst_l, int64_t dlen) {
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
      const uint8_t* src = win.p + s;
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
        uint32_t wv = l2_load_u32((const uint32_t*)(a & ~(uintptr_t)3));
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
    int t = 0;
    if (lane == 0) t = atomicAdd(queue, 1);
    t = __shfl(t, 0, 64);
    if (t >= *total) return;
    PageDev& pg = pages[list[t]];
    if (pg.read_status != kOK || pg.scratch_offset < 0) continue;
    JobDev& job = jobs[pg.job];
    // compressed block location (V2: after the raw level bytes)
    int64_t src_off = pg.payload_offset;
    int64_t clen = pg.csize, ulen = pg.usize;
    if (pg.page_type == 3) {
      int32_t levels = (int32_t)((uint32_t)pg.rep_len + (uint32_t)pg.def_len);
      if (levels > 0) src_off += levels;
      clen = (int32_t)((uint32_t)pg.csize - (uint32_t)levels);
      ulen = (int32_t)((uint32_t)pg.usize - (uint32_t)levels);
    }
    Window win{job.data + src_off, clen, kFarAway, sh.win};
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
    uint8_t* dst = scratch + job.scratch_base + pg.scratch_offset;
    if (e == kOK) {
      if (ulen <= kSnapLds) {
        e = snappy_body<true>(win, hl, clen, nullptr, sh.out, ulen);
        if (e == kOK)
          for (int64_t i = lane; i < ulen; i += 64) dst[i] = sh.out[i];
      } else {
        e = snappy_body<false>(win, hl, clen, dst, nullptr, ulen);
      }
    }
    // V1: getValuesDecoder runs after the block is decompressed (page_v1.go:91-97)
    if (e == kOK && pg.page_type == 0 && !values_supported(job.type, job.type_length, pg.encoding)) e = kUNSUPPORTED;
    if (lane == 0 && e != kOK) pg.read_status = e;
  }
}

// ============================================================================
// Hybrid RLE / bit-packed decoder — wave level.
// hybridDecoder.next hybrid_decoder.go:82-166: a wave-uniform walk over the
// run headers through an LDS window builds a table of runs; lanes then expand
// the table, 4 consecutive values per lane.
// ============================================================================
constexpr int kRuns = 128;

struct Run {
  int64_t out_start;
  int64_t bitpos;   // BP: bit offset of value 0 of the run in the stream
  int32_t count;    // values taken from this run
  int32_t kind;     // 0 RLE, 1 bit-packed
  uint32_t value;   // RLE value
  int32_t pad;
};

struct HybridShared {
  uint8_t win[kWin];
  Run runs[kRuns];
};

// uvarint + readUVariant32 (helpers.go:149-165) through the window.
__device__ __forceinline__ int read_uvar32(Window& w, int64_t& pos, uint32_t* out) {
  uint64_t x = 0;
  unsigned s = 0;
  for (int i = 0;; i++) {
    int b = w.get(pos);
    if (b < 0) return kEOF;
    pos++;
    if (b < 0x80) {
      if (i > 9 || (i == 9 && b > 1)) return kRLE;
      x |= (s < 64 ? (uint64_t)b << s : 0);
      if (x > 0x7fffffffull) return kRLE;
      *out = (uint32_t)x;
      return kOK;
    }
    if (s < 64) x |= (uint64_t)(b & 0x7f) << s;
    s += 7;
  }
}

// Sink interface: void put4(int64_t idx0, const uint32_t v[4], int cnt)
template <class Sink>
__device__ int hybrid_decode(const uint8_t* s, int64_t n, int64_t readable, int w, int64_t count, HybridShared& sh,
                             Sink& sink, int64_t* err_at) {
  const int lane = lane_id();
  *err_at = count;
  if (w == 0) {  // infinite zeros, nothing read (hybrid_decoder.go:84-86)
    for (int64_t b = 0; b < count; b += 256) {
      int64_t i0 = b + lane * 4;
      uint32_t v[4] = {0, 0, 0, 0};
      int cnt = (int)min((int64_t)4, count - i0);
      if (cnt > 0) sink.put4(i0, v, cnt);
    }
    return kOK;
  }
  Window win{s, n, kFarAway, sh.win};
  const int rb = (w + 7) / 8;
  int64_t pos = 0, produced = 0;
  int status = kOK;
  while (produced < count && status == kOK) {
    int nr = 0;
    int64_t walk = produced;
    while (nr < kRuns && walk < count) {
      uint32_t h;
      int e = read_uvar32(win, pos, &h);
      if (e) { status = e; break; }
      Run r;
      r.out_start = walk;
      r.pad = 0;
      if (h & 1) {
        int64_t groups = h >> 1;
        if (groups == 0) { status = kRLE; break; }
        int64_t take = groups * 8;
        if (take > count - walk) take = count - walk;
        int64_t need = (take + 7) / 8;
        // groups whose first byte lies inside the stream (short read is zero padded)
        int64_t ok = pos < n ? (n - pos + w - 1) / w : 0;
        if (ok < need) {
          take = ok * 8;
          status = kEOF;
        }
        r.kind = 1;
        r.bitpos = pos * 8;
        r.value = 0;
        r.count = (int32_t)take;
        pos += groups * w;
      } else {
        int64_t cnt = h >> 1;
        if (cnt == 0) { status = kRLE; break; }
        uint32_t v = 0;
        if (pos >= n || n - pos < rb) { status = kEOF; break; }
        for (int k = 0; k < rb; k++) v |= (uint32_t)win.get(pos + k) << (8 * k);
        pos += rb;
        if (w < 32 && (v >> w) != 0) { status = kRLE; break; }
        int64_t take = cnt < count - walk ? cnt : count - walk;
        r.kind = 0;
        r.bitpos = 0;
        r.value = v;
        r.count = (int32_t)take;
      }
      if (r.count > 0) {
        if (lane == 0) sh.runs[nr] = r;
        nr++;
      }
      walk += r.count;
      if (status) break;
    }
    __builtin_amdgcn_wave_barrier();
    // expand outputs [produced, walk) from runs[0, nr)
    for (int64_t b = produced; b < walk; b += 256) {
      int64_t i0 = b + lane * 4;
      int cnt = (int)min((int64_t)4, walk - i0);
      if (cnt > 0) {
        // largest r with runs[r].out_start <= i0
        int lo = 0, hi = nr - 1;
        while (lo < hi) {
          int mid = (lo + hi + 1) >> 1;
          if (sh.runs[mid].out_start <= i0) lo = mid; else hi = mid - 1;
        }
        int r = lo;
        uint32_t v[4] = {0, 0, 0, 0};
        for (int k = 0; k < cnt; k++) {
          int64_t i = i0 + k;
          while (r + 1 < nr && sh.runs[r + 1].out_start <= i) r++;
          const Run& R = sh.runs[r];
          if (R.kind == 0) v[k] = R.value;
          else v[k] = extract_bits32(s, readable, n, R.bitpos + (i - R.out_start) * w, w);
        }
        sink.put4(i0, v, cnt);
      }
    }
    __builtin_amdgcn_wave_barrier();
    produced = walk;
  }
  if (status) *err_at = produced;
  return status;
}

// ============================================================================
// K3a: levels — one wave per data page.
// ============================================================================
struct LevelSink {
  uint8_t* out;
  int32_t maxl;
  int64_t nn;
  __device__ void put4(int64_t i0, const uint32_t v[4], int cnt) {
    for (int k = 0; k < cnt; k++) {
      out[i0 + k] = (uint8_t)v[k];
      nn += (v[k] == (uint32_t)maxl);
    }
  }
};
struct CountSink {  // levels of a column whose level output is not stored
  int32_t maxl;
  int64_t nn;
  __device__ void put4(int64_t, const uint32_t v[4], int cnt) {
    for (int k = 0; k < cnt; k++) nn += (v[k] == (uint32_t)maxl);
  }
};

__device__ __forceinline__ uint32_t rd_u32(const uint8_t* p) {
  return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

__global__ void __launch_bounds__(64) k_levels(JobDev* jobs, PageDev* pages, const int* list, const int* total,
                                               int* queue, uint8_t* scratch, uint8_t* def_arena,
                                               uint8_t* rep_arena) {
  __shared__ __attribute__((aligned(16))) HybridShared sh;
  const int lane = lane_id();
  for (;;) {
    int t = 0;
    if (lane == 0) t = atomicAdd(queue, 1);
    t = __shfl(t, 0, 64);
    if (t >= *total) return;
    PageDev& pg = pages[list[t]];
    if (pg.read_status != kOK || (pg.page_type != 0 && pg.page_type != 3)) continue;
    JobDev& job = jobs[pg.job];
    if (job.status == kCAPACITY) continue;
    // ---- resolve the page block and the level / value streams (read phase)
    const uint8_t* block;
    int64_t blen;
    int32_t levels = 0;
    if (pg.page_type == 3) {
      levels = (int32_t)((uint32_t)pg.rep_len + (uint32_t)pg.def_len);
      blen = (int32_t)((uint32_t)pg.csize - (uint32_t)levels);
      if (pg.scratch_offset >= 0) blen = (int32_t)((uint32_t)pg.usize - (uint32_t)levels);
    } else {
      blen = pg.scratch_offset >= 0 ? pg.usize : pg.csize;
    }
    if (pg.scratch_offset >= 0) block = scratch + job.scratch_base + pg.scratch_offset;
    else block = job.data + pg.payload_offset + (levels > 0 ? levels : 0);
    // readable bytes from `block` (for wide loads): to the end of its buffer
    int64_t readable = pg.scratch_offset >= 0 ? blen : job.data_len - (block - job.data);
    const int wr = bits_len((uint32_t)job.max_rep), wd = bits_len((uint32_t)job.max_def);
    const uint8_t *rep = nullptr, *def = nullptr;
    int64_t rep_n = -1, def_n = -1, rep_rd = 0, def_rd = 0;  // -1: decoder not initialised
    int64_t vpos = 0;
    int e = kOK;
    if (pg.page_type == 0) {
      // rDecoder.initSize then dDecoder.initSize (page_v1.go:99-105)
      if (job.max_rep > 0) {
        if (blen - vpos < 4) e = kEOF;
        else {
          int64_t sz = rd_u32(block + vpos);
          int64_t take = min(sz, blen - vpos - 4);
          rep = block + vpos + 4; rep_n = take; rep_rd = readable - vpos - 4;
          vpos += 4 + take;
        }
      }
      if (e == kOK && job.max_def > 0) {
        if (blen - vpos < 4) e = kEOF;
        else {
          int64_t sz = rd_u32(block + vpos);
          int64_t take = min(sz, blen - vpos - 4);
          def = block + vpos + 4; def_n = take; def_rd = readable - vpos - 4;
          vpos += 4 + take;
        }
      }
    } else {
      const uint8_t* lv = job.data + pg.payload_offset;
      int64_t lv_rd = job.data_len - pg.payload_offset;
      if (levels > 0 && pg.rep_len > 0) { rep = lv; rep_n = pg.rep_len; rep_rd = lv_rd; }
      if (levels > 0 && pg.def_len > 0) { def = lv + pg.rep_len; def_n = levels - pg.rep_len; def_rd = lv_rd - pg.rep_len; }
    }
    if (e != kOK) {
      if (lane == 0) pg.read_status = e;
      continue;
    }
    if (lane == 0) {
      pg.block = block;
      pg.block_len = blen;
      pg.val = block + vpos;
      pg.val_n = blen - vpos;
      pg.rep = rep; pg.rep_n = rep_n;
      pg.def = def; pg.def_n = def_n;
    }
    // ---- decode phase: readValues (page_v1.go:27-55)
    const int64_t n = pg.num_values;
    int64_t nn = 0;
    int de = kOK;
    int64_t err_at;
    if (n > 0) {
      if (job.max_rep > 0) {
        if (rep_n < 0) de = kLEVELS;  // V2 with zero-length levels: "reader is not initialized"
        else {
          LevelSink sk{rep_arena + job.slot_base + pg.slot_offset, job.max_rep, 0};
          de = hybrid_decode(rep, rep_n, rep_rd, wr, n, sh, sk, &err_at);
        }
      }
      if (de == kOK) {
        if (job.max_def > 0) {
          if (def_n < 0) de = kLEVELS;
          else {
            LevelSink sk{def_arena + job.slot_base + pg.slot_offset, job.max_def, 0};
            de = hybrid_decode(def, def_n, def_rd, wd, n, sh, sk, &err_at);
            nn = wave_sum(sk.nn);
          }
        } else {
          nn = n;
        }
      }
    }
    if (lane == 0) {
      pg.not_null = (int32_t)nn;
      if (de != kOK) pg.decode_status = de;
    }
  }
}

// ============================================================================
// K3s: notNull prefix per chunk + dictionary-page resolution.
// One 256-thread block per job.
// ============================================================================
__global__ void __launch_bounds__(256) k_nn_scan(JobDev* jobs, PageDev* pages, uint8_t* scratch) {
  __shared__ int64_t part[256];
  __shared__ int64_t carry;
  JobDev& job = jobs[blockIdx.x];
  int np = job.num_pages < job.page_cap ? job.num_pages : job.page_cap;
  if (job.status == kCAPACITY) np = 0;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int b = 0; b < np; b += 256) {
    int i = b + threadIdx.x;
    int64_t v = 0;
    if (i < np) {
      PageDev& pg = pages[job.page_base + i];
      if (pg.page_type == 0 || pg.page_type == 3) v = pg.not_null;
    }
    part[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
      int64_t t = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
      __syncthreads();
      part[threadIdx.x] += t;
      __syncthreads();
    }
    if (i < np) pages[job.page_base + i].value_offset = carry + part[threadIdx.x] - v;
    __syncthreads();
    if (threadIdx.x == 255) carry += part[255];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    job.num_values = carry;
    int64_t vb = job.value_width > 0 ? carry * job.value_width : 0;
    if (job.value_width > 0 && vb > job.value_cap) job.status = kCAPACITY;
    job.values_bytes = vb;
    // dictionary page (page_dict.go:30-64): PLAIN entries of the column type.
    if (job.dict_page >= 0 && job.dict_page < np) {
      PageDev& dp = pages[job.page_base + job.dict_page];
      if (dp.read_status == kOK) {
        const uint8_t* blk = dp.scratch_offset >= 0 ? scratch + job.scratch_base + dp.scratch_offset
                                                    : job.data + dp.payload_offset;
        int64_t blen = dp.usize;
        int64_t cnt = dp.num_values;
        int w = job.value_width;
        dp.block = blk;
        dp.block_len = blen;
        if (w > 0) {
          if (job.type == 3) {  // INT96: a partial final entry is left nil, not an error (Q8)
            int64_t full = blen / 12, rem = blen % 12;
            if (cnt > full + (rem > 0 ? 1 : 0)) dp.read_status = kEOF;
            else if (cnt == full + 1 && rem > 0) job.flags |= 1;
          } else if (cnt * w > blen) {
            dp.read_status = kEOF;
          }
          job.dict_data = blk;
          job.dict_count = cnt;
          job.dict_len = blen;
        } else {
          dp.read_status = kUNSUPPORTED;  // variable-length dictionaries: k_dict_var (not in this build)
        }
      }
    }
  }
}

// ============================================================================
// K4: values — one wave per data page.
// ============================================================================
template <int W>
struct DictSink {  // gather dict[key] (type_dict.go:39-59), W bytes per entry
  uint8_t* out;
  const uint8_t* dict;
  int64_t count;
  int64_t bad;  // first index with an invalid key
  int64_t nil_key;  // INT96 partial final entry (-1: none)
  __device__ void put4(int64_t i0, const uint32_t v[4], int cnt) {
    for (int k = 0; k < cnt; k++) {
      uint32_t key = v[k];
      int64_t i = i0 + k;
      if ((int64_t)key >= count || (int32_t)key < 0) {
        bad = i < bad ? i : bad;
        continue;
      }
      if (W == 4) {
        *(uint32_t*)(out + i * 4) = *(const uint32_t*)(dict + (int64_t)key * 4);
      } else if (W == 8) {
        const uint32_t* s = (const uint32_t*)(dict + (int64_t)key * 8);
        uint32_t* d = (uint32_t*)(out + i * 8);
        d[0] = s[0];
        d[1] = s[1];
      } else {
        const uint8_t* s = dict + (int64_t)key * W;
        for (int b = 0; b < W; b++) out[i * W + b] = ((int64_t)key == nil_key) ? 0 : s[b];
      }
    }
  }
};
struct DictSinkN {  // runtime width
  uint8_t* out;
  const uint8_t* dict;
  int64_t count;
  int64_t bad;
  int w;
  int64_t nil_key;
  __device__ void put4(int64_t i0, const uint32_t v[4], int cnt) {
    for (int k = 0; k < cnt; k++) {
      uint32_t key = v[k];
      int64_t i = i0 + k;
      if ((int64_t)key >= count || (int32_t)key < 0) {
        bad = i < bad ? i : bad;
        continue;
      }
      const uint8_t* s = dict + (int64_t)key * w;
      for (int b = 0; b < w; b++) out[i * w + b] = ((int64_t)key == nil_key) ? 0 : s[b];
    }
  }
};
struct BoolSink {
  uint8_t* out;
  __device__ void put4(int64_t i0, const uint32_t v[4], int cnt) {
    for (int k = 0; k < cnt; k++) out[i0 + k] = v[k] == 1;
  }
};

// ---- DELTA_BINARY_PACKED (deltabp_decoder.go) ------------------------------
constexpr int kBlocks = 64;
constexpr int kMaxMb = 8;

struct DbpShared {
  uint8_t win[kWin];
  int64_t body[kBlocks];                // stream offset of the block's first miniblock
  uint64_t mind[kBlocks];               // min delta (as unsigned for wrapping adds)
  uint8_t widths[kBlocks][kMaxMb];
  int64_t mb_off[kBlocks][kMaxMb];      // stream offset of each miniblock
};

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

// Values of a DBP page: emulates deltaBitPackDecoder{32,64}.next for positions
// [0, nn).  Regular layout (miniblock value count a multiple of 8, <= kMaxMb
// miniblocks): wave-parallel unpack + wrapping scan; otherwise one lane.
__device__ int dbp_decode(const uint8_t* s, int64_t n, int64_t readable, bool is64, int64_t nn, uint8_t* out,
                          DbpShared& sh, int stage /*0 = header only (read phase), 1 = decode*/) {
  const int lane = lane_id();
  Window win{s, n, kFarAway, sh.win};
  int64_t pos = 0;
  int32_t bs, mbc, total;
  uint64_t first;
  int e;
  // readBlockHeader
  if ((e = read_u32var_delta(win, pos, &bs))) return e;
  if (bs <= 0 && bs % 128 != 0) return kDELTA;
  if ((e = read_u32var_delta(win, pos, &mbc))) return e;
  if (mbc <= 0 || bs % mbc != 0) return kDELTA;
  int32_t mbvc = bs / mbc;
  if (mbvc == 0) return kDELTA;
  if ((e = read_u32var_delta(win, pos, &total))) return e;
  if ((e = read_signed(win, pos, is64, &first))) return e;
  const int maxw = is64 ? 64 : 32;
  // first readMiniBlockHeader (part of init)
  {
    int64_t p = pos;
    uint64_t md;
    if ((e = read_signed(win, p, is64, &md))) return e;
    if (n - p < mbc) return kEOF;
    for (int m = 0; m < mbc; m++)
      if (win.get(p + m) > maxw) return kBIT_WIDTH;
  }
  if (stage == 0) return kOK;
  const int64_t P = nn < total ? nn : total;  // positions actually produced before EOF
  const bool regular = (mbvc % 8 == 0) && mbc <= kMaxMb;
  if (!regular) {
    // ---- generic single-lane emulation of next() (rare layouts)
    int64_t rp = pos;
    int32_t cur_mb = mbc;  // force header read at position 0 semantics below
    uint64_t mind = 0, prev = first;
    uint8_t widths[256];
    int32_t cw = 0, mbpos = 0;
    uint64_t vals[8] = {0};
    // init already read the first miniblock header: emulate it
    {
      if ((e = read_signed(win, rp, is64, &mind))) return e;
      for (int m = 0; m < mbc && m < 256; m++) widths[m] = (uint8_t)win.get(rp + m);
      if (mbc > 256) return kUNSUPPORTED;
      rp += mbc;
      cur_mb = 0;
    }
    for (int64_t p = 0; p < nn; p++) {
      if (p >= total) return kEOF;
      if (p % 8 == 0) {
        if (p % mbvc == 0) {
          if (cur_mb >= mbc) {
            if ((e = read_signed(win, rp, is64, &mind))) return e;
            if (n - rp < mbc) return kEOF;
            for (int m = 0; m < mbc; m++) {
              int wv = win.get(rp + m);
              if (wv > maxw) return kBIT_WIDTH;
              widths[m] = (uint8_t)wv;
            }
            rp += mbc;
            cur_mb = 0;
          }
          cw = widths[cur_mb];
          mbpos = 0;
          cur_mb++;
        }
        if (n - rp < cw) return kEOF;
        for (int k = 0; k < 8; k++) vals[k] = extract_bits64(s, readable, n, rp * 8 + (int64_t)k * cw, cw);
        rp += cw;
        mbpos += cw;
        if (p + 8 >= total) {
          int64_t l = (int64_t)(mbvc / 8) * cw - mbpos;
          if (l < 0) return kDELTA;
          rp += l;  // padding skip, errors ignored
          if (rp > n) rp = n;
        }
      }
      if (lane == 0) {
        if (is64) *(uint64_t*)(out + p * 8) = prev;
        else *(uint32_t*)(out + p * 4) = (uint32_t)prev;
      }
      prev = prev + vals[p % 8] + mind;
      if (!is64) prev = (uint32_t)prev;
    }
    return kOK;
  }
  // ---- regular layout: walk blocks in batches, then unpack + scan
  uint64_t carry = first;  // value at the first position of the next tile
  int64_t blk_pos = pos;   // stream offset of the next block header
  int64_t p0 = 0;          // first position of the current batch
  bool first_block = true;
  while (p0 < P) {
    int nb = 0;
    int64_t p_end = p0;
    while (nb < kBlocks && p_end < P) {
      // block header: min delta + widths (the first one was read by init)
      int64_t hp = blk_pos;
      uint64_t md;
      if ((e = read_signed(win, hp, is64, &md))) return e;
      if (n - hp < mbc) return kEOF;
      int64_t off = hp + mbc;
      for (int m = 0; m < mbc; m++) {
        int wv = win.get(hp + m);
        if (wv > maxw) return kBIT_WIDTH;
        if (lane == 0) {
          sh.widths[nb][m] = (uint8_t)wv;
          sh.mb_off[nb][m] = off;
        }
        off += (int64_t)(mbvc / 8) * wv;
      }
      // groups of this block that positions < P read: each must be whole
      int64_t bp0 = p_end;
      int64_t bp1 = bp0 + bs < P ? bp0 + bs : P;
      int64_t last_group_pos = ((bp1 - 1) / 8) * 8;   // position of the last group read
      int64_t rel = last_group_pos - bp0;
      int m_last = (int)(rel / mbvc);
      int64_t g_in_mb = (rel % mbvc) / 8;
      int wl = win.get(hp + m_last);
      int64_t g_end = 0;
      {
        // offset of the last group's end
        int64_t mo = hp + mbc;
        for (int m = 0; m < m_last; m++) mo += (int64_t)(mbvc / 8) * win.get(hp + m);
        g_end = mo + (g_in_mb + 1) * wl;
      }
      if (g_end > n) return kEOF;
      if (lane == 0) {
        sh.body[nb] = hp + mbc;
        sh.mind[nb] = md;
      }
      nb++;
      p_end = bp1;
      blk_pos = off;
      first_block = false;
    }
    (void)first_block;
    __builtin_amdgcn_wave_barrier();
    // unpack + wrapping prefix over positions [p0, p_end): value(p) = carry + Σ deltas
    for (int64_t t0 = p0; t0 < p_end; t0 += 256) {
      uint64_t d[4];
      uint64_t local = 0;
      for (int k = 0; k < 4; k++) {
        int64_t p = t0 + lane * 4 + k;
        uint64_t dv = 0;
        if (p < p_end) {
          int64_t rel = p - p0;
          int b = (int)(rel / bs);
          int64_t r2 = rel - (int64_t)b * bs;
          int m = (int)(r2 / mbvc);
          int64_t j = r2 - (int64_t)m * mbvc;
          int wv = sh.widths[b][m];
          uint64_t x = extract_bits64(s, readable, n, sh.mb_off[b][m] * 8 + j * wv, wv);
          dv = x + sh.mind[b];
        }
        d[k] = dv;
        local += dv;
      }
      uint64_t incl = wave_incl_scan_u64(local);
      uint64_t run = carry + (incl - local);
      for (int k = 0; k < 4; k++) {
        int64_t p = t0 + lane * 4 + k;
        if (p < p_end) {
          if (is64) *(uint64_t*)(out + p * 8) = run;
          else *(uint32_t*)(out + p * 4) = (uint32_t)run;
        }
        run += d[k];
      }
      carry += __shfl(incl, 63, 64);
    }
    __builtin_amdgcn_wave_barrier();
    p0 = p_end;
  }
  if (nn > total) return kEOF;
  return kOK;
}

union ValuesShared {
  HybridShared hy;
  DbpShared dbp;
};

__global__ void __launch_bounds__(64) k_values(JobDev* jobs, PageDev* pages, const int* list, const int* total,
                                               int* queue, uint8_t* value_arena) {
  __shared__ __attribute__((aligned(16))) ValuesShared sh;
  const int lane = lane_id();
  for (;;) {
    int t = 0;
    if (lane == 0) t = atomicAdd(queue, 1);
    t = __shfl(t, 0, 64);
    if (t >= *total) return;
    PageDev& pg = pages[list[t]];
    if (pg.read_status != kOK || (pg.page_type != 0 && pg.page_type != 3)) continue;
    JobDev& job = jobs[pg.job];
    if (job.status == kCAPACITY) continue;
    const uint8_t* val = pg.val;
    const int64_t vn = pg.val_n;
    // readable bytes from val (for wide loads)
    int64_t readable = (pg.scratch_offset >= 0) ? vn : job.data_len - (val - job.data);
    const int enc = pg.encoding;
    const int64_t nn = pg.not_null;
    const int w = job.value_width;
    uint8_t* out = value_arena + job.value_base + pg.value_offset * (int64_t)w;
    // ---- valuesDecoder.init (read phase)
    int re = kOK;
    int dict_w = 0;
    if (enc == 8) {
      if (vn < 1) re = kEOF;
      else {
        dict_w = val[0];
        if (dict_w > 32) re = kBIT_WIDTH;
      }
    } else if (enc == 5) {
      re = dbp_decode(val, vn, readable, job.type == 2, 0, nullptr, sh.dbp, 0);
    } else if (enc == 3 && job.type == 0) {
      if (vn < 4) re = kEOF;
    }
    if (re != kOK) {
      if (lane == 0) pg.read_status = re;
      continue;
    }
    if (pg.decode_status != kOK || nn == 0) continue;
    // ---- decodeValues(val[:nn]) (decode phase)
    int de = kOK;
    if (enc == 0) {
      if (job.type == 0) {  // booleanPlainDecoder: one byte per 8 values
        if ((nn + 7) / 8 > vn) de = kEOF;
        else
          for (int64_t i = lane; i < nn; i += 64) out[i] = (val[i >> 3] >> (i & 7)) & 1;
      } else if (job.type == 3) {  // INT96 (type_int96.go:21-42)
        int64_t full = vn / 12, rem = vn % 12;
        if (nn > full + (rem > 0 ? 1 : 0)) de = kEOF;
        else {
          if (nn == full + 1 && rem > 0 && lane == 0) pg.flags |= 1;
          for (int64_t i = lane; i < nn * 12; i += 64) out[i] = (i < full * 12) ? val[i] : 0;
        }
      } else if (w > 0 && (w & 3) != 0) {  // FLBA of odd length: byte copy
        if (nn * w > vn) de = kEOF;
        else
          for (int64_t i = lane; i < nn * w; i += 64) out[i] = val[i];
      } else if (w > 0) {
        if (nn * w > vn) de = kEOF;
        else {
          int64_t nb = nn * w;
          // 16-byte destination chunks; source may be unaligned
          for (int64_t i = (int64_t)lane * 4; i < nb; i += 256) {
            if (i + 4 <= nb) {
              uint64_t x = load_u64_masked(val, readable, i, vn);
              *(uint32_t*)(out + i) = (uint32_t)x;
            } else {
              for (int64_t b = i; b < nb; b++) out[b] = val[b];
            }
          }
        }
      } else {
        de = kUNSUPPORTED;  // PLAIN byte arrays: not in this build yet
      }
    } else if (enc == 8) {
      int64_t err_at;
      const uint8_t* dict = job.dict_data;
      int64_t dcount = job.dict_data ? job.dict_count : 0;
      int64_t nil_key = (job.flags & 1) ? dcount - 1 : -1;
      if (w == 0) {
        de = kUNSUPPORTED;
      } else if (w == 4) {
        DictSink<4> sk{out, dict, dcount, nn, nil_key};
        de = hybrid_decode(val + 1, vn - 1, readable - 1, dict_w, nn, sh.hy, sk, &err_at);
        int64_t bad = wave_min(sk.bad);
        if (bad < nn && (de == kOK || bad < err_at)) de = kDICT_INDEX;
      } else if (w == 8) {
        DictSink<8> sk{out, dict, dcount, nn, nil_key};
        de = hybrid_decode(val + 1, vn - 1, readable - 1, dict_w, nn, sh.hy, sk, &err_at);
        int64_t bad = wave_min(sk.bad);
        if (bad < nn && (de == kOK || bad < err_at)) de = kDICT_INDEX;
      } else {
        DictSinkN sk{out, dict, dcount, nn, w, nil_key};
        de = hybrid_decode(val + 1, vn - 1, readable - 1, dict_w, nn, sh.hy, sk, &err_at);
        int64_t bad = wave_min(sk.bad);
        if (bad < nn && (de == kOK || bad < err_at)) de = kDICT_INDEX;
      }
    } else if (enc == 5) {
      de = dbp_decode(val, vn, readable, job.type == 2, nn, out, sh.dbp, 1);
    } else if (enc == 3 && job.type == 0) {  // booleanRLEDecoder: hybrid w=1 after a u32 length
      int64_t sz = rd_u32(val);
      int64_t take = min(sz, vn - 4);
      BoolSink sk{out};
      int64_t err_at;
      de = hybrid_decode(val + 4, take, readable - 4, 1, nn, sh.hy, sk, &err_at);
    } else {
      de = kUNSUPPORTED;
    }
    if (lane == 0 && de != kOK) pg.decode_status = de;
  }
}

// ============================================================================
// K5: chunk status in reference order (readPages errors first, then
// readPageData errors) — one thread per job.
// ============================================================================
__global__ void k_finalize(JobDev* jobs, int n_jobs, PageDev* pages) {
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_jobs) return;
  JobDev& job = jobs[j];
  if (job.status == kCAPACITY) return;
  int np = job.num_pages < job.page_cap ? job.num_pages : job.page_cap;
  int status = kOK, ep = -1;
  for (int i = 0; i < np; i++) {
    if (pages[job.page_base + i].read_status != kOK) {
      status = pages[job.page_base + i].read_status;
      ep = i;
      break;
    }
  }
  job.n_out_pages = ep >= 0 ? ep + 1 : np;
  if (status == kOK) {
    for (int i = 0; i < np; i++) {
      const PageDev& pg = pages[job.page_base + i];
      if ((pg.page_type == 0 || pg.page_type == 3) && pg.decode_status != kOK) {
        status = pg.decode_status;
        ep = i;
        break;
      }
    }
  }
  job.status = status;
  job.error_page = ep;
}

}  // namespace pqg
