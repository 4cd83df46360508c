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
// K1: page-header scan.
//
// readPages (chunk_reader.go:206-284) walks the chunk serially: parse a
// PageHeader at pos, then pos = payload + CompressedPageSize (or
// DataPageOffset after the dictionary page, :243-249).  A serial walk costs
// one dependent HBM round trip per page, so the GPU finds the pages
// speculatively instead:
//   K1a k_page_cands  every byte position p of every chunk is tested for the
//                     compact-protocol prefix of a PageHeader (field 1 `type`
//                     i32 with a 1-byte value, then field 2 i32: 15 xx 15);
//                     each hit is parsed by one lane and classified.
//   K1b k_tile_scan   per-chunk exclusive scan of the per-tile hit counts.
//   K1c k_cand_link   each candidate finds the candidate at its next-page
//                     position (its successor).
//   K1d k_page_chain  pages = the successor chain from position 0.  False
//                     candidates (payload bytes that happen to parse) are
//                     never on it.  Pages are written in chain order with the
//                     slot / scratch prefix sums.
//   K1e k_scan_pages  the serial walk, run only for chunks the speculative
//                     path cannot settle (a chain position with no candidate,
//                     a tile with more than kCandPerTile hits, deep thrift
//                     nesting): results are identical by construction, since
//                     both paths share classify_page.
// ============================================================================

// Read-phase classification of one parsed header (readPages :216-272 with
// dictPageReader.read page_dict.go:30-64, dataPageReaderV1.read
// page_v1.go:79-108, dataPageReaderV2.read page_v2.go:73-129).  `dict_seen`:
// an earlier page of the walk was a dictionary page.  Sets *next to the
// position of the following page and *comp to the scratch bytes (16-rounded)
// the page's decompressed block needs.
__device__ int classify_page(const JobDev& job, const PageHdr& h, int e, int64_t payload, bool dict_seen,
                             PageDev& pg, int64_t* next, int64_t* comp) {
  *comp = 0;
  *next = payload;
  pg.page_type = h.type;
  pg.encoding = h.encoding;
  pg.num_values = 0;
  pg.csize = h.csize;
  pg.usize = h.usize;
  pg.def_len = h.v2_def_len;
  pg.rep_len = h.v2_rep_len;
  pg.def_enc = h.def_enc;
  pg.rep_enc = h.rep_enc;
  if (e != kOK) return e;
  if (h.type == 2) {  // DICTIONARY_PAGE (page_dict.go:30-64, chunk_reader.go:221-251)
    pg.num_values = h.has_dict ? h.num_values : 0;
    if (dict_seen) e = kDICT_PAGE;
    else if (job.type == 0 || (job.type == 7 && job.type_length < 0)) e = kUNSUPPORTED;
    else if (!h.has_dict || h.num_values < 0) e = kPAGE_HEADER;
    else if (h.encoding != 0 && h.encoding != 2) e = kUNSUPPORTED;
    else if (h.csize < 0 || h.usize < 0) e = kPAGE_HEADER;
    else if (job.data_len - payload < (int64_t)h.csize) e = kSIZE;
    else if (job.codec == 0) { if (h.csize != h.usize) e = kSIZE; }
    else if (job.codec == 1) *comp = ((int64_t)h.usize + 15) & ~(int64_t)15;
    else e = kUNSUPPORTED;
    *next = payload + h.csize;
    if (e == kOK && job.has_dict_off) *next = job.data_page_offset;
    if (e != kOK) *comp = 0;
  } else if (h.type == 0) {  // DATA_PAGE (page_v1.go:57-108)
    pg.num_values = h.has_dph ? h.num_values : 0;
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
    if (e == kOK && job.codec == 1) *comp = ((int64_t)h.usize + 15) & ~(int64_t)15;
    *next = payload + h.csize;
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
    if (e == kOK && job.codec == 1) *comp = ((int64_t)us + 15) & ~(int64_t)15;
    *next = body + cs;
  } else {
    e = kUNSUPPORTED;  // "DATA_PAGE or DATA_PAGE_V2 type supported"
  }
  return e;
}

__device__ __forceinline__ void init_page(PageDev& pg, int j, int64_t pos, int64_t payload) {
  pg.header_offset = pos;
  pg.payload_offset = payload;
  pg.slot_offset = 0;
  pg.value_offset = 0;
  pg.scratch_offset = -1;
  pg.block = nullptr;
  pg.block_len = 0;
  pg.rep = pg.def = pg.val = nullptr;
  pg.rep_n = pg.def_n = pg.val_n = 0;
  pg.job = j;
  pg.read_status = kOK;
  pg.decode_status = kOK;
  pg.not_null = 0;
  pg.flags = 0;
  pg.dict_width = 0;
  pg.pad = 0;
}

__device__ __forceinline__ void init_job_results(JobDev& job) {
  job.num_pages = 0;
  job.dict_page = -1;
  job.scan_status = kOK;
  job.need_scratch = 0;
  job.num_slots = 0;
  job.dict_data = nullptr;
  job.dict_count = 0;
  job.dict_len = 0;
  job.dict_offs = nullptr;
  job.status = kOK;
  job.error_page = -1;
  job.flags = 0;
}

// ---- K1a ------------------------------------------------------------------
// Byte source of the per-lane candidate parse.  Reads stop at `limit`
// (kCandParseBytes past the candidate): a header that needs more is left to
// the serial walk (`hit`), so a garbage candidate cannot run away through the
// chunk (e.g. a thrift list header claiming 2^31 elements).
constexpr int64_t kCandParseBytes = 4096;
struct GlobalSrc {
  const uint8_t* p;
  int64_t n, limit;
  bool hit;
  __device__ int get(int64_t i) {
    if (i >= limit && i < n) {
      hit = true;
      return -1;
    }
    return (i >= 0 && i < n) ? (int)p[i] : -1;
  }
};

__device__ __forceinline__ bool has_byte_15(uint32_t x) {
  uint32_t y = x ^ 0x15151515u;
  return ((y - 0x01010101u) & ~y & 0x80808080u) != 0;
}

constexpr int kCandFrames = 4, kCandLast = 8;

__global__ void __launch_bounds__(256) k_page_cands(JobDev* jobs, int n_jobs, int* tile_count, int* tile_okc,
                                                    Cand* cands) {
  __shared__ int cnt;
  __shared__ int job_s;
  __shared__ Cand loc[kCandPerTile];
  __shared__ SkipFrame frames[256][kCandFrames];
  __shared__ int16_t lasts[256][kCandLast];
  const int tid = threadIdx.x;
  const int64_t tile = blockIdx.x;
  if (tid == 0) {
    cnt = 0;
    int lo = 0, hi = n_jobs - 1;  // last job with tile_base <= tile
    while (lo < hi) {
      int mid = (lo + hi + 1) >> 1;
      if (jobs[mid].tile_base <= tile) lo = mid; else hi = mid - 1;
    }
    job_s = lo;
  }
  __syncthreads();
  const int j = job_s;
  const JobDev& job = jobs[j];
  const int64_t lim = job.tcs < job.data_len ? job.tcs : job.data_len;
  const int64_t t0 = (tile - job.tile_base) * kScanTile;
  const int64_t t1 = t0 + kScanTile < lim ? t0 + kScanTile : lim;
  const uint8_t* base = job.data;
  const uintptr_t a0 = (uintptr_t)(base + t0) & ~(uintptr_t)15;
  for (int64_t off = (int64_t)tid * 16;; off += 256 * 16) {
    const uintptr_t a = a0 + off;
    const int64_t p0 = (int64_t)(a - (uintptr_t)base);
    if (p0 >= t1) break;
    // the 16-byte granule holds a position < t1 <= data_len, so it is mapped
    const uint4 v = *(const uint4*)a;
    if (!(has_byte_15(v.x) || has_byte_15(v.y) || has_byte_15(v.z) || has_byte_15(v.w))) continue;
    uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const int64_t p = p0 + k;
      if (((w4[k >> 2] >> (8 * (k & 3))) & 0xff) != 0x15 || p < t0 || p >= t1) continue;
      int b1 = k + 1 < 16 ? (int)((w4[(k + 1) >> 2] >> (8 * ((k + 1) & 3))) & 0xff)
                          : (p + 1 < job.data_len ? (int)base[p + 1] : -1);
      if (b1 != 0 && b1 != 2 && b1 != 4 && b1 != 6) continue;
      int b2 = k + 2 < 16 ? (int)((w4[(k + 2) >> 2] >> (8 * ((k + 2) & 3))) & 0xff)
                          : (p + 2 < job.data_len ? (int)base[p + 2] : -1);
      if (b2 != 0x15) continue;
      const int slot = atomicAdd(&cnt, 1);
      if (slot >= kCandPerTile) continue;  // tile overflow: the chunk takes the serial walk anyway
      Compact<GlobalSrc> c;
      c.src = GlobalSrc{base, job.data_len, p + kCandParseBytes, false};
      c.pos = p;
      c.frames = frames[tid];
      c.last = lasts[tid];
      c.nlast = 0;
      c.last_id = 0;
      c.bool_set = c.bool_val = false;
      c.fcap = kCandFrames;
      c.lcap = kCandLast;
      PageHdr h;
      int e = c.read_page_header(&h);
      PageDev pg;
      int64_t next, comp;
      e = classify_page(job, h, e, c.pos, false, pg, &next, &comp);
      if (c.overflow || c.src.hit) e = kCOMPLEX;
      Cand cd;
      cd.pos = p;
      cd.next = next;
      cd.payload = c.pos;
      cd.comp = comp;
      cd.type = pg.page_type;
      cd.encoding = pg.encoding;
      cd.num_values = pg.num_values;
      cd.csize = pg.csize;
      cd.usize = pg.usize;
      cd.def_len = pg.def_len;
      cd.rep_len = pg.rep_len;
      cd.def_enc = pg.def_enc;
      cd.rep_enc = pg.rep_enc;
      cd.status = e;
      cd.okrank = 0;
      cd.pad = 0;
      loc[slot] = cd;
    }
  }
  __syncthreads();
  const int n = cnt;
  if (tid == 0) {
    int ok = 0;
    for (int k = 0; k < n && k < kCandPerTile; k++) ok += loc[k].status == kOK;
    tile_count[tile] = n > kCandPerTile ? kCandPerTile + 1 : n;  // overflow: serial walk
    tile_okc[tile] = ok;
  }
  if (n <= kCandPerTile && tid < n) {  // rank sort by position (positions are distinct)
    const int64_t me = loc[tid].pos;
    int rank = 0, okr = 0;
    for (int k = 0; k < n; k++) {
      rank += loc[k].pos < me;
      okr += loc[k].pos < me && loc[k].status == kOK;
    }
    Cand cd = loc[tid];
    cd.okrank = okr;
    cands[tile * kCandPerTile + rank] = cd;
  }
}

// ---- K1b ------------------------------------------------------------------
// Per-chunk exclusive scans of the tile candidate counts (all, and ok-status).
__global__ void __launch_bounds__(1024) k_tile_scan(JobDev* jobs, const int* tile_count, const int* tile_okc,
                                                    int* tile_off, int* tile_okoff) {
  __shared__ int64_t part[17];
  __shared__ int ovf;
  JobDev& job = jobs[blockIdx.x];
  const int tid = threadIdx.x;
  if (tid == 0) ovf = 0;
  __syncthreads();
  const int nt = job.n_tiles;
  const int64_t tb = job.tile_base;
  // each thread sums a contiguous segment, one block scan, then writes
  const int seg = (nt + 1023) / 1024;
  const int s0 = tid * seg, s1 = min(nt, s0 + seg);
  int64_t sum = 0, oks = 0;
  bool bad = false;
  for (int t = s0; t < s1; t++) {
    int c = tile_count[tb + t];
    bad |= c > kCandPerTile;
    sum += c;
    oks += tile_okc[tb + t];
  }
  if (bad) ovf = 1;
  int64_t total, ok_total;
  int64_t ex = block_excl_scan<1024>(sum, &total, part);
  int64_t exo = block_excl_scan<1024>(oks, &ok_total, part);
  for (int t = s0; t < s1; t++) {
    tile_off[tb + t] = (int)ex;
    tile_okoff[tb + t] = (int)exo;
    ex += tile_count[tb + t];
    exo += tile_okc[tb + t];
  }
  if (tid == 0) {
    init_job_results(job);
    job.n_cands = (int32_t)min(total, (int64_t)INT32_MAX);
    job.n_ok = (int32_t)min(ok_total, (int64_t)INT32_MAX);
    job.scan_fallback = (ovf || total > INT32_MAX / 2) ? 1 : 0;
    job.brk = INT32_MAX;
    job.first_dict = INT32_MAX;
  }
}

// successor codes
constexpr int kSuccEnd = -1;      // next >= TotalCompressedSize: the walk ends
constexpr int kSuccTerm = -2;     // this page's read phase fails: the walk stops here
constexpr int kSuccMissing = -3;  // no candidate at the next position
constexpr int kSuccComplex = -4;  // candidate needs the serial parse

// ---- K1c ------------------------------------------------------------------
// One lane per candidate slot (kCandPerTile lanes per tile).  Candidates are
// numbered by position (index i) and, among those whose read phase succeeds,
// by ok-rank r.  A failing candidate can only END a walk, so in-header false
// hits (`15 00 15 06 ..` inside a DataPageHeader), which fail to classify,
// do not break the fast path: it checks that each ok candidate links to the
// ok candidate of the next rank.
__global__ void __launch_bounds__(256) k_cand_link(JobDev* jobs, int n_jobs, int64_t total_tiles,
                                                   const int* tile_count, const int* tile_off,
                                                   const int* tile_okoff, const Cand* cands, int* succ,
                                                   int* idx2slot, int* ok2slot) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t tile = g / kCandPerTile;
  const int s = (int)(g % kCandPerTile);
  if (tile >= total_tiles) return;
  const int cntv = tile_count[tile];
  if (s >= cntv || cntv > kCandPerTile) return;
  int lo = 0, hi = n_jobs - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].tile_base <= tile) lo = mid; else hi = mid - 1;
  }
  JobDev& job = jobs[lo];
  if (job.scan_fallback) return;
  const Cand& cd = cands[tile * kCandPerTile + s];
  const int64_t tb = job.tile_base;
  const int i = tile_off[tile] + s;
  const int slot = (int)((tile - tb) * kCandPerTile + s);
  idx2slot[tb * kCandPerTile + i] = slot;
  const bool ok = cd.status == kOK;
  const int r = tile_okoff[tile] + cd.okrank;
  if (ok) ok2slot[tb * kCandPerTile + r] = slot;
  int code;
  bool next_rank = false;  // successor is the ok candidate of rank r+1
  if (cd.status == kCOMPLEX) code = kSuccComplex;
  else if (!ok) code = kSuccTerm;
  else if (job.tcs - cd.next <= 0) code = kSuccEnd;
  else {
    code = kSuccMissing;
    const int64_t q = cd.next;
    const int64_t lim = job.tcs < job.data_len ? job.tcs : job.data_len;
    if (q >= 0 && q < lim) {
      const int64_t tq = tb + q / kScanTile;
      const int c2 = tile_count[tq];
      const Cand* tc = cands + tq * kCandPerTile;
      int lo2 = 0, hi2 = (c2 < kCandPerTile ? c2 : kCandPerTile) - 1;  // sorted by pos
      while (lo2 < hi2) {
        int mid = (lo2 + hi2) >> 1;
        if (tc[mid].pos < q) lo2 = mid + 1; else hi2 = mid;
      }
      if (hi2 >= 0 && tc[lo2].pos == q) {
        code = tile_off[tq] + lo2;
        next_rank = tc[lo2].status == kOK && tile_okoff[tq] + tc[lo2].okrank == r + 1;
      }
    }
  }
  succ[tile * kCandPerTile + s] = code;
  if (i == 0 && cd.pos != 0) atomicOr(&job.scan_fallback, 1);
  if (ok && !next_rank) atomicMin(&job.brk, r);
  if (ok && cd.type == 2) atomicMin(&job.first_dict, r);
}

// ---- K1d ------------------------------------------------------------------
// The page list = the successor chain from position 0.  Fast path: ok
// candidates of rank 0..brk, plus the failing page the last one links to.
// Otherwise a serial walk over the links (false ok candidates between pages)
// or, when a link has no candidate, the serial header walk (K1e).
__device__ __forceinline__ bool dict_again(const Cand& c, bool dict_seen) {
  // readPages :221-223: a second DICTIONARY_PAGE fails with "only one
  // dictionary" before its own checks (a header that did not parse fails first)
  return dict_seen && c.type == 2 && c.status != kTHRIFT;
}

__global__ void __launch_bounds__(1024) k_page_chain(JobDev* jobs, PageDev* pages, const Cand* cands,
                                                     const int* succ, const int* idx2slot, const int* ok2slot,
                                                     int* order) {
  __shared__ int64_t part[17];
  __shared__ int s_n, s_mode, s_cut, s_status, s_dict, s_extra, s_nok;
  const int j = blockIdx.x;
  JobDev& job = jobs[j];
  const int tid = threadIdx.x;
  const int64_t lim = job.tcs < job.data_len ? job.tcs : job.data_len;
  if (job.scan_fallback) return;
  if (job.tcs <= 0) return;  // the walk reads nothing: no pages
  if (lim <= 0 || job.n_cands == 0) {
    if (tid == 0) job.scan_fallback = 1;  // a page must start at 0: let the serial walk classify it
    return;
  }
  const int64_t cb = job.tile_base * kCandPerTile;  // the job's candidate-slot base
  const int* i2s = idx2slot + cb;
  const int* o2s = ok2slot + cb;
  const int b = job.brk;  // < n_ok when index 0 is ok
  const int d1 = job.first_dict;
  const Cand& head = cands[cb + i2s[0]];  // at position 0 (checked by k_cand_link)
  if (tid == 0) {
    s_cut = INT32_MAX;
    s_mode = 0;
    s_dict = -1;
    s_extra = -1;
    s_nok = 0;
  }
  __syncthreads();
  if (head.status == kOK && d1 < b) {  // second dictionary page within ranks (d1, b]
    for (int r = d1 + 1 + tid; r <= b; r += 1024)
      if (cands[cb + o2s[r]].type == 2) atomicMin(&s_cut, r);
  }
  __syncthreads();
  if (tid == 0) {
    int n = 0, mode = 0;  // mode 0: ok prefix (+ extra), 1: walked (order[]), 2: fallback
    if (head.status == kCOMPLEX) {
      mode = 2;
    } else if (head.status != kOK) {  // the first page fails
      n = 1;
      s_extra = i2s[0];
    } else {
      if (d1 <= b) s_dict = d1;
      if (s_cut != INT32_MAX) {
        n = s_cut + 1;
        s_nok = n;
      } else {
        const int code = succ[cb + o2s[b]];
        s_nok = b + 1;
        n = b + 1;
        if (code == kSuccMissing || code == kSuccComplex) {
          mode = 2;
        } else if (code >= 0) {
          const int ts = i2s[code];
          const Cand& t = cands[cb + ts];
          if (t.status == kCOMPLEX) {
            mode = 2;
          } else if (t.status != kOK) {  // the walk ends on this failing page
            s_extra = ts;
            if (dict_again(t, d1 <= b)) s_cut = n;
            n++;
          } else {
            // false ok candidates between pages: walk the links serially
            int* ord = order + job.page_base;
            for (int r = 0; r <= b && r < job.page_cap; r++) ord[r] = o2s[r];
            bool dict_seen = d1 <= b;
            int k = b + 1, cur = code;
            mode = 1;
            for (;;) {
              if (k >= job.page_cap) { mode = 2; break; }
              const int sl = i2s[cur];
              const Cand& cd = cands[cb + sl];
              if (cd.status == kCOMPLEX) { mode = 2; break; }
              ord[k++] = sl;
              if (dict_again(cd, dict_seen)) { s_cut = k - 1; break; }
              if (cd.type == 2 && cd.status == kOK) {
                dict_seen = true;
                s_dict = k - 1;
              }
              const int c2 = succ[cb + sl];
              if (c2 == kSuccEnd || c2 == kSuccTerm) break;
              if (c2 < 0) { mode = 2; break; }
              cur = c2;
            }
            n = k;
          }
        }
      }
    }
    if (mode == 2) job.scan_fallback = 1;
    s_n = n;
    s_mode = mode;
    s_status = kOK;
  }
  __syncthreads();
  if (s_mode == 2) return;
  const int n = s_n, mode = s_mode, cut = s_cut, nok = s_nok, extra = s_extra;
  const int nw = n < job.page_cap ? n : job.page_cap;
  int64_t slot_carry = 0, scratch_carry = 0;
  for (int b0 = 0; b0 < n; b0 += 1024) {
    const int k = b0 + tid;
    int64_t nv = 0, cp = 0;
    int st = kOK;
    const Cand* cd = nullptr;
    if (k < n) {
      const int sl = mode == 1 ? order[job.page_base + k] : (k < nok ? o2s[k] : extra);
      cd = &cands[cb + sl];
      st = (k == cut) ? kDICT_PAGE : cd->status;
      cp = (k == cut) ? 0 : cd->comp;
      if ((cd->type == 0 || cd->type == 3) && st == kOK) nv = cd->num_values;
      if (st != kOK) s_status = st;  // only the last page can fail
    }
    int64_t tot_nv, tot_cp;
    const int64_t ex_nv = block_excl_scan<1024>(nv, &tot_nv, part);
    const int64_t ex_cp = block_excl_scan<1024>(cp, &tot_cp, part);
    if (k < nw) {
      PageDev pg;
      init_page(pg, j, cd->pos, cd->payload);
      pg.page_type = cd->type;
      pg.encoding = cd->encoding;
      pg.num_values = cd->num_values;
      pg.csize = cd->csize;
      pg.usize = cd->usize;
      pg.def_len = cd->def_len;
      pg.rep_len = cd->rep_len;
      pg.def_enc = cd->def_enc;
      pg.rep_enc = cd->rep_enc;
      pg.read_status = st;
      pg.slot_offset = slot_carry + ex_nv;
      if (cp > 0) pg.scratch_offset = scratch_carry + ex_cp;
      pages[job.page_base + k] = pg;
    }
    slot_carry += tot_nv;
    scratch_carry += tot_cp;
  }
  __syncthreads();
  if (tid == 0) {
    job.num_pages = n;
    job.dict_page = s_dict;
    job.scan_status = s_status;
    job.need_scratch = scratch_carry;
    job.num_slots = slot_carry;
    if (n > job.page_cap || slot_carry > job.slot_cap || scratch_carry > job.scratch_cap) job.status = kCAPACITY;
  }
}

// ---- K1e: the serial walk (fallback) — one wave per chunk ------------------
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
  if (!job.scan_fallback) return;
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
    init_page(pg, j, pos, c.pos);
    pg.slot_offset = slots;
    int64_t next, comp;
    e = classify_page(job, h, e, c.pos, dict_seen, pg, &next, &comp);
    if (comp > 0) {
      pg.scratch_offset = scratch;
      scratch += comp;
    }
    pg.read_status = e;
    if (np < job.page_cap && lane == 0) pages[job.page_base + np] = pg;
    if (h.type == 0 || h.type == 3) slots += (e == kOK) ? pg.num_values : 0;
    if (e == kOK && h.type == 2) {
      dict_seen = true;
      dict_page = np;
    }
    np++;
    if (e != kOK) {
      status = e;
      break;
    }
    pos = next;
  }
  if (lane == 0) {
    init_job_results(job);
    job.num_pages = np;
    job.dict_page = dict_page;
    job.scan_status = status;
    job.need_scratch = scratch;
    job.num_slots = slots;
    if (np > job.page_cap || slots > job.slot_cap || scratch > job.scratch_cap) job.status = kCAPACITY;
  }
}

// ============================================================================
// K1f: compact list of page indices over all jobs.
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
// readPageData errors) — one 256-lane block per job, min-reductions over pages.
// ============================================================================
__global__ void __launch_bounds__(256) k_finalize(JobDev* jobs, int n_jobs, PageDev* pages) {
  __shared__ int s_read, s_dec;
  JobDev& job = jobs[blockIdx.x];
  if (job.status == kCAPACITY) return;
  const int np = job.num_pages < job.page_cap ? job.num_pages : job.page_cap;
  if (threadIdx.x == 0) {
    s_read = INT32_MAX;
    s_dec = INT32_MAX;
  }
  __syncthreads();
  const PageDev* pg = pages + job.page_base;
  int r = INT32_MAX, d = INT32_MAX;
  for (int i = threadIdx.x; i < np; i += 256) {
    if (pg[i].read_status != kOK && i < r) r = i;
    if ((pg[i].page_type == 0 || pg[i].page_type == 3) && pg[i].decode_status != kOK && i < d) d = i;
  }
  if (r != INT32_MAX) atomicMin(&s_read, r);
  if (d != INT32_MAX) atomicMin(&s_dec, d);
  __syncthreads();
  if (threadIdx.x != 0) return;
  int status = kOK, ep = -1;
  if (s_read != INT32_MAX) {
    ep = s_read;
    status = pg[ep].read_status;
  }
  job.n_out_pages = ep >= 0 ? ep + 1 : np;
  if (status == kOK && s_dec != INT32_MAX) {
    ep = s_dec;
    status = pg[ep].decode_status;
  }
  job.status = status;
  job.error_page = ep;
}

}  // namespace pqg
