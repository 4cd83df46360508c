// pqg_scan.hip — K1: page-header scan of every chunk (readPages,
// chunk_reader.go:206-284) and the compact page list.
#include <hip/hip_runtime.h>

#include "pqg_common.h"
#include "pqg_device.h"
#include "pqg_thrift.h"

namespace pqg {

// Byte source over the LDS window, for the thrift reader of the serial walk.
struct WinSrc {
  Window w;  // by value: the parser state stays in registers
  __device__ __forceinline__ int get(int64_t i) { return w.get(i); }
};


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
__device__ __forceinline__ int classify_page(const JobDev& job, const PageHdr& h, int e, int64_t payload, bool dict_seen,
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
    else if (job.codec == kCodecSnappy || job.codec == kCodecGzip) *comp = ((int64_t)h.usize + 15) & ~(int64_t)15;
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
    else if (job.codec != 0 && job.codec != kCodecSnappy && job.codec != kCodecGzip) e = kUNSUPPORTED;
    else if (job.codec == 0 && !values_supported(job.type, job.type_length, enc)) e = kUNSUPPORTED;
    if (e == kOK && job.codec != 0) *comp = ((int64_t)h.usize + 15) & ~(int64_t)15;
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
    else if (job.codec != 0 && job.codec != kCodecSnappy && job.codec != kCodecGzip) e = kUNSUPPORTED;
    if (e == kOK && job.codec != 0) *comp = ((int64_t)us + 15) & ~(int64_t)15;
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
  pg.vmode = -1;
  pg.run_off = pg.blk_off = 0;
  pg.chars = 0;
  pg.char_offset = 0;
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
  job.need_doffs = 0;
  job.status = kOK;
  job.error_page = -1;
  job.flags = 0;
  job.run_used = 0;
  job.blk_used = 0;
}

// ---- K1a ------------------------------------------------------------------
// Byte source of the per-lane candidate parse: the candidate's first bytes,
// prefetched into the lane's LDS window.  Reads stop at `limit` (the window's
// end, at most kCandParseBytes past the candidate): a header that needs more
// is left to the serial walk (`hit`), so a garbage candidate cannot run away
// through the chunk (e.g. a thrift list header claiming 2^31 elements).
// Bytes past the chunk read as -1 (EOF) without `hit`.
constexpr int64_t kCandParseBytes = 1024;
struct CandSrc {
  const PQG_L uint8_t* win;  // bytes [wlo, limit) of the chunk
  int64_t wlo, limit, n;
  bool hit;
  __device__ __forceinline__ int get(int64_t i) {
    if (i >= limit) {
      hit |= i < n;
      return -1;
    }
    return win[i - wlo];  // i >= wlo: the parse never reads before its candidate
  }
};

__device__ __forceinline__ bool has_byte_15(uint32_t x) {
  uint32_t y = x ^ 0x15151515u;
  return ((y - 0x01010101u) & ~y & 0x80808080u) != 0;
}

constexpr int kCandFrames = 4, kCandLast = 8;
// Loop steps of one candidate parse (fields + skipped container elements):
// the headers of parquet writers take at most ~25 (PageHeader, its page
// header struct and a Statistics struct); garbage that runs longer is
// kCOMPLEX (the serial walk reads it if a page link ever lands on it).  A
// lane's steps set its wave's time: without the bound one garbage candidate
// of ~80 one-byte fields held its wave ~0.2 ms.
constexpr int kCandSteps = 40;

// One lane parses and classifies the candidate at position p (kept out of
// line: the scan loop around it must stay small).
// The candidate's first bytes are prefetched into the lane's LDS window with
// independent 16-byte loads, and the parse is confined to them: a header that
// does not end inside the window is kCOMPLEX (its chunk takes the serial walk
// only if a page link lands on it).  Without the bound, the slowest candidate
// — garbage that passes the pre-check and reads on through the chunk one
// dependent granule load at a time — set the kernel's time.
constexpr int kCandWin = 10;  // granules: >= 144 bytes from any start
__device__ __forceinline__ void parse_candidate(const JobDev& job, int64_t p, SkipFrame* frames, int16_t* lasts,
                                             PQG_L uint8_t* win, Cand* out) {
  Compact<CandSrc> c;
  {
    const uintptr_t a0 = (uintptr_t)(job.data + p) & ~(uintptr_t)15;
    const int64_t lo = p - (int64_t)((uintptr_t)(job.data + p) - a0);  // chunk offset of the first granule
    uint4 g[kCandWin];
    // a granule holding a byte < n is mapped; the others read the first one
    // and are zeroed after every load is issued (a load under a branch is
    // waited for inside it)
#pragma unroll
    for (int k = 0; k < kCandWin; k++) g[k] = ldg16(lo + 16 * k < job.data_len ? a0 + 16 * k : a0);
#pragma unroll
    for (int k = 0; k < kCandWin; k++) sts16(win + 16 * k, lo + 16 * k < job.data_len ? g[k] : make_uint4(0, 0, 0, 0));
    const int64_t whi = lo + 16 * kCandWin < job.data_len ? lo + 16 * kCandWin : job.data_len;
    const int64_t lim = p + kCandParseBytes < whi ? p + kCandParseBytes : whi;
    c.src = CandSrc{win, lo, lim, job.data_len, false};
  }
  // Structural pre-check: every thrift writer of PageHeader emits fields 1, 2,
  // 3 in id order with short-form i32 headers (15 t 15 <varint> 15).  A
  // candidate without that shape is not parsed: it is marked kCOMPLEX, which
  // sends the chunk to the serial walk only if a page link ever lands on it.
  {
    int64_t q = p + 3;
    int b = 0x80;
    for (int k = 0; k < 5 && (b & 0x80); k++) b = c.src.get(q++);
    if (b < 0 || (b & 0x80) || c.src.get(q) != 0x15) {
      Cand cd;
      cd.pos = p;
      cd.next = p;
      cd.payload = p;
      cd.comp = 0;
      cd.type = cd.encoding = cd.num_values = cd.csize = cd.usize = 0;
      cd.def_len = cd.rep_len = cd.def_enc = cd.rep_enc = 0;
      cd.status = kCOMPLEX;
      *out = cd;
      return;
    }
  }
  c.pos = p;
  c.frames = frames;
  c.last = lasts;
  c.nlast = 0;
  c.last_id = 0;
  c.bool_set = c.bool_val = false;
  c.fcap = kCandFrames;
  c.lcap = kCandLast;
  c.budget = kCandSteps;
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
  *out = cd;
}

// cand_total: kQShards counters kQStride ints apart; tile t appends to shard
// t & 7, whose list region starts at (t & 7) * region (a single list head
// would take one contended device-scope atomic per tile).
// tile -> job map (one block per job): the scan kernels look a tile's job up
// with one load instead of a binary search over the job table.
__global__ void __launch_bounds__(256) k_tile_jobs(const JobDev* jobs, int* tile_job) {
  const JobDev& job = jobs[blockIdx.x];
  for (int64_t t = threadIdx.x; t < job.n_tiles; t += 256) tile_job[job.tile_base + t] = (int)blockIdx.x;
}

__global__ void __launch_bounds__(256) k_page_cands(JobDev* jobs, const int* tile_job, int* tile_count, int* tile_okc,
                                                    int64_t* cand_pos, int* cand_list, int* cand_total, int region) {
  __shared__ int cnt;
  __shared__ int job_s;
  __shared__ int64_t loc[kCandPerTile];
  const int tid = threadIdx.x;
  const int64_t tile = blockIdx.x;
  if (tid == 0) {
    cnt = 0;
    job_s = tile_job[tile];
  }
  __syncthreads();
  const JobDev& job = jobs[job_s];
  if (job.scan_fallback == 2) {  // walked before the scan: no candidates
    if (tid == 0) {
      tile_count[tile] = 0;
      tile_okc[tile] = 0;
    }
    return;
  }
  const int64_t lim = job.tcs < job.data_len ? job.tcs : job.data_len;
  const int64_t t0 = (tile - job.tile_base) * kScanTile;
  const int64_t t1 = t0 + kScanTile < lim ? t0 + kScanTile : lim;
  const gcu8 base = gconst(job.data);
  const int64_t data_len = job.data_len;
  const uintptr_t a0 = (uintptr_t)(base + t0) & ~(uintptr_t)15;
  // the tile's granules (<= 5 per thread: the tile start is aligned down) are
  // all loaded before any is examined, so each thread keeps 80 bytes in flight
  constexpr int kG = kScanTile / (256 * 16) + 1;
  uint4 vv[kG];
#pragma unroll
  for (int it = 0; it < kG; it++) {
    const uintptr_t a = a0 + (int64_t)tid * 16 + (int64_t)it * 256 * 16;
    const int64_t p0 = (int64_t)(a - (uintptr_t)base);
    // a granule holding a position < t1 <= data_len is mapped; the others
    // re-read the tile's first one (unconditional: a load under a branch is
    // waited for inside it) and are never examined
    vv[it] = ldg16(p0 < t1 ? a : a0);
  }
#pragma unroll
  for (int it = 0; it < kG; it++) {
    const uintptr_t a = a0 + (int64_t)tid * 16 + (int64_t)it * 256 * 16;
    const int64_t p0 = (int64_t)(a - (uintptr_t)base);
    if (p0 >= t1) break;
    const uint4 v = vv[it];
    if (!(has_byte_15(v.x) || has_byte_15(v.y) || has_byte_15(v.z) || has_byte_15(v.w))) continue;
    // bytes 16, 17 (lookahead of the last two positions), read only when
    // byte 14 or 15 is 0x15; 0xff (no match) past the end of the buffer
    uint32_t nx = 0xffffu;
    if (((v.w >> 16) & 0xff) == 0x15 || (v.w >> 24) == 0x15) {
      const int64_t q = p0 + 16;
      nx = (q < data_len ? (uint32_t)base[q] : 0xffu) | (q + 1 < data_len ? (uint32_t)base[q + 1] : 0xffu) << 8;
    }
    const uint32_t w5[5] = {v.x, v.y, v.z, v.w, nx};
    uint32_t mask = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint32_t c0 = (w5[k >> 2] >> (8 * (k & 3))) & 0xff;
      const uint32_t c1 = (w5[(k + 1) >> 2] >> (8 * ((k + 1) & 3))) & 0xff;
      const uint32_t c2 = (w5[(k + 2) >> 2] >> (8 * ((k + 2) & 3))) & 0xff;
      mask |= (uint32_t)(c0 == 0x15 && (c1 & 0xf9) == 0 && c2 == 0x15) << k;
    }
    // positions outside [t0, t1) belong to the neighbouring tiles
    while (mask) {
      const int k = __builtin_ctz(mask);
      mask &= mask - 1;
      const int64_t p = p0 + k;
      if (p < t0 || p >= t1) continue;
      const int slot = atomicAdd(&cnt, 1);
      if (slot < kCandPerTile) loc[slot] = p;  // beyond: overflow, the chunk takes the serial walk
    }
  }
  __syncthreads();
  const int n = cnt;
  if (tid == 0) {
    tile_count[tile] = n > kCandPerTile ? kCandPerTile + 1 : n;
    tile_okc[tile] = 0;  // counted by k_cand_parse
  }
  __shared__ int list_base;
  if (tid == 0 && n > 0 && n <= kCandPerTile) {
    const int sh = (int)(tile & (kQShards - 1));
    list_base = sh * region + atomicAdd(cand_total + sh * kQStride, n);
  }
  __syncthreads();
  if (n <= kCandPerTile && tid < n) {  // rank sort by position (positions are distinct)
    const int64_t me = loc[tid];
    int rank = 0;
    for (int k = 0; k < n; k++) rank += loc[k] < me;
    cand_pos[tile * kCandPerTile + rank] = me;
    cand_list[list_base + tid] = (int)(tile * kCandPerTile + rank);  // slot to parse
  }
}

// ---- K1a' ------------------------------------------------------------------
// One lane per candidate slot: parse + classify (kept apart from the byte scan
// so that the scan has no scratch and runs at full occupancy).
__global__ void __launch_bounds__(256) k_cand_parse(JobDev* jobs, const int* tile_job, const int* cand_list,
                                                    const int* cand_total, int region, int* tile_okc,
                                                    const int64_t* cand_pos, Cand* cands) {
  __shared__ SkipFrame frames[256][kCandFrames];
  __shared__ int16_t lasts[256][kCandLast];
  __shared__ __attribute__((aligned(16))) uint8_t wins[256][16 * kCandWin];
  int pre[kQShards + 1];  // the shards' list lengths, prefix-summed (uniform)
  pre[0] = 0;
#pragma unroll
  for (int k = 0; k < kQShards; k++) pre[k + 1] = pre[k] + cand_total[k * kQStride];
  const int nc = pre[kQShards];
  for (int i = blockIdx.x * 256 + threadIdx.x; i < nc; i += gridDim.x * 256) {
    int sh = 0;
#pragma unroll
    for (int k = 1; k < kQShards; k++) sh += i >= pre[k];
    const int slot = cand_list[sh * region + (i - pre[sh])];
    const int64_t tile = slot / kCandPerTile;
    const int lo = tile_job[tile];
    Cand* out = &cands[slot];
    parse_candidate(jobs[lo], cand_pos[slot], frames[threadIdx.x], lasts[threadIdx.x], lds_ptr(wins[threadIdx.x]), out);
    if (out->status == kOK) atomicAdd(&tile_okc[tile], 1);
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
  if (job.scan_fallback == 2) return;  // walked before the scan (k_scan_pages prewalk)
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
__global__ void __launch_bounds__(256) k_cand_link(JobDev* jobs, const int* tile_job, int64_t total_tiles,
                                                   const int* tile_count, const int* tile_off,
                                                   const int* tile_okoff, const Cand* cands, int* succ,
                                                   int* idx2slot, int* ok2slot) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t tile = g / kCandPerTile;
  const int s = (int)(g % kCandPerTile);
  if (tile >= total_tiles) return;
  const int cntv = tile_count[tile];
  if (s >= cntv || cntv > kCandPerTile) return;
  JobDev& job = jobs[tile_job[tile]];
  if (job.scan_fallback) return;
  const Cand& cd = cands[tile * kCandPerTile + s];
  const int64_t tb = job.tile_base;
  const int i = tile_off[tile] + s;
  const int slot = (int)((tile - tb) * kCandPerTile + s);
  idx2slot[tb * kCandPerTile + i] = slot;
  const bool ok = cd.status == kOK;
  int okr = 0;  // ok candidates before this one in the tile
  for (int k = 0; k < s; k++) okr += cands[tile * kCandPerTile + k].status == kOK;
  const int r = tile_okoff[tile] + okr;
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
        if (tc[lo2].status == kOK) {
          int okt = 0;
          for (int k = 0; k < lo2; k++) okt += tc[k].status == kOK;
          next_rank = tile_okoff[tq] + okt == r + 1;
        }
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
  // Rounds of 1024 pages, software-pipelined: the next round's candidate
  // records are loaded before this round's page records are stored (a load
  // issued after the stores would wait for them: vmcnt counts both in order).
  // Loads are unconditional (the page index clamped to n - 1).
  auto fetch = [&](int k, Cand& c) {
    const int kk = k < n ? k : n - 1;
    const int sl = mode == 1 ? order[job.page_base + kk] : (kk < nok ? o2s[kk] : extra);
    c = cands[cb + sl];
  };
  Cand cur;
  if (n > 0) fetch(tid, cur);
  for (int b0 = 0; b0 < n; b0 += 1024) {
    const int k = b0 + tid;
    int64_t nv = 0, cp = 0;
    int st = kOK;
    if (k < n) {
      st = (k == cut) ? kDICT_PAGE : cur.status;
      cp = (k == cut) ? 0 : cur.comp;
      if ((cur.type == 0 || cur.type == 3) && st == kOK) nv = cur.num_values;
      if (st != kOK) s_status = st;  // only the last page can fail
    }
    int64_t tot_nv, tot_cp;
    const int64_t ex_nv = block_excl_scan<1024>(nv, &tot_nv, part);
    const int64_t ex_cp = block_excl_scan<1024>(cp, &tot_cp, part);
    Cand nxt;
    if (b0 + 1024 < n) fetch(b0 + 1024 + tid, nxt);
    if (k < nw) {
      PageDev pg;
      init_page(pg, j, cur.pos, cur.payload);
      pg.page_type = cur.type;
      pg.encoding = cur.encoding;
      pg.num_values = cur.num_values;
      pg.csize = cur.csize;
      pg.usize = cur.usize;
      pg.def_len = cur.def_len;
      pg.rep_len = cur.rep_len;
      pg.def_enc = cur.def_enc;
      pg.rep_enc = cur.rep_enc;
      pg.read_status = st;
      pg.slot_offset = slot_carry + ex_nv;
      if (cp > 0) pg.scratch_offset = scratch_carry + ex_cp;
      pages[job.page_base + k] = pg;
    }
    slot_carry += tot_nv;
    scratch_carry += tot_cp;
    cur = nxt;
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
  // the stride walk's per-lane candidate parses (parse_candidate)
  __attribute__((aligned(16))) uint8_t cw[64][16 * kCandWin];
  SkipFrame cf[64][kCandFrames];
  int16_t cl[64][kCandLast];
};

// Chunks of equal small pages (fixed-width PLAIN columns: parquet-go's writer
// cuts pages by row count, so every page but the last has one length and the
// same header bytes): after the serial prewalk reached the first small data
// page at `spos` with length `slen`, that page's header is parsed
// (parse_candidate) and every later predicted page spos + k * slen is checked
// against it byte for byte, 64 pages per round, one per lane, with one round
// of loads: identical header bytes read identically (the same fields, shifted
// positions), so the page's record is page 0's with its offsets.  The chunk's
// last page (fewer rows) is parsed and must end at or past the chunk's end.
// Any other difference returns false: the candidate scan then settles the
// chunk and overwrites every page record written here.  The pages before
// spos (a dictionary page, big pages) are the serial walk's.
__device__ bool stride_walk(JobDev& job, int j, PageDev* pages, int64_t spos, int64_t slen, int np0, int64_t slots0,
                            int64_t scratch0, ScanShared& sh) {
  const int lane = lane_id();
  const int64_t tcs = job.tcs;
  if (slen <= 0 || tcs - spos <= 0) return false;
  // page 0 of the stride (every lane parses it: wave-uniform result)
  Cand c0;
  parse_candidate(job, spos, sh.cf[lane], sh.cl[lane], lds_ptr(sh.cw[lane]), &c0);
  const int64_t hl = c0.payload - spos;  // header bytes
  if (c0.status != kOK || !(c0.type == 0 || c0.type == 3) || c0.next - spos != slen || hl <= 0 || hl > 64)
    return false;
  // page 0's header bytes: LDS bytes [0, hl) of sh.win (16 granules max)
  const gcu8 base = gconst(job.data);
  constexpr int kHG = 5;  // granules holding a <= 64-byte header from any alignment
  {
    const uintptr_t a0 = (uintptr_t)(base + spos) & ~(uintptr_t)15;
    const int64_t at = (int64_t)(a0 + 16 * (uintptr_t)lane - (uintptr_t)base);
    const uint4 g = ldg16(lane < kHG && at < job.data_len ? a0 + 16 * lane : a0);  // granules holding a chunk byte
    if (lane < kHG) sts16(lds_ptr(sh.win) + 16 * lane, g);
  }
  __builtin_amdgcn_wave_barrier();
  const uint32_t off0 = (uint32_t)((uintptr_t)(base + spos) & 15);
  const int64_t npages = (tcs - spos + slen - 1) / slen;
  int64_t slots = slots0, scratch = scratch0;
  const int64_t nv0 = c0.num_values, cp0 = c0.comp;
  for (int64_t k0 = 0; k0 < npages; k0 += 64) {
    const int64_t k = k0 + lane;
    const bool live = k < npages;
    const int64_t q = spos + (live ? k : 0) * slen;
    // this lane's page header bytes: kHG granules from q's aligned address
    const uintptr_t a = (uintptr_t)(base + q) & ~(uintptr_t)15;
    uint4 g[kHG];
#pragma unroll
    for (int t = 0; t < kHG; t++) {
      const int64_t at = (int64_t)(a + 16 * t - (uintptr_t)base);
      g[t] = ldg16(at < job.data_len ? a + 16 * t : a);
    }
    PQG_L uint32_t* W = (PQG_L uint32_t*)lds_ptr(sh.cw[lane]);
#pragma unroll
    for (int t = 0; t < kHG; t++) sts16((PQG_L uint8_t*)W + 16 * t, g[t]);
    __builtin_amdgcn_wave_barrier();
    const uint32_t offk = (uint32_t)((uintptr_t)(base + q) & 15);
    const PQG_L uint32_t* W0 = (const PQG_L uint32_t*)lds_ptr(sh.win);
    bool same = live;
    for (int i = 0; i < (int)hl; i += 4) {
      const uint32_t ok_ = offk + (uint32_t)i, o0 = off0 + (uint32_t)i;
      const uint32_t x = __builtin_amdgcn_alignbit(W[(ok_ >> 2) + 1], W[ok_ >> 2], (ok_ & 3) * 8);
      const uint32_t y = __builtin_amdgcn_alignbit(W0[(o0 >> 2) + 1], W0[o0 >> 2], (o0 & 3) * 8);
      const int r = (int)hl - i;
      const uint32_t m = r >= 4 ? 0xffffffffu : ((1u << (8 * r)) - 1);
      same &= ((x ^ y) & m) == 0;
    }
    // the header past the chunk's end cannot be page 0's
    same &= q + hl <= tcs;
    __builtin_amdgcn_wave_barrier();
    const bool lastp = live && k == npages - 1;
    Cand ck = c0;
    bool ok = same;
    if (live && !same) {
      if (lastp) {  // the short last page: parsed, and it must end the chunk
        parse_candidate(job, q, sh.cf[lane], sh.cl[lane], lds_ptr(sh.cw[lane]), &ck);
        ok = ck.status == kOK && (ck.type == 0 || ck.type == 3) && ck.next >= tcs;
      }
    } else if (same) {  // page 0's fields at this page's position
      ck.pos = q;
      ck.payload = c0.payload + (q - spos);
      ck.next = c0.next + (q - spos);
      // classify_page's size check at this position (an understated buffer),
      // and a full-length last page ends the chunk exactly
      ok = ck.next <= job.data_len && (!lastp || ck.next >= tcs);
    }
    const uint64_t lb = __ballot(live), okb = __ballot(live && ok);
    if (okb != lb) return false;
    const int nl = __popcll(lb);
    const bool mine = live;
    const int64_t nv = mine ? ck.num_values : 0, cp = mine ? ck.comp : 0;
    const int64_t inv = (int64_t)wave_incl_scan_u64((uint64_t)nv), icp = (int64_t)wave_incl_scan_u64((uint64_t)cp);
    if (mine && np0 + k < job.page_cap) {
      PageDev pg;
      init_page(pg, j, q, ck.payload);
      pg.page_type = ck.type;
      pg.encoding = ck.encoding;
      pg.num_values = ck.num_values;
      pg.csize = ck.csize;
      pg.usize = ck.usize;
      pg.def_len = ck.def_len;
      pg.rep_len = ck.rep_len;
      pg.def_enc = ck.def_enc;
      pg.rep_enc = ck.rep_enc;
      pg.read_status = kOK;
      pg.slot_offset = slots + inv - nv;
      if (cp > 0) pg.scratch_offset = scratch + icp - cp;
      pages[job.page_base + np0 + k] = pg;
    }
    auto lane64 = [](int64_t v, int l) {
      return (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l) |
                       (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l) << 32);
    };
    slots += lane64(inv, nl - 1);
    scratch += lane64(icp, nl - 1);
  }
  (void)nv0;
  (void)cp0;
  if (lane == 0) {
    const int np = np0 + (int)npages;
    init_job_results(job);
    job.scan_fallback = 2;
    job.num_pages = np;
    job.scan_status = kOK;
    job.need_scratch = scratch;
    job.num_slots = slots;
    if (np > job.page_cap || slots > job.slot_cap || scratch > job.scratch_cap) job.status = kCAPACITY;
  }
  return true;
}

// prewalk > 0: before the candidate scan, chunks of at most `prewalk` big
// pages (each data page >= 1/8 of the chunk: parquet-go's writer puts a whole
// chunk in one page) are walked here, and their bytes are not scanned
// (scan_fallback = 2 tells K1a-K1d to skip the job).  A headers-only walk
// decides; only a walk that reaches the chunk's end (or its first failing
// page) within the limit is redone with its page records.  prewalk == 0: the
// jobs the speculative path could not settle (scan_fallback == 1).
__global__ void __launch_bounds__(64) k_scan_pages(JobDev* jobs, PageDev* pages, int n_jobs, int prewalk, int stride) {
  __shared__ __attribute__((aligned(16))) ScanShared sh;
  int j = blockIdx.x;
  if (j >= n_jobs) return;
  JobDev& job = jobs[j];
  const int64_t tcs = job.tcs;
  if (prewalk > 0) {
    if (job.scan_fallback || tcs <= 0 || job.no_prewalk) return;
    Window win{gconst(job.data), job.data_len, kFarAway, lds_ptr(sh.win)};
    int64_t pos = 0;
    bool dict_seen = false, done = false;
    int64_t spos = -1, slen = 0;  // the first small data page (a stride walk's start)
    int snp = 0;
    for (int np = 0;; np++) {
      if (tcs - pos <= 0) {
        done = true;
        break;
      }
      if (np == prewalk) break;
      Compact<WinSrc> c;
      c.src.w = win;
      c.pos = pos;
      c.frames = sh.frames;
      c.last = sh.last;
      c.nlast = 0;
      c.last_id = 0;
      c.bool_set = false;
      c.bool_val = false;
      PageHdr h;
      int e = c.read_page_header(&h);
      win = c.src.w;
      PageDev pg;
      init_page(pg, j, pos, c.pos);
      int64_t next, comp;
      e = classify_page(job, h, e, c.pos, dict_seen, pg, &next, &comp);
      if (e != kOK) {
        done = true;
        break;
      }
      if (h.type != 2 && next - pos < tcs / 8) {  // small pages: many of them, a stride walk or the candidate scan
        spos = pos;
        slen = next - pos;
        snp = np;
        break;
      }
      if (h.type == 2) dict_seen = true;
      pos = next;
    }
    if (!done) {
      if (spos < 0 || !stride) return;
      // the pages before spos (serially, with their records), then the stride
      Window w2{gconst(job.data), job.data_len, kFarAway, lds_ptr(sh.win)};
      int64_t p2 = 0, slots = 0, scratch = 0;
      int dict_page = -1;
      bool ds2 = false;
      for (int k = 0; k < snp; k++) {
        Compact<WinSrc> c;
        c.src.w = w2;
        c.pos = p2;
        c.frames = sh.frames;
        c.last = sh.last;
        c.nlast = 0;
        c.last_id = 0;
        c.bool_set = false;
        c.bool_val = false;
        PageHdr h;
        int e = c.read_page_header(&h);
        w2 = c.src.w;
        PageDev pg;
        init_page(pg, j, p2, c.pos);
        pg.slot_offset = slots;
        int64_t next, comp;
        e = classify_page(job, h, e, c.pos, ds2, pg, &next, &comp);
        if (comp > 0) {
          pg.scratch_offset = scratch;
          scratch += comp;
        }
        pg.read_status = e;
        if (k < job.page_cap && lane_id() == 0) pages[job.page_base + k] = pg;
        if (h.type == 0 || h.type == 3) slots += pg.num_values;
        if (h.type == 2) {
          ds2 = true;
          dict_page = k;
        }
        p2 = next;
      }
      if (stride_walk(job, j, pages, spos, slen, snp, slots, scratch, sh) && lane_id() == 0) job.dict_page = dict_page;
      return;
    }
  } else if (job.scan_fallback != 1) {
    return;
  }
  Window win{gconst(job.data), job.data_len, kFarAway, lds_ptr(sh.win)};
  int64_t pos = 0;
  int np = 0;
  int status = kOK;
  bool dict_seen = false;
  int dict_page = -1;
  int64_t scratch = 0;
  int64_t slots = 0;
  const int lane = lane_id();
  while (tcs - pos > 0) {
    Compact<WinSrc> c;
    c.src.w = win;
    c.pos = pos;
    c.frames = sh.frames;
    c.last = sh.last;
    c.nlast = 0;
    c.last_id = 0;
    c.bool_set = false;
    c.bool_val = false;
    PageHdr h;
    int e = c.read_page_header(&h);
    win = c.src.w;
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
    if (prewalk > 0) job.scan_fallback = 2;
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
// One 1024-lane block per job: the job's pages in the list (at the offset of
// the pages of the jobs before it), and each data page's region of the value
// stream's run table / block index — an exclusive scan of a bound from the
// page's sizes (the same bound reg_stream used to take with two contended
// atomics per page): a value stream of B bytes and n values has at most
// B/2 + 2 runs and 2 n/kHBlock + 2 runs/kHBlockRuns + B/(kHBlockBytes/2) + 5 blocks.
__global__ void __launch_bounds__(1024) k_page_list(JobDev* jobs, PageDev* pages, int n_jobs, int* list, int list_cap,
                                                    int* total, int* queues) {
  __shared__ int64_t part[17];
  __shared__ int s_off;
  const int j = blockIdx.x;
  auto pages_of = [&](int i) {
    int n = jobs[i].num_pages;
    if (n > jobs[i].page_cap) n = jobs[i].page_cap;
    if (jobs[i].status == kCAPACITY) n = 0;
    return n;
  };
  if (threadIdx.x == 0) {
    int off = 0;
    for (int i = 0; i < j; i++) off += pages_of(i);
    s_off = off;
    if (j == n_jobs - 1) {
      const int all = off + pages_of(j);
      *total = all < list_cap ? all : list_cap;
      for (int q = 0; q < 16; q++) queues[q] = 0;  // ctr[8..23]
      for (int q = kCtrItems; q <= kCtrLongWalk; q++) queues[q - 8] = 0;  // the big-page counters
    }
  }
  __syncthreads();
  const int off = s_off;
  JobDev& job = jobs[j];
  const int n = pages_of(j);
  int64_t rc = 0, bc = 0;
  // rounds of 1024 pages, the next round's page fields loaded (unconditionally,
  // index clamped) before this round's stores: see k_page_chain
  struct F { int32_t type, usize, csize, nv; int64_t so; };
  auto fetch = [&](int i, F& f) {
    const PageDev& pg = pages[job.page_base + (i < n ? i : n - 1)];
    f.type = pg.page_type;
    f.usize = pg.usize;
    f.csize = pg.csize;
    f.nv = pg.num_values;
    f.so = pg.scratch_offset;
  };
  F cur;
  if (n > 0) fetch((int)threadIdx.x, cur);
  for (int b = 0; b < n; b += 1024) {
    const int i = b + threadIdx.x;
    int64_t nr = 0, nb = 0;
    if (i < n && (cur.type == 0 || cur.type == 3)) {
      const int64_t B = cur.so >= 0 ? (int64_t)(uint32_t)cur.usize : (int64_t)(uint32_t)cur.csize;
      nr = B / 2 + 2;
      // the lane walker's greedy blocks: n/kHBlock + runs/kHBlockRuns + B/(kHBlockBytes/2) + 3
      nb = (int64_t)(uint32_t)cur.nv / kHBlock + nr / kHBlockRuns + B / (kHBlockBytes / 2) + 3;
    }
    int64_t tr, tb;
    const int64_t er = block_excl_scan<1024>(nr, &tr, part);
    const int64_t eb = block_excl_scan<1024>(nb, &tb, part);
    F nxt;
    if (b + 1024 < n) fetch(b + 1024 + (int)threadIdx.x, nxt);
    if (i < n) {
      if (off + i < list_cap) list[off + i] = (int)(job.page_base + i);
      pages[job.page_base + i].run_off = rc + er;
      pages[job.page_base + i].blk_off = bc + eb;
    }
    rc += tr;
    bc += tb;
    cur = nxt;
  }
  if (threadIdx.x == 0) {
    job.run_used = rc;
    job.blk_used = bc;
    if (rc > job.run_cap || bc > job.blk_cap) job.status = kCAPACITY;  // the host grows the run arenas
  }
}

}  // namespace pqg
