// pqg_runtime.hip — host runtime behind include/pqgpu.h (libpqgpu.so).
//
// One pqg_ctx per GPU: a HIP stream, grow-only device arenas and a pinned
// host mirror of the job table.  pqg_decode_chunks_async enqueues the kernel
// pipeline of pqg_kernels.hip for a batch of column chunks whose bytes are
// already resident in HBM; pqg_sync waits and reports per-chunk status.  No
// allocation or host synchronisation happens inside the enqueue once the
// arenas have grown to the working-set size (capture-safe steady state).
#include <hip/hip_runtime.h>
#include <cstdlib>

#include <algorithm>
#include <cstdio>
#include <map>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/pqgpu.h"
#include "pqg_common.h"

namespace pqg {
int assemble_launch(hipStream_t s, const pqg_assemble_args* a, int64_t* seg_scratch, int64_t* tot);  // pqg_assemble.hip
int list_count_launch(hipStream_t s, const pqg_list_args* a, int64_t* seg_scratch, int64_t* tot);    // pqg_assemble.hip
int list_write_launch(hipStream_t s, const pqg_list_args* a, int64_t* seg_scratch);                  // pqg_assemble.hip
int pack_levels_launch(hipStream_t s, const uint8_t* levels, int64_t n, int bw, uint8_t* packed);     // pqg_assemble.hip
}

namespace pqg {
__global__ void k_tile_jobs(const JobDev* jobs, int* tile_job);
__global__ void k_page_cands(JobDev* jobs, const int* tile_job, int* tile_count, int* tile_okc, int64_t* cand_pos,
                             int* cand_list, int* cand_total, int region);
__global__ void k_cand_parse(JobDev* jobs, const int* tile_job, const int* cand_list, const int* cand_total, int region,
                             int* tile_okc,
                             const int64_t* cand_pos, Cand* cands);
__global__ void k_tile_scan(JobDev* jobs, const int* tile_count, const int* tile_okc, int* tile_off, int* tile_okoff);
__global__ void k_cand_link(JobDev* jobs, const int* tile_job, int64_t total_tiles, const int* tile_count,
                            const int* tile_off, const int* tile_okoff, const Cand* cands, int* succ, int* idx2slot,
                            int* ok2slot);
__global__ void k_page_chain(JobDev* jobs, PageDev* pages, const Cand* cands, const int* succ,
                             const int* idx2slot, const int* ok2slot, int* order);
__global__ void k_scan_pages(JobDev* jobs, PageDev* pages, int n_jobs, int prewalk, int stride);
__global__ void k_page_list(JobDev* jobs, PageDev* pages, int n_jobs, int* list, int list_cap, int* total,
                            int* queues);
__global__ void k_snappy(JobDev* jobs, PageDev* pages, const int* list, const int* total, int* queue,
                         uint8_t* scratch);
__global__ void k_inflate(JobDev* jobs, PageDev* pages, const int* list, const int* total, int* queue,
                          uint8_t* scratch, int mode);
__global__ void k_inflate_s(JobDev* jobs, PageDev* pages, const int* list, const int* total, int* queue,
                            uint8_t* scratch);
__global__ void k_snap_plan(const JobDev* jobs, PageDev* pages, const int* list, const int* total, int* ctr,
                            SnapSub* subs, int sub_cap, int* seg_page, int seg_cap);
__global__ void k_snap_seg(const JobDev* jobs, const PageDev* pages, const int* seg_page, const int* seg_total,
                           int seg_cap, uint2* F);
__global__ void k_snap_link(const JobDev* jobs, PageDev* pages, const int* list, const int* total, SnapSub* subs,
                            const uint2* F);
__global__ void k_snap_decode(const JobDev* jobs, PageDev* pages, const SnapSub* subs, const int* sub_total,
                              int sub_cap, int* queue, uint8_t* scratch);
__global__ void k_page_levels(JobDev* jobs, PageDev* pages, const int* list, const int* total, int* queue,
                              uint8_t* scratch, HStream* streams, uint8_t* def_arena, uint8_t* rep_arena,
                              LongLev* longs, int long_cap, LevPiece* pieces, int piece_cap, int split);
__global__ void k_page_levels_w1(JobDev* jobs, PageDev* pages, const int* list, const int* total, int* queue,
                              uint8_t* scratch, HStream* streams, uint8_t* def_arena, uint8_t* rep_arena,
                              LongLev* longs, int long_cap, LevPiece* pieces, int piece_cap, int split);
__global__ void k_dict_resolve(JobDev* jobs, int n_jobs, PageDev* pages, uint8_t* scratch);
__global__ void k_level_long(PageDev* pages, const int* ctr, const LongLev* longs, int long_cap,
                             const LevPiece* pieces, int piece_cap, int* queue);
__global__ void k_hybrid_walk(const PageDev* pages, const int* list, const int* total, HStream* streams,
                              RunEnt* runs, BlockDesc* blks, LongWalk* longs, int long_cap);
__global__ void k_walk_long(const int* ctr, const LongWalk* longs, int long_cap, BlockDesc* blks);
__global__ void k_nn_scan(JobDev* jobs, PageDev* pages, uint8_t* scratch, const HStream* streams, const BlockDesc* blks,
                          int* ctr, PartRec* parts, int64_t parts_cap);
template <int Mode>
__global__ void k_values(JobDev* jobs, PageDev* pages, const PartRec* parts, const int* total, int* queue,
                         uint8_t* value_arena, const HStream* streams, const RunEnt* runs, const BlockDesc* blks);
__global__ void k_dict_plan(JobDev* jobs, PageDev* pages, const PartRec* parts, const int* total,
                            uint8_t* value_arena, const HStream* streams, const RunEnt* runs, const BlockDesc* blks,
                            VRec* recs);
__global__ void k_dict4(PageDev* pages, const int* total, int* queue, const VRec* recs, int big);
__global__ void k_dict4_big(PageDev* pages, const int* total, int* queue, const VRec* recs);
constexpr int kBigDictThreads = 512;
__global__ void k_finalize(JobDev* jobs, int n_jobs, PageDev* pages);
__global__ void k_str_dict(JobDev* jobs, PageDev* pages, int64_t* doffs_arena);
__global__ void k_str_count(JobDev* jobs, PageDev* pages, PartRec* parts, const int* total, int* queue,
                            int64_t* offs_arena, const HStream* streams, const RunEnt* runs, const BlockDesc* blks);
__global__ void k_str_plain(JobDev* jobs, PageDev* pages, const int* list, const int* total, int* queue,
                            int64_t* offs_arena);
__global__ void k_char_scan(JobDev* jobs, PageDev* pages, PartRec* parts, int64_t* offs_arena);
__global__ void k_str_delta(JobDev* jobs, PageDev* pages, const int* list, const int* total, int* queue,
                            int64_t* offs_arena);
__global__ void k_str_dba(JobDev* jobs, PageDev* pages, const int* list, const int* total, int* queue,
                          uint8_t* value_arena, int64_t* offs_arena);
__global__ void k_str_copy(JobDev* jobs, PageDev* pages, const PartRec* parts, const int* total, int* queue,
                           uint8_t* value_arena, int64_t* offs_arena);
}  // namespace pqg

#ifdef PQG_PROFILE
namespace pqg {
int prof_read_values(unsigned long long* out);
int prof_read_levels(unsigned long long* out);
int prof_read_strings(unsigned long long* out);
int prof_read_snappy(unsigned long long* out);
int prof_read_dict(unsigned long long* out);
int prof_read_inflate(unsigned long long* out);
}  // namespace pqg
#endif

using namespace pqg;

namespace {

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  int grow(size_t bytes) {
    if (bytes <= cap) return 0;
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max(bytes, (size_t)256);
    want = (want + 0xFFFFF) & ~(size_t)0xFFFFF;  // 1 MiB granules
    if (hipMalloc(&p, want) != hipSuccess) {
      p = nullptr;
      return -1;
    }
    cap = want;
    return 0;
  }
  void release() {
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

constexpr int kStages = 10;
constexpr int kWalkLanes = kWalkThreads;  // k_hybrid_walk block size (pqg_common.h)
// stages timed by pqg_last_timings: scan (K1a-e), list, snappy, setup, walk, levels, nn_scan, values, strings,
// finalize
constexpr int kMaxAttempts = 6;  // decode + up to 5 arena grows in one pqg_sync

// Arena capacities of one chunk job (see plan_batch); 0 = use the planner's estimate.
struct Caps {
  int64_t pages = 0, slots = 0, scratch = 0, values = 0, runs = 0, blks = 0, doffs = 0;
};
// Capacities learned for a chunk (its bytes, size and value count), kept for
// later decodes of the same chunk so a grown arena is planned right away.
struct JobKey {
  uintptr_t data;
  int64_t tcs, hint;
  bool operator<(const JobKey& o) const {
    return data != o.data ? data < o.data : tcs != o.tcs ? tcs < o.tcs : hint < o.hint;
  }
};

int64_t align_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

// Grid of a queue-driven kernel: shard s of a queue (items s, s + 8, ...) is
// pulled only by blocks with blockIdx & 7 == s (queue_pull, pqg_device.h), so
// every launch needs at least kQShards blocks or a shard's pages are skipped.
unsigned qgrid(int64_t blocks) { return (unsigned)std::max<int64_t>(blocks, kQShards); }

int value_width_of(const pqg_column_desc& c) {
  switch (c.physical_type) {
    case PQG_BOOLEAN: return 1;
    case PQG_INT32: case PQG_FLOAT: return 4;
    case PQG_INT64: case PQG_DOUBLE: return 8;
    case PQG_INT96: return 12;
    case PQG_FIXED_LEN_BYTE_ARRAY: return c.type_length > 0 ? c.type_length : 0;
  }
  return 0;
}

}  // namespace

struct pqg_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int num_cus = 256;
  DevBuf vrecs;          // VRec per page-list entry (k_dict_plan -> k_dict4)
  int dict4_per_cu = 2;  // resident k_dict4 workgroups per CU (LDS-bound), from the occupancy query
  int dict4_threads = 256;
  bool dict4 = true;     // k_dict4 for 4-byte dictionary pages (PQG_DICT4=0: k_values<1>, for A/B runs)
  bool stride = true;     // the K1 stride walk of equal-page chunks (PQG_STRIDE=0: the candidate scan takes them)
  bool dict_big = true;   // k_dict4_big for dictionaries past 4096 entries (PQG_DICT_BIG=0: k_dict4 gathers them)
  bool lev1 = true;       // the whole-page 1-bit level decoder in k_page_levels_w1 (PQG_LEV1=0: the batch decoder alone)
  int seg_waves = 31;     // PQG_SEG_WAVES: k_snap_seg waves per CU (its 5 KiB of LDS allow 31; 16: C4 +10 %)
  int levlong_waves = 28; // PQG_LEVLONG_WAVES: k_level_long waves per CU (66 VGPRs: 7 per SIMD; 8: C5 0.61 ms, 28: 0.32)
  int link_waves = 16;    // PQG_LINK_WAVES: k_snap_link waves per CU (one wave per big page; 4: C4 +50 %)
  int snappy_per_cu = 2;  // resident k_snappy waves per CU (LDS-bound: the output history ring)
  int inflate_per_cu = 8; // resident k_inflate_s waves per CU (LDS / VGPR bound), from the occupancy query
  DevBuf jobs, pages, list, counters, def_arena, rep_arena, value_arena, scratch;
  DevBuf tile_job;  // K1: tile -> job
  DevBuf tile_count, tile_okc, tile_off, tile_okoff, cand_pos, cands, succ, idx2slot, ok2slot, order;  // K1
  DevBuf streams, runs, blks;  // K3 hybrid run tables
  DevBuf cand_list, vlists;
  DevBuf asm_seg;  // K8 per-segment counts + totals
  DevBuf offs_arena, doffs_arena;  // K7: value offsets (int64), dictionary record starts
  DevBuf page_stage;               // pqg_decode_page: [dictionary page][data page]
  DevBuf blk_src, blk_dst, blk_meta, blk_subs, blk_segpage, blk_F;  // pqg_block_decompress
  DevBuf sn_subs, sn_segpage, sn_F;   // K2 split: sub-block table, segment -> page, segment exits
  int64_t sn_sub_cap = 0, sn_seg_cap = 0;
  DevBuf parts, lev_long, lev_pieces, walk_long;  // big pages: values-stage parts, long level / value-stream runs
  int64_t parts_cap = 0, lev_long_cap = 0, lev_piece_cap = 0, walk_long_cap = 0;
  int64_t total_tiles = 0;
  JobDev* h_jobs = nullptr;  // pinned
  int h_jobs_cap = 0;
  std::vector<pqg_chunk_job> cur;       // jobs of the in-flight batch
  std::vector<JobDev> plan;             // per-job capacities used
  std::vector<Caps> force;              // per-job capacities forced for this batch
  std::map<JobKey, Caps> learned;       // grown capacities, across calls
  // chunks the K1 prewalk / stride walk did not take (scan_fallback != 2): a batch of only
  // such chunks skips the prewalk launch (performance only: the candidate
  // scan settles any chunk, so a stale entry never changes a result)
  std::map<JobKey, bool> many_pages;
  bool prewalk = true;
  int launches = 0;                     // pipeline launches of the last decode
  bool any_var = false;                 // batch holds variable-length columns
  bool any_fixed_other = false;         // batch holds fixed-width columns (k_values<0> pages possible)
  bool any_w4 = false;                  // batch holds 4-byte columns (the 4-byte dictionary stage: mode 1 pages)
  bool any_levels = false;              // batch holds columns with levels (long level runs possible)
  int n_jobs = 0;
  int64_t list_cap = 0;
  hipEvent_t ev[kStages + 1];
  hipEvent_t ev_k8[4];   // K8: [0,1] assemble / list count, [2,3] list write
  float k8_ms = 0.f;     // device time of the last pqg_assemble / pqg_assemble_list
  bool timed = true;
  bool last_timed = false;              // the last pipeline launch recorded the stage events
};

static int hip_ok(hipError_t e) { return e == hipSuccess ? PQG_OK : PQG_ERR_HIP; }

extern "C" {

const char* pqg_status_string(int s) {
  switch (s) {
    case PQG_OK: return "ok";
    case PQG_ERR_EOF: return "unexpected end of stream";
    case PQG_ERR_THRIFT: return "page header: thrift decode failed";
    case PQG_ERR_PAGE_HEADER: return "page header: missing or negative field";
    case PQG_ERR_SIZE: return "page size mismatch";
    case PQG_ERR_SNAPPY: return "snappy: corrupt input";
    case PQG_ERR_RLE: return "rle: invalid run";
    case PQG_ERR_DICT_INDEX: return "dict: invalid index";
    case PQG_ERR_BIT_WIDTH: return "invalid bit width";
    case PQG_ERR_DELTA: return "delta: invalid stream";
    case PQG_ERR_UNSUPPORTED: return "unsupported encoding/codec/type";
    case PQG_ERR_DICT_PAGE: return "there should be only one dictionary";
    case PQG_ERR_BYTE_ARRAY: return "bytearray/plain: len is negative";
    case PQG_ERR_LEVELS: return "level reader is not initialized";
    case PQG_ERR_FIXED_LEN: return "bytearray/delta: value length is not the fixed length";
    case PQG_ERR_GZIP: return "gzip: invalid data";
    case PQG_ERR_CAPACITY: return "capacity";
    case PQG_ERR_INVALID_ARG: return "invalid argument";
    case PQG_ERR_HIP: return "HIP runtime error";
    case PQG_ERR_METADATA: return "invalid file metadata";
  }
  return "unknown";
}

int pqg_ctx_create(int device, pqg_ctx** out) {
  if (!out) return PQG_ERR_INVALID_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return PQG_ERR_HIP;
  if (hipSetDevice(device) != hipSuccess) return PQG_ERR_HIP;
  pqg_ctx* c = new pqg_ctx();
  c->device = device;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->num_cus = prop.multiProcessorCount;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return PQG_ERR_HIP;
  }
  for (auto& e : c->ev) hipEventCreate(&e);
  for (auto& e : c->ev_k8) hipEventCreate(&e);
  if (const char* e = getenv("PQG_DICT4")) c->dict4 = atoi(e) != 0;
  if (const char* e = getenv("PQG_DICT_BIG")) c->dict_big = atoi(e) != 0;
  if (const char* e = getenv("PQG_STRIDE")) c->stride = atoi(e) != 0;
  if (const char* e = getenv("PQG_LEV1")) c->lev1 = atoi(e) != 0;
  if (const char* e = getenv("PQG_SEG_WAVES")) c->seg_waves = atoi(e) > 0 ? atoi(e) : c->seg_waves;
  if (const char* e = getenv("PQG_LEVLONG_WAVES")) c->levlong_waves = atoi(e) > 0 ? atoi(e) : c->levlong_waves;
  if (const char* e = getenv("PQG_LINK_WAVES")) c->link_waves = atoi(e) > 0 ? atoi(e) : c->link_waves;
  {
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&k_dict4)) == hipSuccess && fa.maxThreadsPerBlock > 0)
      c->dict4_threads = fa.maxThreadsPerBlock;  // kDWaves * 64 (pqg_dict.hip)
    int o = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, reinterpret_cast<const void*>(&k_dict4), c->dict4_threads, 0) ==
            hipSuccess && o > 0)
      c->dict4_per_cu = o;
  }
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(&k_snappy), 64, 0) ==
          hipSuccess &&
      occ > 0)
    c->snappy_per_cu = occ;
  occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(&k_inflate_s), 64, 0) ==
          hipSuccess && occ > 0)
    c->inflate_per_cu = occ;
  // counters: ctr[0..1023] + the kQShards-sharded work queues and the per-stage flags
  if (c->counters.grow(sizeof(int) * (size_t)(1024 + kQueueSlots * kQueueInts))) {
    pqg_ctx_destroy(c);
    return PQG_ERR_HIP;
  }
  *out = c;
  return PQG_OK;
}

void pqg_ctx_destroy(pqg_ctx* c) {
  if (!c) return;
  hipSetDevice(c->device);
  hipStreamSynchronize(c->stream);
  for (auto& e : c->ev) hipEventDestroy(e);
  for (auto& e : c->ev_k8) hipEventDestroy(e);
  for (DevBuf* b : {&c->jobs, &c->pages, &c->list, &c->counters, &c->def_arena, &c->rep_arena, &c->value_arena,
                    &c->scratch, &c->streams, &c->runs, &c->blks, &c->cand_list, &c->vlists, &c->tile_count, &c->tile_okc, &c->tile_off, &c->tile_okoff, &c->cand_pos, &c->cands, &c->succ, &c->idx2slot,
                    &c->ok2slot, &c->order, &c->asm_seg, &c->offs_arena, &c->doffs_arena, &c->page_stage,
                    &c->blk_src, &c->blk_dst, &c->blk_meta, &c->tile_job, &c->sn_subs, &c->sn_segpage, &c->sn_F,
                    &c->blk_subs, &c->blk_segpage, &c->blk_F, &c->vrecs, &c->parts, &c->lev_long, &c->lev_pieces,
                    &c->walk_long})
    b->release();
  if (c->h_jobs) hipHostFree(c->h_jobs);
  hipStreamDestroy(c->stream);
  delete c;
}

int pqg_device_alloc(pqg_ctx* c, int64_t bytes, void** dptr) {
  if (!c || !dptr) return PQG_ERR_INVALID_ARG;
  hipSetDevice(c->device);
  return hip_ok(hipMalloc(dptr, (size_t)std::max<int64_t>(bytes, 1)));
}
int pqg_device_free(pqg_ctx* c, void* dptr) {
  if (!c) return PQG_ERR_INVALID_ARG;
  hipSetDevice(c->device);
  return hip_ok(hipFree(dptr));
}
int pqg_memcpy_h2d(pqg_ctx* c, void* dst, const void* src, int64_t bytes) {
  if (!c) return PQG_ERR_INVALID_ARG;
  hipSetDevice(c->device);
  int e = hip_ok(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyHostToDevice, c->stream));
  if (e) return e;
  return hip_ok(hipStreamSynchronize(c->stream));
}
int pqg_memcpy_d2h(pqg_ctx* c, void* dst, const void* src, int64_t bytes) {
  if (!c) return PQG_ERR_INVALID_ARG;
  hipSetDevice(c->device);
  int e = hip_ok(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToHost, c->stream));
  if (e) return e;
  return hip_ok(hipStreamSynchronize(c->stream));
}

// Plan arena regions for the current batch and upload the job table.
static int plan_batch(pqg_ctx* c) {
  const int n = c->n_jobs;
  if (c->h_jobs_cap < n) {
    if (c->h_jobs) hipHostFree(c->h_jobs);
    c->h_jobs_cap = std::max(n, 64);
    if (hipHostMalloc((void**)&c->h_jobs, sizeof(JobDev) * (size_t)c->h_jobs_cap) != hipSuccess) return PQG_ERR_HIP;
  }
  int64_t page_total = 0, slot_total = 0, value_total = 0, scratch_total = 0, tile_total = 0, run_total = 0,
          blk_total = 0, offs_total = 0, doffs_total = 0, seg_total = 0;
  c->plan.resize((size_t)n);
  for (int i = 0; i < n; i++) {
    const pqg_chunk_job& in = c->cur[(size_t)i];
    const Caps& f = c->force[(size_t)i];
    JobDev d;
    memset(&d, 0, sizeof(d));
    d.data = in.data;
    d.data_len = in.data_len;
    d.tcs = in.total_compressed_size;
    d.data_page_offset = in.data_page_offset;
    d.type = in.col.physical_type;
    d.type_length = in.col.type_length;
    d.max_def = in.col.max_def;
    d.max_rep = in.col.max_rep;
    d.codec = in.col.codec;
    d.has_dict_off = in.has_dict_page_offset;
    d.value_width = value_width_of(in.col);
    d.no_prewalk = c->many_pages.count(JobKey{(uintptr_t)in.data, in.total_compressed_size, in.num_values_hint}) ? 1 : 0;
    int64_t pcap = in.total_compressed_size / 256 + 16;
    if (f.pages > 0) pcap = f.pages;
    pcap = std::min<int64_t>(pcap, (int64_t)1 << 30);
    d.page_cap = (int32_t)pcap;
    d.page_base = page_total;
    page_total += pcap;
    int64_t scap = std::max<int64_t>(in.num_values_hint, 0) + 64;
    if (f.slots > 0) scap = f.slots;
    d.slot_cap = scap;
    d.slot_base = slot_total;
    slot_total += align_up(scap, 256);
    // variable-length values: chars estimated from the page bytes (dictionary
    // chunks may need more: the first decode reports it and the arena grows)
    int64_t vcap = d.value_width > 0 ? scap * d.value_width
                                     : std::max<int64_t>(in.total_uncompressed_size, in.total_compressed_size) + 1024;
    if (f.values > 0) vcap = f.values;
    d.value_cap = vcap;
    d.value_base = value_total;
    value_total += align_up(vcap, 256);
    int64_t xcap = 0;
    if (in.col.codec != PQG_CODEC_UNCOMPRESSED)
      xcap = std::max<int64_t>(in.total_uncompressed_size, in.total_compressed_size) + pcap * 16 + 1024;
    if (f.scratch > 0) xcap = f.scratch;
    d.scratch_cap = xcap;
    d.scratch_base = scratch_total;
    scratch_total += align_up(xcap, 256);
    if (in.col.codec != PQG_CODEC_UNCOMPRESSED) seg_total += in.total_compressed_size / kSnapSeg + pcap;
    d.dict_page = -1;
    d.error_page = -1;
    const int64_t lim = std::max<int64_t>(0, std::min(in.total_compressed_size, in.data_len));
    // hybrid run tables: a stream of n bytes has at most n/2 + 2 runs, and a
    // page at most three streams (see reg_stream)
    int64_t rcap = (in.total_compressed_size + xcap) / 2 + 6 * pcap + 64;
    if (f.runs > 0) rcap = f.runs;
    d.run_cap = rcap;
    d.run_base = run_total;
    run_total += rcap;
    int64_t bcap = 3 * (scap / kHBlock + 3 * pcap) + rcap / kHBlockRuns + 2 * rcap / (kHBlockBytes / 2) + 64;
    if (f.blks > 0) bcap = f.blks;
    d.blk_cap = bcap;
    d.blk_base = blk_total;
    blk_total += bcap;
    // offsets: variable-length values; FLBA columns too (their DELTA_BYTE_ARRAY
    // pages park prefix / suffix lengths there, k_str_delta)
    if (d.value_width == 0 || d.type == PQG_FIXED_LEN_BYTE_ARRAY) {
      d.offs_cap = scap + 1;
      d.offs_base = offs_total;
      offs_total += align_up(scap + 1, 32);
    }
    if (d.value_width == 0) {
      // dictionary entries take >= 4 bytes each
      int64_t dcap = std::min<int64_t>(std::max<int64_t>(in.total_uncompressed_size, 0) / 4, 1 << 17) + 64;
      if (f.doffs > 0) dcap = f.doffs;
      d.doffs_cap = dcap;
      d.doffs_base = doffs_total;
      doffs_total += align_up(dcap, 32);
    }
    d.tile_base = tile_total;
    d.n_tiles = (int32_t)((lim + kScanTile - 1) / kScanTile);
    tile_total += d.n_tiles;
    c->plan[(size_t)i] = d;
    c->h_jobs[i] = d;
  }
  c->list_cap = page_total;
  // big pages (pqg_common.h): a page of nn values has <= nn / kPart + 1 parts;
  // a long level run (rep and def streams) has > kLongLev values, a long
  // value-stream run > kLongWalk
  c->parts_cap = page_total + slot_total / kPart + n + 64;
  c->lev_long_cap = 2 * slot_total / kLongLev + 64;
  c->lev_piece_cap = 2 * slot_total / kLevPiece + 2 * c->lev_long_cap + 64;
  c->walk_long_cap = slot_total / kLongWalk + 64;
  if (c->parts.grow(sizeof(PartRec) * (size_t)c->parts_cap) || c->lev_long.grow(sizeof(LongLev) * (size_t)c->lev_long_cap) ||
      c->lev_pieces.grow(sizeof(LevPiece) * (size_t)c->lev_piece_cap) ||
      c->walk_long.grow(sizeof(LongWalk) * (size_t)c->walk_long_cap))
    return PQG_ERR_HIP;
  // K2 split tables: a page of u bytes has ceil(u / 64 KiB) sub-blocks (>= 1)
  // and a block of b bytes ceil(b / 4 KiB) segments
  c->sn_sub_cap = scratch_total / kSnapSub + page_total + 64;
  c->sn_seg_cap = seg_total + 64;
  if (c->sn_subs.grow(sizeof(SnapSub) * (size_t)c->sn_sub_cap) || c->sn_segpage.grow(sizeof(int) * (size_t)c->sn_seg_cap) ||
      c->sn_F.grow(sizeof(uint2) * 64 * (size_t)c->sn_seg_cap))
    return PQG_ERR_HIP;
  if (c->jobs.grow(sizeof(JobDev) * (size_t)n) || c->pages.grow(sizeof(PageDev) * (size_t)page_total) ||
      c->list.grow(sizeof(int) * (size_t)std::max<int64_t>(page_total, 1)) || c->def_arena.grow((size_t)slot_total + 64) ||
      c->rep_arena.grow((size_t)slot_total + 64) || c->value_arena.grow((size_t)value_total + 64) ||
      c->scratch.grow((size_t)scratch_total + 64) || c->tile_count.grow(sizeof(int) * (size_t)tile_total + 64) ||
      c->tile_off.grow(sizeof(int) * (size_t)tile_total + 64) || c->tile_okc.grow(sizeof(int) * (size_t)tile_total + 64) ||
      c->tile_okoff.grow(sizeof(int) * (size_t)tile_total + 64) || c->tile_job.grow(sizeof(int) * (size_t)tile_total + 64) ||
      c->ok2slot.grow(sizeof(int) * (size_t)tile_total * kCandPerTile + 64) ||
      c->cand_pos.grow(sizeof(int64_t) * (size_t)tile_total * kCandPerTile + 64) ||
      c->cand_list.grow(sizeof(int) * (size_t)(tile_total + kQShards) * kCandPerTile + 64) ||
      c->vlists.grow(sizeof(int) * 3 * (size_t)page_total + 64) ||
      c->cands.grow(sizeof(Cand) * (size_t)tile_total * kCandPerTile + 64) ||
      c->succ.grow(sizeof(int) * (size_t)tile_total * kCandPerTile + 64) ||
      c->idx2slot.grow(sizeof(int) * (size_t)tile_total * kCandPerTile + 64) ||
      c->order.grow(sizeof(int) * (size_t)page_total + 64) ||
      c->streams.grow(sizeof(HStream) * 3 * (size_t)page_total + 64) ||
      // slack past the last entry: k_dict4 stages run / descriptor granules past a stream's end
      c->runs.grow(sizeof(RunEnt) * (size_t)run_total + 8192) || c->blks.grow(sizeof(BlockDesc) * (size_t)blk_total + 8192) ||
      c->vrecs.grow(sizeof(VRec) * (size_t)std::max<int64_t>(c->parts_cap, 1)) ||
      c->offs_arena.grow(sizeof(int64_t) * (size_t)offs_total + 64) ||
      c->doffs_arena.grow(sizeof(int64_t) * (size_t)doffs_total + 64))
    return PQG_ERR_HIP;
  c->total_tiles = tile_total;
  return hip_ok(hipMemcpyAsync(c->jobs.p, c->h_jobs, sizeof(JobDev) * (size_t)n, hipMemcpyHostToDevice, c->stream));
}

// K2: the split snappy decode of every compressed page in `list` (pqg_snappy.hip):
// plan -> segment exits -> chain link -> 64 KiB sub-blocks, then the serial
// path for the pages it sent back.  sctr: 2 ints (sub-block / segment totals),
// q_split and q_serial: zeroed sharded queues.
struct SnapTables {
  SnapSub* subs;
  int sub_cap;
  int* segpage;
  int seg_cap;
  uint2* F;
};
static void launch_snappy(pqg_ctx* c, hipStream_t s, JobDev* jobs, PageDev* pages, const int* list, const int* total,
                          int64_t list_cap, int* sctr, int* q_split, int* q_serial, uint8_t* scratch,
                          const SnapTables& T) {
  const int waves = c->num_cus * c->snappy_per_cu;  // as many as fit (LDS: the history ring)
  hipMemsetAsync(sctr, 0, 2 * sizeof(int), s);
  hipLaunchKernelGGL(k_snap_plan, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((list_cap + 255) / 256, c->num_cus * 4))),
                     dim3(256), 0, s, jobs, pages, list, total, sctr, T.subs, T.sub_cap, T.segpage, T.seg_cap);
  hipLaunchKernelGGL(k_snap_seg, dim3(c->num_cus * c->seg_waves), dim3(64), 0, s, jobs, pages, T.segpage, sctr + 1, T.seg_cap, T.F);
  hipLaunchKernelGGL(k_snap_link, dim3(c->num_cus * c->link_waves), dim3(64), 0, s, jobs, pages, list, total, T.subs, T.F);
  hipLaunchKernelGGL(k_snap_decode, dim3(qgrid(waves)), dim3(64), 0, s, jobs, pages, T.subs, sctr, T.sub_cap, q_split,
                     scratch);
  hipLaunchKernelGGL(k_snappy, dim3(qgrid(waves)), dim3(64), 0, s, jobs, pages, list, total, q_serial, scratch);
}

static int launch_pipeline(pqg_ctx* c) {
  const int n = c->n_jobs;
  c->launches++;
  c->last_timed = c->timed;
  JobDev* jobs = (JobDev*)c->jobs.p;
  PageDev* pages = (PageDev*)c->pages.p;
  int* list = (int*)c->list.p;
  int* ctr = (int*)c->counters.p;  // [0] total pages in the list
  // work queues (sharded over the XCDs, see queue_pull): 0 snappy, 1 levels,
  // 2 values<0>, 3 values<1>, 4 str_count, 5 str_plain, 6 str_copy, 7 the
  // candidate list heads of k_page_cands, 8 values<3> (DELTA_BINARY_PACKED); then
  // the per-stage page flags (kModePresentOff)
  auto Q = [&](int k) { return ctr + 1024 + k * kQueueInts; };
  uint8_t* scratch = (uint8_t*)c->scratch.p;
  // page-queue kernels: one wave per page; enough waves per SIMD to hide the
  // dependent HBM reads (bounded by VGPRs / LDS per kernel)
  const int waves = c->num_cus * 20;
  hipStream_t s = c->stream;
  if (c->timed) hipEventRecord(c->ev[0], s);
  hipMemsetAsync(Q(0), 0, sizeof(int) * kQueueSlots * kQueueInts, s);  // queues + the stage flags (kModePresentOff)
  const int64_t nt = c->total_tiles;
  int* tcount = (int*)c->tile_count.p;
  int* toff = (int*)c->tile_off.p;
  Cand* cands = (Cand*)c->cands.p;
  int* tokc = (int*)c->tile_okc.p;
  int* tokoff = (int*)c->tile_okoff.p;
  // chunks of a few big pages (parquet-go's writer layout) are walked first
  // and skipped by the candidate scan
  if (c->prewalk) hipLaunchKernelGGL(k_scan_pages, dim3(n), dim3(64), 0, s, jobs, pages, n, kPrewalkPages, (int)c->stride);
  if (nt > 0) {
    int64_t* cpos = (int64_t*)c->cand_pos.p;
    int* clist = (int*)c->cand_list.p;
    const int region = (int)((nt + kQShards - 1) / kQShards) * kCandPerTile;  // one list region per head
    hipLaunchKernelGGL(k_tile_jobs, dim3(n), dim3(256), 0, s, jobs, (int*)c->tile_job.p);
    hipLaunchKernelGGL(k_page_cands, dim3((unsigned)nt), dim3(256), 0, s, jobs, (const int*)c->tile_job.p, tcount, tokc,
                       cpos, clist, Q(7),
                       region);
    hipLaunchKernelGGL(k_cand_parse, dim3((unsigned)std::min<int64_t>((nt * kCandPerTile + 255) / 256, c->num_cus * 4)),
                       dim3(256), 0, s, jobs, (const int*)c->tile_job.p, clist, Q(7), region, tokc, cpos, cands);
  }
  hipLaunchKernelGGL(k_tile_scan, dim3(n), dim3(1024), 0, s, jobs, tcount, tokc, toff, tokoff);
  if (nt > 0)
    hipLaunchKernelGGL(k_cand_link, dim3((unsigned)((nt * kCandPerTile + 255) / 256)), dim3(256), 0, s, jobs,
                       (const int*)c->tile_job.p, nt,
                       tcount, toff, tokoff, cands, (int*)c->succ.p, (int*)c->idx2slot.p, (int*)c->ok2slot.p);
  hipLaunchKernelGGL(k_page_chain, dim3(n), dim3(1024), 0, s, jobs, pages, cands, (const int*)c->succ.p,
                     (const int*)c->idx2slot.p, (const int*)c->ok2slot.p, (int*)c->order.p);
  hipLaunchKernelGGL(k_scan_pages, dim3(n), dim3(64), 0, s, jobs, pages, n, 0, 0);
  if (c->timed) hipEventRecord(c->ev[1], s);
  hipLaunchKernelGGL(k_page_list, dim3(n), dim3(1024), 0, s, jobs, pages, n, list,
                     (int)std::min<int64_t>(c->list_cap, INT32_MAX), ctr, ctr + 8);
  if (c->timed) hipEventRecord(c->ev[2], s);
  bool any_snappy = false, any_gzip = false;
  for (int i = 0; i < n; i++) {
    any_snappy |= c->cur[(size_t)i].col.codec == PQG_CODEC_SNAPPY;
    any_gzip |= c->cur[(size_t)i].col.codec == PQG_CODEC_GZIP;
  }
  if (any_snappy) {
    const SnapTables T{(SnapSub*)c->sn_subs.p, (int)std::min<int64_t>(c->sn_sub_cap, INT32_MAX), (int*)c->sn_segpage.p,
                       (int)std::min<int64_t>(c->sn_seg_cap, INT32_MAX), (uint2*)c->sn_F.p};
    launch_snappy(c, s, jobs, pages, list, ctr, c->list_cap, ctr + 32, Q(0), Q(kQueueSnapSerial), scratch, T);
  }
  if (any_gzip) {  // one wave per GZIP page (pqg_inflate.hip): the 8 KiB ring, then the pages it left
    hipLaunchKernelGGL(k_inflate_s, dim3(qgrid(c->num_cus * c->inflate_per_cu)), dim3(64), 0, s, jobs, pages, list, ctr,
                       Q(kQueueInflate), scratch);
    hipLaunchKernelGGL(k_inflate, dim3(qgrid(c->num_cus * 4)), dim3(64), 0, s, jobs, pages, list, ctr,
                       Q(kQueueInflateRedo), scratch, 1);
  }
  if (c->timed) hipEventRecord(c->ev[3], s);
  HStream* streams = (HStream*)c->streams.p;
  RunEnt* runs = (RunEnt*)c->runs.p;
  BlockDesc* blks = (BlockDesc*)c->blks.p;
  // setup + def/rep levels, one wave per data page (value streams registered
  // for the walk); long level runs then expand in pieces over the whole chip
  LongLev* llong = (LongLev*)c->lev_long.p;
  LevPiece* lpieces = (LevPiece*)c->lev_pieces.p;
  const int llc = (int)std::min<int64_t>(c->lev_long_cap, INT32_MAX), lpc = (int)std::min<int64_t>(c->lev_piece_cap, INT32_MAX);
  // each job's dictionary page
  hipLaunchKernelGGL(k_dict_resolve, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, jobs, n, pages, scratch);
  // pages of jobs with 1-bit levels (maxR = 0, maxD <= 1) to the w = 1
  // decoder, the others to the general one; a kernel with no job stays idle
  bool any_w1 = false, any_gen = false;
  for (int i = 0; i < n; i++) {
    const pqg_column_desc& d = c->cur[(size_t)i].col;
    (d.max_rep == 0 && d.max_def <= 1 ? any_w1 : any_gen) = true;
  }
  const int split = any_w1 && any_gen;
  if (any_w1)
    hipLaunchKernelGGL(k_page_levels_w1, dim3(qgrid(c->num_cus * 32)), dim3(64), 0, s, jobs, pages, list, ctr, Q(1),
                       scratch, streams, (uint8_t*)c->def_arena.p, (uint8_t*)c->rep_arena.p, llong, llc, lpieces, lpc,
                       split | (c->lev1 ? 2 : 0));
  if (any_gen)
    hipLaunchKernelGGL(k_page_levels, dim3(qgrid(c->num_cus * 24)), dim3(64), 0, s, jobs, pages, list, ctr,
                       Q(split ? kQueueLevGen : 1), scratch, streams, (uint8_t*)c->def_arena.p,
                       (uint8_t*)c->rep_arena.p, llong, llc, lpieces, lpc, split);
  // stages with no possible work are not launched (the host knows each job's
  // type and levels; the kernels' own flags stay as the backstop)
  if (c->any_levels)
    hipLaunchKernelGGL(k_level_long, dim3(qgrid(c->num_cus * c->levlong_waves)), dim3(64), 0, s, pages, ctr, llong, llc, lpieces, lpc,
                       Q(kQueueLevLong));
  if (c->timed) hipEventRecord(c->ev[4], s);
  const unsigned walk_blocks = (unsigned)std::max<int64_t>(
      1, std::min<int64_t>((c->list_cap + kWalkLanes - 1) / kWalkLanes, c->num_cus * (2048 / kWalkLanes)));
  LongWalk* wlong = (LongWalk*)c->walk_long.p;
  const int wlc = (int)std::min<int64_t>(c->walk_long_cap, INT32_MAX);
  // one lane per value stream
  hipLaunchKernelGGL(k_hybrid_walk, dim3(walk_blocks), dim3(kWalkLanes), 0, s, pages, list, ctr, streams, runs, blks,
                     wlong, wlc);
  hipLaunchKernelGGL(k_walk_long, dim3(c->num_cus * 2), dim3(256), 0, s, ctr, wlong, wlc, blks);
  if (c->timed) hipEventRecord(c->ev[5], s);
  if (c->timed) hipEventRecord(c->ev[6], s);
  PartRec* parts = (PartRec*)c->parts.p;
  hipLaunchKernelGGL(k_nn_scan, dim3(n), dim3(1024), 0, s, jobs, pages, scratch, streams, blks, ctr, parts, c->parts_cap);
  if (c->timed) hipEventRecord(c->ev[7], s);
  // every values kernel takes the work items (the pages' parts) and keeps the
  // ones whose vmode (set by k_page_levels) is its own
  const int64_t items_cap = c->parts_cap;
  if (!c->any_w4) {
    // no 4-byte column: no mode 1 page
  } else if (c->dict4) {  // 4-byte dictionary pages: pieces staged in LDS, small dictionaries in LDS (pqg_dict.hip)
    VRec* recs = (VRec*)c->vrecs.p;
    hipLaunchKernelGGL(k_dict_plan, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((items_cap + 255) / 256, c->num_cus * 4))),
                       dim3(256), 0, s, jobs, pages, parts, ctr, (uint8_t*)c->value_arena.p, streams, runs, blks, recs);
    // dictionaries past 4096 entries: k_dict4_big (a 104 KiB LDS prefix, one
    // 8-wave workgroup per CU) takes their run-table pages (PQG_DICT_BIG=0: k_dict4)
    hipLaunchKernelGGL(k_dict4, dim3(qgrid(c->num_cus * c->dict4_per_cu)), dim3(c->dict4_threads), 0, s, pages, ctr, Q(3),
                       recs, (int)c->dict_big);
    if (c->dict_big)
      hipLaunchKernelGGL(k_dict4_big, dim3(qgrid(c->num_cus)), dim3(kBigDictThreads), 0, s, pages, ctr,
                         Q(kQueueDictBig), recs);
  } else
    hipLaunchKernelGGL(k_values<1>, dim3(qgrid(waves)), dim3(64), 0, s, jobs, pages, parts, ctr, Q(3),
                       (uint8_t*)c->value_arena.p, streams, runs, blks);
  if (c->any_fixed_other) {
    hipLaunchKernelGGL(k_values<0>, dim3(qgrid(waves)), dim3(64), 0, s, jobs, pages, parts, ctr, Q(2),
                       (uint8_t*)c->value_arena.p, streams, runs, blks);
    hipLaunchKernelGGL(k_values<3>, dim3(qgrid(waves)), dim3(64), 0, s, jobs, pages, parts, ctr, Q(8),
                       (uint8_t*)c->value_arena.p, streams, runs, blks);
  }
  if (c->timed) hipEventRecord(c->ev[8], s);
  if (c->any_var) {
    int64_t* offs = (int64_t*)c->offs_arena.p;
    hipLaunchKernelGGL(k_str_dict, dim3(n), dim3(512), 0, s, jobs, pages, (int64_t*)c->doffs_arena.p);
    hipLaunchKernelGGL(k_str_plain, dim3(qgrid(c->num_cus * 4 * 512 / kPwThreads)), dim3(kPwThreads), 0, s, jobs, pages, list, ctr, Q(5), offs);
    hipLaunchKernelGGL(k_str_count, dim3(qgrid(waves)), dim3(64), 0, s, jobs, pages, parts, ctr, Q(4), offs, streams,
                       runs, blks);
    hipLaunchKernelGGL(k_str_delta, dim3(qgrid(c->num_cus * 8)), dim3(64), 0, s, jobs, pages, list, ctr,
                       Q(kQueueStrDelta), offs);
    hipLaunchKernelGGL(k_char_scan, dim3(n), dim3(256), 0, s, jobs, pages, parts, offs);
    hipLaunchKernelGGL(k_str_copy, dim3(qgrid(c->num_cus * 4)), dim3(512), 0, s, jobs, pages, parts, ctr, Q(6),
                       (uint8_t*)c->value_arena.p, offs);
    hipLaunchKernelGGL(k_str_dba, dim3(qgrid(c->num_cus * 6)), dim3(64), 0, s, jobs, pages, list, ctr,
                       Q(kQueueStrDba), (uint8_t*)c->value_arena.p, offs);
  }
  if (c->timed) hipEventRecord(c->ev[9], s);
  hipLaunchKernelGGL(k_finalize, dim3(n), dim3(1024), 0, s, jobs, n, pages);
  if (c->timed) hipEventRecord(c->ev[10], s);
  return hip_ok(hipGetLastError());
}

int pqg_decode_chunks_async(pqg_ctx* c, const pqg_chunk_job* jobs, int n_jobs) {
  if (!c || (!jobs && n_jobs) || n_jobs < 0) return PQG_ERR_INVALID_ARG;
  hipSetDevice(c->device);
  for (int i = 0; i < n_jobs; i++) {
    const pqg_column_desc& d = jobs[i].col;
    if (d.max_def < 0 || d.max_def > 255 || d.max_rep < 0 || d.max_rep > 255) return PQG_ERR_INVALID_ARG;
    if (jobs[i].data_len < 0 || jobs[i].total_compressed_size < 0 || (!jobs[i].data && jobs[i].data_len > 0))
      return PQG_ERR_INVALID_ARG;
    if (jobs[i].quirks != 0) return PQG_ERR_INVALID_ARG;  // spec-correct only (quirks: oracle triage mode)
  }
  c->cur.assign(jobs, jobs + n_jobs);
  c->n_jobs = n_jobs;
  c->launches = 0;
  c->force.assign((size_t)n_jobs, Caps());
  c->any_var = false;
  c->any_fixed_other = false;
  c->any_w4 = false;
  c->any_levels = false;
  c->prewalk = false;
  for (int i = 0; i < n_jobs; i++) {
    const JobKey key{(uintptr_t)jobs[i].data, jobs[i].total_compressed_size, jobs[i].num_values_hint};
    auto it = c->learned.find(key);
    if (it != c->learned.end()) c->force[(size_t)i] = it->second;
    c->prewalk |= c->many_pages.find(key) == c->many_pages.end();
    // the strings stage: variable-length columns, and FLBA (DELTA_BYTE_ARRAY pages)
    c->any_var |= value_width_of(jobs[i].col) == 0 || jobs[i].col.physical_type == PQG_FIXED_LEN_BYTE_ARRAY;
    // k_values<0>: every fixed-width column but 4-byte ones with only dictionary pages
    c->any_fixed_other |= value_width_of(jobs[i].col) != 0;
    c->any_w4 |= value_width_of(jobs[i].col) == 4;
    c->any_levels |= jobs[i].col.max_def > 0 || jobs[i].col.max_rep > 0;
  }
  if (n_jobs == 0) return PQG_OK;
  int e = plan_batch(c);
  if (e) return e;
  return launch_pipeline(c);
}

// Copy job results back; grow and re-run chunks that ran out of arena space.
int pqg_sync(pqg_ctx* c, pqg_chunk_result* results, int n_jobs) {
  if (!c || n_jobs != c->n_jobs) return PQG_ERR_INVALID_ARG;
  hipSetDevice(c->device);
  const int n = c->n_jobs;
  if (n == 0) return PQG_OK;
  // Every launch is followed by a copy-back and a sync, so the results below
  // never describe a pipeline still in flight; a job still short of space
  // after the last attempt reports PQG_ERR_CAPACITY.
  for (int attempt = 0;; attempt++) {
    if (hipMemcpyAsync(c->h_jobs, c->jobs.p, sizeof(JobDev) * (size_t)n, hipMemcpyDeviceToHost, c->stream) !=
            hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
      return PQG_ERR_HIP;
    bool retry = false;
    for (int i = 0; i < n; i++) {
      const JobDev& d = c->h_jobs[i];
      if (d.status != PQG_ERR_CAPACITY) continue;
      retry = true;
      Caps& f = c->force[(size_t)i];
      f.pages = std::max<int64_t>((int64_t)d.num_pages + 16, d.page_cap);
      f.slots = std::max<int64_t>(d.num_slots + 64, d.slot_cap);
      f.scratch = std::max<int64_t>(d.need_scratch + 1024, d.scratch_cap);
      if (d.value_width > 0) {
        const int64_t nv = std::max<int64_t>(d.num_values, d.num_slots);
        f.values = std::max<int64_t>(nv * d.value_width + 64, d.value_cap);
      } else {
        f.values = std::max<int64_t>(d.values_bytes + 1024, d.value_cap);
      }
      f.runs = std::max<int64_t>(d.run_used + 64, d.run_cap);
      f.blks = std::max<int64_t>(d.blk_used + 64, d.blk_cap);
      f.doffs = std::max<int64_t>(d.need_doffs + 64, d.doffs_cap);
      const pqg_chunk_job& in = c->cur[(size_t)i];
      c->learned[JobKey{(uintptr_t)in.data, in.total_compressed_size, in.num_values_hint}] = f;
    }
    if (!retry || attempt + 1 >= kMaxAttempts) break;
    int e = plan_batch(c);
    if (e) return e;
    e = launch_pipeline(c);
    if (e) return e;
  }
  for (int i = 0; i < n; i++) {
    const JobDev& d = c->h_jobs[i];
    if (d.status != PQG_ERR_CAPACITY && d.scan_fallback != 2) {  // neither walked nor stride-walked by the prewalk
      if (c->many_pages.size() >= 65536) c->many_pages.clear();  // bounded: a cache, not a record
      const pqg_chunk_job& in = c->cur[(size_t)i];
      c->many_pages[JobKey{(uintptr_t)in.data, in.total_compressed_size, in.num_values_hint}] = true;
    }
    pqg_chunk_result& r = results[i];
    memset(&r, 0, sizeof(r));
    r.status = d.status;
    r.error_page = d.error_page;
    r.num_pages = d.status == PQG_ERR_CAPACITY ? 0 : d.n_out_pages;
    r.value_width = d.value_width;
    r.col_flags = c->cur[(size_t)i].col.flags;
    r.num_slots = d.num_slots;
    r.num_values = d.num_values;
    r.values_bytes = d.values_bytes;
    r.def_levels = d.max_def > 0 ? (uint8_t*)c->def_arena.p + d.slot_base : nullptr;
    r.rep_levels = d.max_rep > 0 ? (uint8_t*)c->rep_arena.p + d.slot_base : nullptr;
    r.values = (uint8_t*)c->value_arena.p + d.value_base;
    r.offsets = d.value_width == 0 ? (int64_t*)c->offs_arena.p + d.offs_base : nullptr;
  }
  return PQG_OK;
}

int pqg_assemble(pqg_ctx* c, pqg_assemble_args* a) {
  if (!c || !a || a->num_slots < 0 || a->max_def < 0 || a->max_def > 255 || a->boundary_level < 0)
    return PQG_ERR_INVALID_ARG;
  if (a->values_spaced && (a->value_width <= 0 || (!a->values && a->num_slots > 0))) return PQG_ERR_INVALID_ARG;
  hipSetDevice(c->device);
  const int64_t nseg = (a->num_slots + 4095) / 4096;
  if (c->asm_seg.grow((size_t)(2 * nseg + 2) * sizeof(int64_t))) return PQG_ERR_HIP;
  int64_t* seg = (int64_t*)c->asm_seg.p;
  int64_t* tot = seg + 2 * nseg;
  hipEventRecord(c->ev_k8[0], c->stream);
  int e = pqg::assemble_launch(c->stream, a, seg, tot);
  if (e) return e;
  hipEventRecord(c->ev_k8[1], c->stream);
  int64_t h[2] = {0, 0};
  if (hipMemcpyAsync(h, tot, sizeof(h), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess)
    return PQG_ERR_HIP;
  hipEventElapsedTime(&c->k8_ms, c->ev_k8[0], c->ev_k8[1]);
  a->num_valid = h[0];
  a->null_count = a->num_slots - h[0];
  a->num_boundaries = h[1];
  return PQG_OK;
}

int pqg_assemble_list(pqg_ctx* c, pqg_list_args* a) {
  if (!c || !a || a->num_slots < 0 || !a->def_levels || a->max_def < 0 || a->max_def > 255 || a->value_width < 0)
    return PQG_ERR_INVALID_ARG;
  if (a->elem_values && (a->value_width <= 0 || (!a->values && a->num_slots > 0))) return PQG_ERR_INVALID_ARG;
  hipSetDevice(c->device);
  const int64_t nseg = (a->num_slots + 4095) / 4096;
  if (c->asm_seg.grow((size_t)(4 * nseg + 4) * sizeof(int64_t))) return PQG_ERR_HIP;
  int64_t* seg = (int64_t*)c->asm_seg.p;
  int64_t* tot = seg + 4 * nseg;
  hipEventRecord(c->ev_k8[0], c->stream);
  int e = pqg::list_count_launch(c->stream, a, seg, tot);
  if (e) return e;
  hipEventRecord(c->ev_k8[1], c->stream);
  int64_t h[4] = {0, 0, 0, 0};
  if (hipMemcpyAsync(h, tot, sizeof(h), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess)
    return PQG_ERR_HIP;
  a->num_rows = h[0];
  a->num_elements = h[1];
  a->num_valid = h[2];
  a->null_lists = h[3];
  // int32 offsets cannot hold the elements: fail before any output is written
  if (h[1] > INT32_MAX) return PQG_ERR_INVALID_ARG;
  hipEventRecord(c->ev_k8[2], c->stream);
  e = pqg::list_write_launch(c->stream, a, seg);
  if (e) return e;
  hipEventRecord(c->ev_k8[3], c->stream);
  e = hip_ok(hipStreamSynchronize(c->stream));
  float m0 = 0.f, m1 = 0.f;
  hipEventElapsedTime(&m0, c->ev_k8[0], c->ev_k8[1]);
  hipEventElapsedTime(&m1, c->ev_k8[2], c->ev_k8[3]);
  c->k8_ms = m0 + m1;
  return e;
}

int pqg_last_assemble_ms(pqg_ctx* c, float* ms) {
  if (!c || !ms) return PQG_ERR_INVALID_ARG;
  *ms = c->k8_ms;
  return PQG_OK;
}

int pqg_decode_chunks(pqg_ctx* c, const pqg_chunk_job* jobs, int n_jobs, pqg_chunk_result* results) {
  int e = pqg_decode_chunks_async(c, jobs, n_jobs);
  if (e) return e;
  return pqg_sync(c, results, n_jobs);
}

int pqg_decode_page(pqg_ctx* c, const pqg_page_job* pj, pqg_chunk_result* result) {
  if (!c || !pj || !result || !pj->page || pj->page_len <= 0 || pj->dict_page_len < 0 ||
      (pj->dict_page_len > 0 && !pj->dict_page))
    return PQG_ERR_INVALID_ARG;
  hipSetDevice(c->device);
  const int64_t dl = pj->dict_page ? pj->dict_page_len : 0, total = dl + pj->page_len;
  // the page (after its dictionary) as a one-page column chunk
  if (c->page_stage.grow((size_t)total + 64)) return PQG_ERR_HIP;
  uint8_t* st = (uint8_t*)c->page_stage.p;
  if ((dl && hipMemcpyAsync(st, pj->dict_page, (size_t)dl, hipMemcpyDeviceToDevice, c->stream) != hipSuccess) ||
      hipMemcpyAsync(st + dl, pj->page, (size_t)pj->page_len, hipMemcpyDeviceToDevice, c->stream) != hipSuccess)
    return PQG_ERR_HIP;
  pqg_chunk_job job;
  memset(&job, 0, sizeof(job));
  job.col = pj->col;
  job.data = st;
  job.data_len = total;
  job.total_compressed_size = total;
  job.data_page_offset = dl;
  job.total_uncompressed_size = total;
  return pqg_decode_chunks(c, &job, 1, result);
}

// gzipCompressor.DecompressBlock (compress.go:63-76): gzip.NewReader +
// ioutil.ReadAll.  The decoded length is not in the block, so k_inflate decodes
// it as a bare block (kPageBareBlock): bytes past the device buffer's `store`
// are counted and CRC'd but not stored, and the count comes back in
// PageDev.gz_len.  The first pass stores at most kInflateFirst bytes; a block
// that decodes to more (and fits `cap`) is decoded again into a buffer of its
// size, so the device buffer never grows to `cap` before the length is known,
// and no byte past what k_inflate stored is ever copied out.
static int inflate_pass(pqg_ctx* c, int64_t n, int64_t store, PageDev* out) {
  if (c->blk_dst.grow((size_t)store + 64)) return PQG_ERR_HIP;
  JobDev jd;
  memset(&jd, 0, sizeof(jd));
  jd.data = (const uint8_t*)c->blk_src.p;
  jd.data_len = n;
  jd.tcs = n;
  jd.codec = PQG_CODEC_GZIP;
  jd.scratch_cap = store + 16;
  PageDev pd;
  memset(&pd, 0, sizeof(pd));
  pd.page_type = PQG_PAGE_DICTIONARY;  // no values-decoder check after the block
  pd.flags = kPageBareBlock;
  pd.csize = (int32_t)n;
  pd.usize = (int32_t)store;
  pd.read_status = kOK;
  uint8_t* meta = (uint8_t*)c->blk_meta.p;
  JobDev* djob = (JobDev*)meta;
  PageDev* dpage = (PageDev*)(meta + sizeof(JobDev));
  int* ints = (int*)(meta + sizeof(JobDev) + sizeof(PageDev));  // [0] list, [1] total, then the queue
  int hi[2] = {0, 1};
  if (hipMemcpyAsync(djob, &jd, sizeof(jd), hipMemcpyHostToDevice, c->stream) != hipSuccess ||
      hipMemcpyAsync(dpage, &pd, sizeof(pd), hipMemcpyHostToDevice, c->stream) != hipSuccess ||
      hipMemcpyAsync(ints, hi, sizeof(hi), hipMemcpyHostToDevice, c->stream) != hipSuccess ||
      hipMemsetAsync(ints + 4, 0, sizeof(int) * kQueueInts, c->stream) != hipSuccess)
    return PQG_ERR_HIP;
  hipLaunchKernelGGL(k_inflate, dim3(qgrid(1)), dim3(64), 0, c->stream, djob, dpage, ints, ints + 1, ints + 4,
                     (uint8_t*)c->blk_dst.p, 0);
  if (hipGetLastError() != hipSuccess) return PQG_ERR_HIP;
  if (hipMemcpyAsync(out, dpage, sizeof(PageDev), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess)
    return PQG_ERR_HIP;
  return PQG_OK;
}

static int block_inflate(pqg_ctx* c, const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap, int64_t* out_len) {
  constexpr int64_t kInflateFirst = 64 << 20;
  hipSetDevice(c->device);
  if (c->blk_src.grow((size_t)n + 64) ||
      c->blk_meta.grow(sizeof(JobDev) + sizeof(PageDev) + (4 + 2 * kQueueInts) * sizeof(int)))
    return PQG_ERR_HIP;
  if (n && hipMemcpyAsync(c->blk_src.p, src, (size_t)n, hipMemcpyHostToDevice, c->stream) != hipSuccess)
    return PQG_ERR_HIP;
  int64_t store = std::min<int64_t>(std::max<int64_t>(cap, 0), kInflateFirst);
  PageDev pd;
  int e = inflate_pass(c, n, store, &pd);
  if (e) return e;
  if (pd.read_status != kOK) return pd.read_status;
  *out_len = pd.gz_len;
  if (pd.gz_len > cap) return PQG_ERR_CAPACITY;
  if (pd.gz_len > INT32_MAX) return PQG_ERR_UNSUPPORTED;  // one block of >= 2 GiB: the kernel's 32-bit offsets
  if (pd.gz_len > store) {  // decoded length known now: again, storing all of it
    store = pd.gz_len;
    e = inflate_pass(c, n, store, &pd);
    if (e) return e;
    if (pd.read_status != kOK) return pd.read_status;
    if (pd.gz_len != store) return PQG_ERR_HIP;  // the same bytes decode to the same length
  }
  if (pd.gz_len && (hipMemcpyAsync(dst, c->blk_dst.p, (size_t)pd.gz_len, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
                    hipStreamSynchronize(c->stream) != hipSuccess))
    return PQG_ERR_HIP;
  return PQG_OK;
}

int pqg_block_decompress(pqg_ctx* c, int codec, const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap,
                         int64_t* out_len) {
  if (!c || (!src && n > 0) || n < 0 || n > INT32_MAX || !out_len) return PQG_ERR_INVALID_ARG;
  *out_len = 0;
  if (codec == PQG_CODEC_UNCOMPRESSED) {
    *out_len = n;
    if (n > cap) return PQG_ERR_CAPACITY;
    if (n) memcpy(dst, src, (size_t)n);
    return PQG_OK;
  }
  if (codec == PQG_CODEC_GZIP) return block_inflate(c, src, n, dst, cap, out_len);
  if (codec != PQG_CODEC_SNAPPY) return PQG_ERR_UNSUPPORTED;
  // decodedLen (decode.go:32-43): the varint header, on the host to size the output
  uint64_t v = 0;
  int hl = 0;
  for (unsigned sft = 0;; hl++, sft += 7) {
    if (hl >= n) return PQG_ERR_SNAPPY;
    const uint8_t b = src[hl];
    if (b < 0x80) {
      if (hl > 9 || (hl == 9 && b > 1)) return PQG_ERR_SNAPPY;
      v |= sft < 64 ? (uint64_t)b << sft : 0;
      hl++;
      break;
    }
    if (sft < 64) v |= (uint64_t)(b & 0x7f) << sft;
  }
  if (v > 0xffffffffull || v > (uint64_t)INT32_MAX) return PQG_ERR_SNAPPY;
  *out_len = (int64_t)v;
  if ((int64_t)v > cap) return PQG_ERR_CAPACITY;
  hipSetDevice(c->device);
  // one block = one page of a one-job batch: k_snappy decodes it into scratch
  if (c->blk_src.grow((size_t)n + 64) || c->blk_dst.grow((size_t)v + 64) ||
      c->blk_meta.grow(sizeof(JobDev) + sizeof(PageDev) + (4 + 2 * kQueueInts) * sizeof(int)))
    return PQG_ERR_HIP;
  const int64_t bsub = (int64_t)v / kSnapSub + 2, bseg = n / kSnapSeg + 2;
  if (c->blk_subs.grow(sizeof(SnapSub) * (size_t)bsub) || c->blk_segpage.grow(sizeof(int) * (size_t)bseg) ||
      c->blk_F.grow(sizeof(uint2) * 64 * (size_t)bseg))
    return PQG_ERR_HIP;
  JobDev jd;
  memset(&jd, 0, sizeof(jd));
  jd.data = (const uint8_t*)c->blk_src.p;
  jd.data_len = n;
  jd.tcs = n;
  jd.codec = PQG_CODEC_SNAPPY;
  jd.scratch_cap = (int64_t)v + 16;
  PageDev pd;
  memset(&pd, 0, sizeof(pd));
  pd.page_type = PQG_PAGE_DICTIONARY;  // a bare block: no values-decoder check after it
  pd.csize = (int32_t)n;
  pd.usize = (int32_t)v;
  pd.payload_offset = 0;
  pd.scratch_offset = 0;
  pd.read_status = kOK;
  uint8_t* meta = (uint8_t*)c->blk_meta.p;
  JobDev* djob = (JobDev*)meta;
  PageDev* dpage = (PageDev*)(meta + sizeof(JobDev));
  // ints: [0] list, [1] total, [2..3] split counters, then the two sharded queues
  int* ints = (int*)(meta + sizeof(JobDev) + sizeof(PageDev));
  int hi[2] = {0, 1};
  if (hipMemcpyAsync(c->blk_src.p, src, (size_t)n, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
      hipMemcpyAsync(djob, &jd, sizeof(jd), hipMemcpyHostToDevice, c->stream) != hipSuccess ||
      hipMemcpyAsync(dpage, &pd, sizeof(pd), hipMemcpyHostToDevice, c->stream) != hipSuccess ||
      hipMemcpyAsync(ints, hi, sizeof(hi), hipMemcpyHostToDevice, c->stream) != hipSuccess ||
      hipMemsetAsync(ints + 4, 0, sizeof(int) * 2 * kQueueInts, c->stream) != hipSuccess)
    return PQG_ERR_HIP;
  // the page decode's own snappy stage, on a one-page list
  const SnapTables T{(SnapSub*)c->blk_subs.p, (int)bsub, (int*)c->blk_segpage.p, (int)bseg, (uint2*)c->blk_F.p};
  launch_snappy(c, c->stream, djob, dpage, ints, ints + 1, 1, ints + 2, ints + 4, ints + 4 + kQueueInts,
                (uint8_t*)c->blk_dst.p, T);
  if (hipGetLastError() != hipSuccess) return PQG_ERR_HIP;
  if (hipMemcpyAsync(&pd, dpage, sizeof(pd), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess)
    return PQG_ERR_HIP;
  if (pd.read_status != kOK) return pd.read_status;
  if (v && (hipMemcpyAsync(dst, c->blk_dst.p, (size_t)v, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
            hipStreamSynchronize(c->stream) != hipSuccess))
    return PQG_ERR_HIP;
  return PQG_OK;
}

int pqg_pack_levels(pqg_ctx* c, const uint8_t* levels, int64_t n, int max_level, uint8_t* packed) {
  if (!c || n < 0 || max_level < 0 || max_level > 255 || (n > 0 && (!levels || !packed))) return PQG_ERR_INVALID_ARG;
  hipSetDevice(c->device);
  int bw = 0;
  while ((max_level >> bw) != 0) bw++;  // bits.Len16(maxLevel)
  int e = pqg::pack_levels_launch(c->stream, levels, n, bw, packed);
  if (e) return e;
  return hip_ok(hipStreamSynchronize(c->stream));
}

int pqg_get_pages(pqg_ctx* c, int job, pqg_page_info* out, int cap) {
  if (!c || job < 0 || job >= c->n_jobs) return PQG_ERR_INVALID_ARG;
  hipSetDevice(c->device);
  const JobDev& d = c->h_jobs[job];
  int np = std::min<int>(d.n_out_pages, d.page_cap);
  if (d.status == PQG_ERR_CAPACITY) np = 0;
  std::vector<PageDev> tmp((size_t)np);
  if (np > 0) {
    if (hipMemcpyAsync(tmp.data(), (PageDev*)c->pages.p + d.page_base, sizeof(PageDev) * (size_t)np,
                       hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
      return PQG_ERR_HIP;
  }
  int k = 0;
  for (int i = 0; i < np && i < cap; i++, k++) {
    const PageDev& p = tmp[(size_t)i];
    pqg_page_info& o = out[i];
    memset(&o, 0, sizeof(o));
    o.header_offset = p.header_offset;
    o.payload_offset = p.payload_offset;
    o.slot_offset = p.slot_offset;
    o.value_offset = p.value_offset;
    o.page_type = p.page_type;
    o.encoding = p.encoding;
    o.num_values = p.num_values;
    o.not_null = p.not_null;
    o.compressed_size = p.csize;
    o.uncompressed_size = p.usize;
    o.def_len = p.def_len;
    o.rep_len = p.rep_len;
    o.def_encoding = p.def_enc;
    o.rep_encoding = p.rep_enc;
    o.status = p.read_status != PQG_OK ? p.read_status : p.decode_status;
    // bits 8+: why the split snappy decode gave the page up (diagnostics, pqg_snappy.hip)
    o.flags = p.flags | (p.sn_fallback ? PQG_PAGE_FLAG_SNAPPY_SERIAL | (p.sn_fallback << 8) : 0);
  }
  return k;
}

// Diagnostic builds (-DPQG_PROFILE): in-kernel phase cycle counters of the
// values (slots 0-31), levels (slots 32-63), strings (64-95), snappy
// (96-127) and dictionary (128-159) translation units; read + reset.
int pqg_debug_counters(pqg_ctx* c, uint64_t* out, int cap) {
  if (!c || !out) return PQG_ERR_INVALID_ARG;
#ifdef PQG_PROFILE
  hipSetDevice(c->device);
  hipStreamSynchronize(c->stream);
  unsigned long long a[64], b[64], c3[64], d4[64], e5[64], f6[64];
  if (pqg::prof_read_values(a) || pqg::prof_read_levels(b) || pqg::prof_read_strings(c3) ||
      pqg::prof_read_snappy(d4) || pqg::prof_read_dict(e5) || pqg::prof_read_inflate(f6))
    return PQG_ERR_HIP;
  int k = 0;
  for (; k < 192 && k < cap; k++)
    out[k] = k < 32    ? a[k]
             : k < 64  ? b[k - 32]
             : k < 96  ? c3[k - 64]
             : k < 128 ? d4[k - 96]
             : k < 160 ? e5[k - 128]
                       : f6[k - 160];
  return k;
#else
  return 0;
#endif
}

int pqg_debug_job(pqg_ctx* c, int job, int64_t* out, int cap) {
  if (!c || !out || job < 0 || job >= c->n_jobs) return PQG_ERR_INVALID_ARG;
  const JobDev& d = c->h_jobs[job];
  const int64_t v[5] = {d.scan_fallback, d.n_cands, d.num_pages, d.need_scratch, c->launches};
  int k = 0;
  for (; k < 5 && k < cap; k++) out[k] = v[k];
  return k;
}

int pqg_set_timing(pqg_ctx* c, int on) {
  if (!c) return PQG_ERR_INVALID_ARG;
  c->timed = on != 0;
  return PQG_OK;
}

int pqg_last_timings(pqg_ctx* c, float* out, int cap) {
  if (!c || !out) return PQG_ERR_INVALID_ARG;
  if (!c->last_timed) return 0;  // the last decode recorded no events: nothing to report
  int k = 0;
  float tot = 0;
  hipEventElapsedTime(&tot, c->ev[0], c->ev[kStages]);
  if (k < cap) out[k++] = tot;
  for (int i = 0; i < kStages && k < cap; i++) {
    float ms = 0;
    hipEventElapsedTime(&ms, c->ev[i], c->ev[i + 1]);
    out[k++] = ms;
  }
  return k;
}

int pqg_bench_decode(pqg_ctx* c, const pqg_chunk_job* jobs, int n_jobs, int iters, float* ms_total, float* ms_stage,
                     int stage_cap) {
  if (!c || iters < 1) return PQG_ERR_INVALID_ARG;
  hipSetDevice(c->device);
  std::vector<pqg_chunk_result> res((size_t)std::max(n_jobs, 1));
  // first call sizes the arenas (and retries on capacity)
  int e = pqg_decode_chunks(c, jobs, n_jobs, res.data());
  if (e) return e;
  // the first call grew the arenas; its capacities are the learned ones now
  for (int i = 0; i < n_jobs; i++) {
    Caps& f = c->force[(size_t)i];
    const JobDev& d = c->h_jobs[i];
    f.pages = d.page_cap;
    f.slots = d.slot_cap;
    f.scratch = d.scratch_cap;
    f.values = d.value_cap;
    f.runs = d.run_cap;
    f.blks = d.blk_cap;
    f.doffs = d.doffs_cap;
  }
  e = plan_batch(c);
  if (e) return e;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  std::vector<float> stage_acc(kStages, 0.f);
  hipEventRecord(a, c->stream);
  for (int it = 0; it < iters; it++) {
    e = launch_pipeline(c);
    if (e) break;
  }
  hipEventRecord(b, c->stream);
  hipStreamSynchronize(c->stream);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  if (ms_total) *ms_total = ms / (float)iters;
  if (ms_stage) {
    for (int i = 0; i < kStages && i < stage_cap; i++) {
      float x = 0;
      hipEventElapsedTime(&x, c->ev[i], c->ev[i + 1]);
      ms_stage[i] = x;
    }
  }
  hipEventDestroy(a);
  hipEventDestroy(b);
  return e;
}

}  // extern "C"
