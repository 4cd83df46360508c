// pqg_levels.hip — K3: page streams, the RLE/bit-packed hybrid run walk and
// the level expansion.
//
//   K3a k_page_setup     one lane per page: the read phase of the level
//                        streams (V1 initSize: page_v1.go:99-105,
//                        hybrid_decoder.go:57-67; V2 raw level bytes:
//                        page_v2.go:103-121) and registration of every hybrid
//                        stream of the page (levels, dictionary indices
//                        type_dict.go:22-37, RLE booleans type_boolean.go:100-120)
//   K3b k_hybrid_walk    one LANE per hybrid stream: the serial run-header walk
//                        of hybridDecoder.next (hybrid_decoder.go:82-166) writes
//                        a run table and a block index.  The walk is the only
//                        serial part of the format; giving each lane its own
//                        stream keeps all 64 lanes busy on it.
//   K3c k_levels_expand  one wave per page: rep then def levels, 8 values per
//                        lane per 512-value block, notNull = #(def == maxD)
//                        (decodePackedArray helpers.go:131-147)
//   K3d k_nn_scan        per chunk: value offsets = exclusive scan of notNull
//                        (readPageData chunk_reader.go:380-402) and the
//                        dictionary page (page_dict.go:30-64)
#include <hip/hip_runtime.h>

#include "pqg_common.h"
#include "pqg_device.h"
#include "pqg_hybrid.h"

namespace pqg {

#ifdef PQG_PROFILE
// host reader of this translation unit's phase counters (see pqg_debug_counters)
int prof_read_levels(unsigned long long* out) {
  unsigned long long z[64] = {0};
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pqg_prof), sizeof(z)) != hipSuccess) return -1;
  hipMemcpyToSymbol(HIP_SYMBOL(pqg_prof), z, sizeof(z));
  return 0;
}
#endif

// ---- K3a ---------------------------------------------------------------------
__device__ __forceinline__ int reg_stream(JobDev& job, HStream* streams, int32_t* slot, int pidx, int kind,
                                          gcu8 p, int64_t n, int w, int64_t count) {
  const int64_t nruns = n / 2 + 2;  // every run but a truncated last one takes >= 2 bytes
  // blocks close at kHBlock values, kHBlockRuns runs or kHBlockBytes payload bytes
  const int64_t nblks = count / kHBlock + nruns / kHBlockRuns + n / (kHBlockBytes / 2) + 3;
  const int64_t rb = (int64_t)atomicAdd((unsigned long long*)&job.run_used, (unsigned long long)nruns);
  const int64_t bb = (int64_t)atomicAdd((unsigned long long*)&job.blk_used, (unsigned long long)nblks);
  if (rb + nruns > job.run_cap || bb + nblks > job.blk_cap) {
    job.status = kCAPACITY;  // the host grows the run arenas and decodes again
    return -1;
  }
  const int id = pidx * 3 + (kind > 2 ? 2 : kind);
  HStream& S = streams[id];
  S.p = (const uint8_t*)p;
  S.n = n;
  S.run_base = job.run_base + rb;
  S.blk_base = job.blk_base + bb;
  S.page = pidx;
  S.kind = kind;
  S.w = w;
  S.count = (int32_t)count;
  S.n_runs = 0;
  S.produced = 0;
  S.status = kOK;
  S.n_blocks = 0;
  *slot = id;
  return id;
}

__global__ void __launch_bounds__(256) k_page_setup(JobDev* jobs, PageDev* pages, const int* list, const int* total,
                                                    uint8_t* scratch, HStream* streams, int* vlists, int* vcount,
                                                    int list_cap) {
  const int nt = *total;
  for (int t = blockIdx.x * 256 + threadIdx.x; t < nt; t += gridDim.x * 256) {
    const int pidx = list[t];
    PageDev& pg = pages[pidx];
    pg.hs_rep = pg.hs_def = pg.hs_val = -1;
    if (pg.read_status != kOK || (pg.page_type != 0 && pg.page_type != 3)) continue;
    JobDev& job = jobs[pg.job];
    if (job.status == kCAPACITY) continue;
    // ---- the page block and its level / value streams (read phase)
    gcu8 block;
    int64_t blen;
    int32_t levels = 0;
    if (pg.page_type == 3) {
      levels = (int32_t)((uint32_t)pg.rep_len + (uint32_t)pg.def_len);
      blen = (int32_t)((uint32_t)pg.csize - (uint32_t)levels);
      if (pg.scratch_offset >= 0) blen = (int32_t)((uint32_t)pg.usize - (uint32_t)levels);
    } else {
      blen = pg.scratch_offset >= 0 ? pg.usize : pg.csize;
    }
    if (pg.scratch_offset >= 0) block = gconst(scratch) + job.scratch_base + pg.scratch_offset;
    else block = gconst(job.data) + pg.payload_offset + (levels > 0 ? levels : 0);
    gcu8 rep = nullptr, def = nullptr;
    int64_t rep_n = -1, def_n = -1;  // -1: the level decoder is not initialised
    int64_t vpos = 0;
    int e = kOK;
    if (pg.page_type == 0) {
      // rDecoder.initSize then dDecoder.initSize (page_v1.go:99-105)
      if (job.max_rep > 0) {
        if (blen - vpos < 4) e = kEOF;
        else {
          const int64_t sz = rd_u32(block + vpos);
          const int64_t take = min(sz, blen - vpos - 4);
          rep = block + vpos + 4;
          rep_n = take;
          vpos += 4 + take;
        }
      }
      if (e == kOK && job.max_def > 0) {
        if (blen - vpos < 4) e = kEOF;
        else {
          const int64_t sz = rd_u32(block + vpos);
          const int64_t take = min(sz, blen - vpos - 4);
          def = block + vpos + 4;
          def_n = take;
          vpos += 4 + take;
        }
      }
    } else {
      // V2: raw level bytes, a decoder only for a non-empty section (page_v2.go:110-120)
      gcu8 lv = gconst(job.data) + pg.payload_offset;
      if (levels > 0 && pg.rep_len > 0) { rep = lv; rep_n = pg.rep_len; }
      if (levels > 0 && pg.def_len > 0) { def = lv + pg.rep_len; def_n = levels - pg.rep_len; }
    }
    if (e != kOK) {
      pg.read_status = e;
      continue;
    }
    pg.block = (const uint8_t*)block;
    pg.block_len = blen;
    pg.val = (const uint8_t*)(block + vpos);
    pg.val_n = blen - vpos;
    pg.rep = (const uint8_t*)rep;
    pg.rep_n = rep_n;
    pg.def = (const uint8_t*)def;
    pg.def_n = def_n;
    const int64_t n = pg.num_values;
    if (n > 0) {
      if (job.max_rep > 0 && rep_n >= 0)
        reg_stream(job, streams, &pg.hs_rep, pidx, 0, rep, rep_n, bits_len((uint32_t)job.max_rep), n);
      if (job.max_def > 0 && def_n >= 0)
        reg_stream(job, streams, &pg.hs_def, pidx, 1, def, def_n, bits_len((uint32_t)job.max_def), n);
    }
    // values: RLE_DICTIONARY indices (first byte = bit width) / RLE booleans (u32 length)
    const int64_t vn = blen - vpos;
    gcu8 val = block + vpos;
    if (pg.encoding == 8 && vn >= 1) {
      const int w = val[0];
      pg.dict_width = w;
      if (w >= 1 && w <= 32 && n > 0) reg_stream(job, streams, &pg.hs_val, pidx, 2, val + 1, vn - 1, w, n);
    } else if (pg.encoding == 3 && job.type == 0 && vn >= 4) {
      const int64_t sz = rd_u32(val);
      const int64_t take = min(sz, vn - 4);
      if (n > 0) reg_stream(job, streams, &pg.hs_val, pidx, 3, val + 4, take, 1, n);
    }
    // value-stage page lists: 4-byte dictionary pages (the hot path, a kernel
    // of its own), variable-length values (pqg_strings.hip) and everything else
    const int mode = job.value_width == 0 ? 2 : (pg.encoding == 8 && job.value_width == 4) ? 1 : 0;
    vlists[mode * list_cap + atomicAdd(&vcount[mode], 1)] = pidx;
  }
}

// ---- K3b ---------------------------------------------------------------------
// One lane walks one stream.  The lane's window on its stream: 64-byte chunks
// (16-byte aligned in memory); the chunk holding `pos` and the next one sit in
// two LDS slots and the one after is prefetched into registers, so the walk
// waits on global memory about once per 64 bytes, for a load issued a chunk
// earlier.  Positions are 32-bit (a page is < 2 GiB: its sizes are thrift
// i32); the per-run path is kept short because a single wave per SIMD walks
// it with nothing to hide its latency behind.
constexpr int kWalkThreads = 256;

struct LaneRing {
  gcu8 base;       // 16-byte aligned address at or below the stream start
  uint32_t n;      // stream bytes
  uint32_t d0;     // stream byte 0 is byte d0 of chunk 0
  uint32_t cur;    // chunk of the current position (slots hold cur, cur+1)
  PQG_L uint32_t* lds;  // dword k of slot s at lds[(16 s + k) * kWalkThreads]

  // Load chunk c into its slot.  No prefetch is carried in registers across
  // iterations: a loop-carried register holding an in-flight load makes the
  // compiler wait for it (vmcnt(0)) at every iteration's latch, and that wait
  // also covers the run-table store just issued.
  __device__ __forceinline__ void load(uint32_t c) {
    uint4 r[4];
#pragma unroll
    for (int g = 0; g < 4; g++) {
      // granule [c*64 + 16g - d0, +16): mapped when it holds a stream byte < n
      const int64_t s0 = (int64_t)c * 64 + 16 * g - d0;
      r[g] = (s0 < (int64_t)n && s0 + 16 > 0) ? ldg16((uintptr_t)(base + (size_t)c * 64 + 16 * g))
                                               : make_uint4(0, 0, 0, 0);
    }
    PQG_L uint32_t* b = lds + (c & 1) * 16 * kWalkThreads;
#pragma unroll
    for (int g = 0; g < 4; g++) {
      b[(4 * g + 0) * kWalkThreads] = r[g].x;
      b[(4 * g + 1) * kWalkThreads] = r[g].y;
      b[(4 * g + 2) * kWalkThreads] = r[g].z;
      b[(4 * g + 3) * kWalkThreads] = r[g].w;
    }
  }
  __device__ __forceinline__ void move_to(uint32_t c) {
    if (c != cur + 1) load(c);  // a jump: both chunks are new
    load(c + 1);
    cur = c;
  }
  __device__ __forceinline__ void init(const uint8_t* p, uint32_t n_, PQG_L uint32_t* lds_) {
    d0 = (uint32_t)((uintptr_t)p & 15);
    base = gconst(p) - d0;
    n = n_;
    lds = lds_;
    cur = 0xfffffff0u;
    move_to(0);
  }
  // 8 bytes at stream position pos (< n; bytes past n are garbage)
  __device__ __forceinline__ uint64_t peek8(uint32_t pos) {
    const uint32_t off = pos + d0;
    const uint32_t c = off >> 6;
    if (c != cur) move_to(c);
    const uint32_t k0 = ((c & 1) << 4) | ((off >> 2) & 15);
    const uint32_t a = lds[k0 * kWalkThreads], b = lds[((k0 + 1) & 31) * kWalkThreads],
                   cc = lds[((k0 + 2) & 31) * kWalkThreads];
    const uint32_t sh = (off & 3) * 8;
    const uint32_t lo = __builtin_amdgcn_alignbit(b, a, sh), hi = __builtin_amdgcn_alignbit(cc, b, sh);
    return (uint64_t)lo | (uint64_t)hi << 32;
  }
};

// Lanes [0, total) walk the rep streams, [total, 2 total) the def streams,
// [2 total, 3 total) the value streams, so a wave's lanes do alike work.
__global__ void __launch_bounds__(kWalkThreads) k_hybrid_walk(const PageDev* pages, const int* list, const int* total,
                                                              HStream* streams, RunEnt* runs, BlockDesc* blks) {
  __shared__ uint32_t buf[32 * kWalkThreads];  // two 64-byte chunks per lane
  const int nt = *total;
  for (int g = blockIdx.x * kWalkThreads + threadIdx.x; g < 3 * nt; g += gridDim.x * kWalkThreads) {
    const int kind = g / nt;
    const PageDev& pg = pages[list[g - kind * nt]];
    const int hs = kind == 0 ? pg.hs_rep : kind == 1 ? pg.hs_def : pg.hs_val;
    if (hs < 0) continue;
    HStream& S = streams[hs];
    const uint32_t w = (uint32_t)S.w;
    const uint32_t n = (uint32_t)S.n, count = (uint32_t)S.count;
    const uint32_t rb = (w + 7) >> 3;
    const uint64_t vmask = rb >= 4 ? 0xffffffffull : ((1ull << (8 * rb)) - 1);
    PQG_G uint32_t* R = (PQG_G uint32_t*)(gmut(runs) + S.run_base);
    PQG_G uint32_t* B = (PQG_G uint32_t*)(gmut(blks) + S.blk_base);
    LaneRing rd;
    rd.init(S.p, n, lds_ptr(buf) + threadIdx.x);
    uint32_t pos = 0, produced = 0, nr = 0;
    int status = kOK;
    // block under construction (see BlockDesc)
    uint32_t nb = 0, bv0 = 0, br0 = 0, bn = 0;
    uint64_t blo = ~0ull, bhi = 0;
    auto close_block = [&]() {
      if (bn == 0) return;
      const uint32_t lo = blo == ~0ull ? 0u : (uint32_t)blo;
      const uint32_t nbytes = blo == ~0ull ? 0u : (uint32_t)(bhi - blo);
      PQG_G uint32_t* d = B + 4 * nb;
      stg16((uintptr_t)d, make_uint4(bv0, br0, lo, (nbytes & 0xffff) | (bn << 16)));
      nb++;
    };
    while (produced < count) {
      // hybridDecoder.next: run header = readUVariant32 (helpers.go:149-165)
      if (pos >= n) { status = kEOF; break; }
      uint64_t x = rd.peek8(pos);
      uint32_t h, hl;
      if ((x & 0x80) == 0) {
        h = (uint32_t)x & 0x7f;
        hl = 1;
      } else {  // multi-byte header: exactly binary.ReadUvarint + the MaxInt32 check
        uint64_t v = 0;
        unsigned sft = 0;
        int e = kOK;
        hl = 0;
        for (uint32_t i = 0;; i++) {
          if (pos + i >= n) { e = kEOF; break; }
          const uint32_t b = i < 8 ? (uint32_t)(x >> (8 * i)) & 0xff : (uint32_t)rd.peek8(pos + i) & 0xff;
          if (b < 0x80) {
            if (i > 9 || (i == 9 && b > 1)) e = kRLE;  // overflows uint64
            else {
              v |= sft < 64 ? (uint64_t)b << sft : 0;
              if (v > 0x7fffffffull) e = kRLE;  // > MaxInt32
            }
            hl = i + 1;
            break;
          }
          if (sft < 64) v |= (uint64_t)(b & 0x7f) << sft;
          sft += 7;
        }
        if (e) { status = e; break; }
        h = (uint32_t)v;
        x = rd.peek8(pos + hl) << 8;  // the RLE value at byte 1, like the fast path
      }
      pos += hl;
      uint32_t take, st, src;
      const uint32_t left = count - produced;
      if (h & 1) {  // bit-packed: h>>1 groups of 8 values, w bytes each
        const uint32_t groups = h >> 1;
        if (groups == 0) { status = kRLE; break; }  // "empty bit-packed run"
        take = groups >= (left + 7) >> 3 ? left : groups * 8;
        const uint32_t need = (take + 7) >> 3;
        // every group read must start inside the stream; a short one is zero padded (Q5)
        if ((uint64_t)pos + (uint64_t)(need - 1) * w >= n) {
          const uint32_t ok = pos < n ? (n - pos + w - 1) / w : 0;
          take = ok * 8;
          status = kEOF;
        }
        st = produced | kRunBP;
        src = pos;
        pos = (uint64_t)pos + (uint64_t)groups * w > 0xffffffffull ? 0xffffffffu : pos + groups * w;
      } else {  // RLE: h>>1 repeats of a ceil(w/8)-byte little-endian value
        const uint32_t cnt = h >> 1;
        if (cnt == 0) { status = kRLE; break; }
        if (pos >= n || n - pos < rb) { status = kEOF; break; }
        src = (uint32_t)((x >> 8) & vmask);
        pos += rb;
        if (w < 32 && (src >> w) != 0) { status = kRLE; break; }  // readRLERunValue :127-129
        take = cnt < left ? cnt : left;
        st = produced;
      }
      if (take > 0) {
        stg8((uintptr_t)(R + 2 * nr), st, src);
        // the run joins the open block, and every block it reaches into
        const uint32_t rend = produced + take;
        for (uint32_t v = produced; v < rend;) {
          if (bn == kHBlockRuns || v >= bv0 + kHBlock) {
            close_block();
            bv0 = v;
            br0 = nr;
            bn = 0;
            blo = ~0ull;
            bhi = 0;
          }
          uint32_t pe = rend < bv0 + kHBlock ? rend : bv0 + kHBlock;
          if (st & kRunBP) {
            const uint64_t rbit = (uint64_t)src * 8;  // bit of the run's value 0
            const uint64_t b0 = (rbit + (uint64_t)(v - produced) * w) >> 3;
            const uint64_t org = blo < b0 ? blo : b0;
            // values whose bits end within org + kHBlockBytes
            const uint64_t lim = (org + kHBlockBytes) * 8;
            const uint64_t fit = lim > rbit ? (lim - rbit) / w : 0;  // values [0, fit) of the run fit
            if (produced + fit <= v) {  // not even one more value: start a new block here
              close_block();
              bv0 = v;
              br0 = nr;
              bn = 0;
              blo = ~0ull;
              bhi = 0;
              continue;
            }
            if (produced + fit < pe) pe = (uint32_t)(produced + fit);
            const uint64_t b1 = (rbit + (uint64_t)(pe - produced) * w + 7) >> 3;
            blo = org;
            bhi = b1 > bhi ? b1 : bhi;
          }
          bn++;
          v = pe;
        }
        produced = rend;
        nr++;
      }
      if (status) break;
    }
    close_block();
    S.n_runs = (int32_t)nr;
    S.produced = (int32_t)produced;
    S.status = status;
    S.n_blocks = (int32_t)nb;
  }
}

// ---- K3c ---------------------------------------------------------------------
struct LevelSink {
  gu8 out;
  uint32_t maxl;
  int64_t nn;
  __device__ __forceinline__ void group(const uint32_t (&v)[kGroup][8], const uint32_t (&i0)[kGroup],
                                        const int (&cnt)[kGroup]) {
#pragma unroll
    for (int b = 0; b < kGroup; b++) {
      if (cnt[b] == 0) continue;
      gu8 o = out + i0[b];
      if (cnt[b] == 8 && ((uintptr_t)o & 7) == 0) {
        stg8((uintptr_t)o, v[b][0] | v[b][1] << 8 | v[b][2] << 16 | v[b][3] << 24,
             v[b][4] | v[b][5] << 8 | v[b][6] << 16 | v[b][7] << 24);
      } else {
        for (int q = 0; q < cnt[b]; q++) o[q] = (uint8_t)v[b][q];
      }
      for (int q = 0; q < cnt[b]; q++) nn += v[b][q] == maxl;
    }
  }
};

__global__ void __launch_bounds__(64) k_levels_expand(JobDev* jobs, PageDev* pages, const int* list,
                                                      const int* total, int* queue, const HStream* streams,
                                                      const RunEnt* runs, const BlockDesc* blks, uint8_t* def_arena,
                                                      uint8_t* rep_arena) {
  __shared__ __attribute__((aligned(16))) ExpandShared sh;
  const int lane = lane_id();
  for (;;) {
    const int t = queue_next(queue);
    if (t >= *total) return;
    // wave-uniform index: the page / job / stream records below are read once
    // with scalar loads into locals; read through references, every output
    // store (which might alias them) would force a re-load and a vmcnt wait
    const int pidx = __builtin_amdgcn_readfirstlane(list[t]);
    const PageDev pg = pages[pidx];
    if (pg.read_status != kOK || (pg.page_type != 0 && pg.page_type != 3)) continue;
    const JobDev job = jobs[pg.job];
    if (job.status == kCAPACITY) continue;
    // readValues (page_v1.go:27-55): rep levels, then def levels, then values
    const int64_t n = pg.num_values;
    int64_t nn = 0;
    int de = kOK;
    if (n > 0) {
      if (job.max_rep > 0) {
        if (pg.rep_n < 0) {
          de = kLEVELS;  // V2 with no rep-level bytes: "reader is not initialized"
        } else {
          const HStream S = streams[pg.hs_rep];
          if (S.status != kOK) de = S.status;
          else {
            LevelSink sk{gmut(rep_arena) + job.slot_base + pg.slot_offset, (uint32_t)job.max_rep, 0};
            hybrid_expand(S, runs, blks, n, sh, sk);
          }
        }
      }
      if (de == kOK) {
        if (job.max_def > 0) {
          if (pg.def_n < 0) {
            de = kLEVELS;
          } else {
            const HStream S = streams[pg.hs_def];
            if (S.status != kOK) de = S.status;
            else {
              LevelSink sk{gmut(def_arena) + job.slot_base + pg.slot_offset, (uint32_t)job.max_def, 0};
              hybrid_expand(S, runs, blks, n, sh, sk);
              nn = wave_sum(sk.nn);
            }
          }
        } else {
          nn = n;
        }
      }
    }
    if (lane == 0) {
      pages[pidx].not_null = (int32_t)nn;
      if (de != kOK) pages[pidx].decode_status = de;
    }
  }
}

// ---- K3d ---------------------------------------------------------------------
// notNull prefix per chunk + dictionary-page resolution; one 256-lane block per job.
__global__ void __launch_bounds__(256) k_nn_scan(JobDev* jobs, PageDev* pages, uint8_t* scratch) {
  __shared__ int64_t part[5];
  JobDev& job = jobs[blockIdx.x];
  int np = job.num_pages < job.page_cap ? job.num_pages : job.page_cap;
  if (job.status == kCAPACITY) np = 0;
  int64_t carry = 0;
  for (int b = 0; b < np; b += 256) {
    const int i = b + threadIdx.x;
    int64_t v = 0;
    if (i < np) {
      const PageDev& pg = pages[job.page_base + i];
      if (pg.page_type == 0 || pg.page_type == 3) v = pg.not_null;
    }
    int64_t tot;
    const int64_t ex = block_excl_scan<256>(v, &tot, part);
    if (i < np) pages[job.page_base + i].value_offset = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) {
    job.num_values = carry;
    const int64_t vb = job.value_width > 0 ? carry * job.value_width : 0;
    if (job.value_width > 0 && vb > job.value_cap) job.status = kCAPACITY;
    job.values_bytes = vb;
    // dictionary page (page_dict.go:30-64): PLAIN entries of the column type.
    // The dictionary is published only when the page's read phase succeeds:
    // the gather sinks bound keys by dict_count alone, so a short page must
    // never be visible (the reference fails the chunk in readPages first).
    if (job.dict_page >= 0 && job.dict_page < np) {
      PageDev& dp = pages[job.page_base + job.dict_page];
      if (dp.read_status == kOK) {
        const uint8_t* blk =
            dp.scratch_offset >= 0 ? scratch + job.scratch_base + dp.scratch_offset : job.data + dp.payload_offset;
        const int64_t blen = dp.usize;
        const int64_t cnt = dp.num_values;
        const int w = job.value_width;
        dp.block = blk;
        dp.block_len = blen;
        int st = kOK;
        int flags = 0;
        if (w > 0) {
          if (job.type == 3) {  // INT96: a partial final entry is left nil, not an error (Q8)
            const int64_t full = blen / 12, rem = blen % 12;
            if (cnt > full + (rem > 0 ? 1 : 0)) st = kEOF;
            else if (cnt == full + 1 && rem > 0) flags = 1;
          } else if (cnt * w > blen) {
            st = kEOF;
          }
        } else {
          // u32-length entries (type_bytearray.go:24-45): k_str_dict walks them
          // (every entry takes >= 4 bytes: a walk fails before entry blen/4 + 1)
          flags = 2;
          job.need_doffs = (cnt < blen / 4 ? cnt : blen / 4) + 2;
          if (job.need_doffs > job.doffs_cap) job.status = kCAPACITY;
        }
        if (st == kOK) {
          job.flags |= flags;
          job.dict_data = blk;
          job.dict_count = (flags & 2) ? 0 : cnt;  // byte arrays: published by k_str_dict after its walk
          job.dict_len = blen;
        } else {
          dp.read_status = st;
        }
      }
    }
  }
}

}  // namespace pqg
