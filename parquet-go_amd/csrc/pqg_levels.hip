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

// ---- K3a ---------------------------------------------------------------------
__device__ __forceinline__ int reg_stream(JobDev& job, HStream* streams, int32_t* slot, int pidx, int kind,
                                          const uint8_t* p, int64_t n, int w, int64_t count) {
  const int64_t nruns = n / 2 + 2;  // every run but a truncated last one takes >= 2 bytes
  const int64_t nblks = count / kHBlock + 2;
  const int64_t rb = (int64_t)atomicAdd((unsigned long long*)&job.run_used, (unsigned long long)nruns);
  const int64_t bb = (int64_t)atomicAdd((unsigned long long*)&job.blk_used, (unsigned long long)nblks);
  if (rb + nruns > job.run_cap || bb + nblks > job.blk_cap) {
    job.status = kCAPACITY;  // the host grows the run arenas and decodes again
    return -1;
  }
  const int id = pidx * 3 + (kind > 2 ? 2 : kind);
  HStream& S = streams[id];
  S.p = p;
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
  S.pad = 0;
  *slot = id;
  return id;
}

__global__ void __launch_bounds__(256) k_page_setup(JobDev* jobs, PageDev* pages, const int* list, const int* total,
                                                    uint8_t* scratch, HStream* streams) {
  const int nt = *total;
  for (int t = blockIdx.x * 256 + threadIdx.x; t < nt; t += gridDim.x * 256) {
    const int pidx = list[t];
    PageDev& pg = pages[pidx];
    pg.hs_rep = pg.hs_def = pg.hs_val = -1;
    if (pg.read_status != kOK || (pg.page_type != 0 && pg.page_type != 3)) continue;
    JobDev& job = jobs[pg.job];
    if (job.status == kCAPACITY) continue;
    // ---- the page block and its level / value streams (read phase)
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
    const uint8_t *rep = nullptr, *def = nullptr;
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
      const uint8_t* lv = job.data + pg.payload_offset;
      if (levels > 0 && pg.rep_len > 0) { rep = lv; rep_n = pg.rep_len; }
      if (levels > 0 && pg.def_len > 0) { def = lv + pg.rep_len; def_n = levels - pg.rep_len; }
    }
    if (e != kOK) {
      pg.read_status = e;
      continue;
    }
    pg.block = block;
    pg.block_len = blen;
    pg.val = block + vpos;
    pg.val_n = blen - vpos;
    pg.rep = rep;
    pg.rep_n = rep_n;
    pg.def = def;
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
    const uint8_t* val = block + vpos;
    if (pg.encoding == 8 && vn >= 1) {
      const int w = val[0];
      pg.dict_width = w;
      if (w >= 1 && w <= 32 && n > 0) reg_stream(job, streams, &pg.hs_val, pidx, 2, val + 1, vn - 1, w, n);
    } else if (pg.encoding == 3 && job.type == 0 && vn >= 4) {
      const int64_t sz = rd_u32(val);
      const int64_t take = min(sz, vn - 4);
      if (n > 0) reg_stream(job, streams, &pg.hs_val, pidx, 3, val + 4, take, 1, n);
    }
  }
}

// ---- K3b ---------------------------------------------------------------------
// readUVariant32 (helpers.go:149-165) over the lane's byte reader.
__device__ __forceinline__ int lane_uvar32(LaneBytes& rd, int64_t& pos, uint32_t* out) {
  uint64_t x = 0;
  unsigned s = 0;
  for (int i = 0;; i++) {
    const int b = rd.get(pos);
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

// Lanes [0, total) walk the rep streams, [total, 2 total) the def streams,
// [2 total, 3 total) the value streams, so a wave's lanes do alike work.
__global__ void __launch_bounds__(256) k_hybrid_walk(const PageDev* pages, const int* list, const int* total,
                                                     HStream* streams, RunEnt* runs, int32_t* blks) {
  const int nt = *total;
  for (int g = blockIdx.x * 256 + threadIdx.x; g < 3 * nt; g += gridDim.x * 256) {
    const int kind = g / nt;
    const PageDev& pg = pages[list[g - kind * nt]];
    const int hs = kind == 0 ? pg.hs_rep : kind == 1 ? pg.hs_def : pg.hs_val;
    if (hs < 0) continue;
    HStream& S = streams[hs];
    const int w = S.w;
    const int64_t n = S.n, count = S.count;
    const int rb = (w + 7) / 8;
    RunEnt* R = runs + S.run_base;
    int32_t* B = blks + S.blk_base;
    LaneBytes rd;
    rd.init(S.p, n);
    int64_t pos = 0, produced = 0, next_blk = 0;
    int nr = 0, status = kOK;
    while (produced < count) {
      uint32_t h;
      int e = lane_uvar32(rd, pos, &h);
      if (e) { status = e; break; }
      int64_t take;
      RunEnt ent;
      if (h & 1) {  // bit-packed: h>>1 groups of 8 values, w bytes each
        const int64_t groups = h >> 1;
        if (groups == 0) { status = kRLE; break; }  // "empty bit-packed run"
        take = groups * 8 < count - produced ? groups * 8 : count - produced;
        const int64_t need = (take + 7) / 8;
        // groups whose first byte is inside the stream; a short read is zero padded
        const int64_t ok = pos < n ? (n - pos + w - 1) / w : 0;
        if (ok < need) {
          take = ok * 8;
          status = kEOF;
        }
        ent.start = (uint32_t)produced | kRunBP;
        ent.src = (uint32_t)pos;
        pos += groups * w;
      } else {  // RLE: h>>1 repeats of a ceil(w/8)-byte little-endian value
        const int64_t cnt = h >> 1;
        if (cnt == 0) { status = kRLE; break; }
        if (pos >= n || n - pos < rb) { status = kEOF; break; }
        uint32_t v = 0;
        for (int k = 0; k < rb; k++) v |= (uint32_t)rd.get(pos + k) << (8 * k);
        pos += rb;
        if (w < 32 && (v >> w) != 0) { status = kRLE; break; }  // readRLERunValue :127-129
        take = cnt < count - produced ? cnt : count - produced;
        ent.start = (uint32_t)produced;
        ent.src = v;
      }
      if (take > 0) {
        R[nr] = ent;
        produced += take;
        while (next_blk * kHBlock < produced) B[next_blk++] = nr;
        nr++;
      }
      if (status) break;
    }
    S.n_runs = nr;
    S.produced = (int32_t)produced;
    S.status = status;
  }
}

// ---- K3c ---------------------------------------------------------------------
struct LevelSink {
  uint8_t* out;
  uint32_t maxl;
  int64_t nn;
  __device__ __forceinline__ void put(int64_t i0, const uint32_t (&v)[8], int cnt) {
    uint8_t* o = out + i0;
    if (cnt == 8 && ((uintptr_t)o & 7) == 0) {
      uint2 x;
      x.x = v[0] | v[1] << 8 | v[2] << 16 | v[3] << 24;
      x.y = v[4] | v[5] << 8 | v[6] << 16 | v[7] << 24;
      *(uint2*)o = x;
    } else {
      for (int q = 0; q < cnt; q++) o[q] = (uint8_t)v[q];
    }
    for (int q = 0; q < cnt; q++) nn += v[q] == maxl;
  }
};

__global__ void __launch_bounds__(64) k_levels_expand(JobDev* jobs, PageDev* pages, const int* list,
                                                      const int* total, int* queue, const HStream* streams,
                                                      const RunEnt* runs, const int32_t* blks, uint8_t* def_arena,
                                                      uint8_t* rep_arena) {
  __shared__ __attribute__((aligned(16))) ExpandShared sh;
  const int lane = lane_id();
  for (;;) {
    int t = 0;
    if (lane == 0) t = atomicAdd(queue, 1);
    t = __shfl(t, 0, 64);
    if (t >= *total) return;
    PageDev& pg = pages[list[t]];
    if (pg.read_status != kOK || (pg.page_type != 0 && pg.page_type != 3)) continue;
    const JobDev& job = jobs[pg.job];
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
          const HStream& S = streams[pg.hs_rep];
          if (S.status != kOK) de = S.status;
          else {
            LevelSink sk{rep_arena + job.slot_base + pg.slot_offset, (uint32_t)job.max_rep, 0};
            hybrid_expand(S, runs, blks, n, sh, sk);
          }
        }
      }
      if (de == kOK) {
        if (job.max_def > 0) {
          if (pg.def_n < 0) {
            de = kLEVELS;
          } else {
            const HStream& S = streams[pg.hs_def];
            if (S.status != kOK) de = S.status;
            else {
              LevelSink sk{def_arena + job.slot_base + pg.slot_offset, (uint32_t)job.max_def, 0};
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
      pg.not_null = (int32_t)nn;
      if (de != kOK) pg.decode_status = de;
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
        if (w > 0) {
          if (job.type == 3) {  // INT96: a partial final entry is left nil, not an error (Q8)
            const int64_t full = blen / 12, rem = blen % 12;
            if (cnt > full + (rem > 0 ? 1 : 0)) dp.read_status = kEOF;
            else if (cnt == full + 1 && rem > 0) job.flags |= 1;
          } else if (cnt * w > blen) {
            dp.read_status = kEOF;
          }
          job.dict_data = blk;
          job.dict_count = cnt;
          job.dict_len = blen;
        } else {
          dp.read_status = kUNSUPPORTED;  // variable-length dictionaries: not in this build yet
        }
      }
    }
  }
}

}  // namespace pqg
