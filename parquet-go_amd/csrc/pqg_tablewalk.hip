// pqg_tablewalk.hip — K3b, wave-parallel: the run tables of the value streams
// (dictionary indices, RLE booleans) for the values kernels, one WAVE per
// stream instead of k_hybrid_walk's one lane per stream.
//
// hybridDecoder.next (hybrid_decoder.go:82-166) walked as the in-kernel index
// walk does (IdxWalk, pqg_idxwalk.h: its ring window and speculative header
// parse are reused as they are): per step every lane parses a run header at
// pos + lane, the chain from the step's first run is marked by pointer
// doubling, a saturating DPP scan gives each chain run its first value.  The
// sink writes tables instead of keys:
//   * RunEnt {first value | kRunBP, payload offset | RLE value} of every run,
//     at its rank in the chain (one coalesced store per run lane);
//   * BlockDesc {v0, r0, payload lo, bytes | runs << 16}: a step's runs form
//     one batch of at most kHBlock values whose bit-packed payload spans at
//     most kHBlockBytes (the step is cut where a run would pass either); a
//     batch joins the open block while the block stays within kHBlock values,
//     kHBlockRuns runs and kHBlockBytes of payload, else it closes the block
//     and opens the next.  A run longer than a batch is cut into blocks of K
//     values written by the lanes (the long-run case k_walk_long takes for
//     the lane walker).
// Greedy merging leaves no two consecutive blocks that fit one, so a stream
// has at most 2 (n / kHBlock + runs / kHBlockRuns + bytes / kHBlockBytes) + 1
// + (long runs) blocks: k_page_list reserves that many (`wave_walk`).
// n_runs, produced and status are exactly the lane walker's: the walk runs
// to `count` values (an upper bound of the page's notNull) or the stream's
// first error, with the same error classes.
#include <hip/hip_runtime.h>

#include "pqg_common.h"
#include "pqg_device.h"
#include "pqg_hybrid.h"
#include "pqg_idxwalk.h"

namespace pqg {

__device__ __forceinline__ uint32_t ldpp_incl_min_u32(uint32_t x) {
  uint32_t t;
#define PQG_MIN_STEP(ctrl, rm, bc)                                                   \
  t = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)x, ctrl, rm, 0xf, bc);          \
  x = t < x ? t : x;
  PQG_MIN_STEP(0x111, 0xf, true) PQG_MIN_STEP(0x112, 0xf, true) PQG_MIN_STEP(0x114, 0xf, true)
  PQG_MIN_STEP(0x118, 0xf, true) PQG_MIN_STEP(0x142, 0xa, false) PQG_MIN_STEP(0x143, 0xc, false)
#undef PQG_MIN_STEP
  return x;
}

struct TableWalk {
  IdxWalk<GlobalDict, false> iw;  // the stream's ring window and header parse (no keys sunk)
  PQG_G uint32_t* R;              // RunEnt table, 2 dwords per run
  PQG_G uint32_t* B;              // BlockDesc table, 4 dwords per block
  uint32_t count;
  uint32_t K;                     // values per block of a long bit-packed run
  uint32_t produced = 0, nr = 0, nb = 0;
  int status = kOK;
  // the open block
  bool ob = false;
  uint32_t ob_v0 = 0, ob_r0 = 0, ob_nv = 0, ob_nr = 0;
  uint32_t ob_lo = 0xffffffffu, ob_hi = 0;  // payload bytes [lo, hi) (lo = ~0: none)

  __device__ __forceinline__ void put_block(uint32_t v0, uint32_t r0, uint32_t lo, uint32_t hi, uint32_t nruns) {
    const bool pay = lo != 0xffffffffu;
    stg16((uintptr_t)(B + 4 * nb), make_uint4(v0, r0, pay ? lo : 0u, ((pay ? hi - lo : 0u) & 0xffffu) | (nruns << 16)));
  }
  __device__ __forceinline__ void close_open() {
    if (ob && lane_id() == 0) put_block(ob_v0, ob_r0, ob_lo, ob_hi, ob_nr);
    nb += ob ? 1u : 0u;
    ob = false;
  }
  // values [v0, v0 + nv) over runs [r0, r0 + nruns) with payload [lo, hi):
  // joins the open block or starts the next one
  __device__ __forceinline__ void add(uint32_t v0, uint32_t r0, uint32_t nv, uint32_t nruns, uint32_t lo, uint32_t hi,
                                      bool same_run) {
    if (ob) {
      const uint32_t l2 = lo < ob_lo ? lo : ob_lo, h2 = hi > ob_hi ? hi : ob_hi;
      const uint32_t runs2 = ob_nr + nruns - (same_run ? 1u : 0u);
      if (ob_nv + nv <= (uint32_t)kHBlock && runs2 <= (uint32_t)kHBlockRuns &&
          (l2 == 0xffffffffu || h2 - l2 <= (uint32_t)kHBlockBytes)) {
        ob_nv += nv;
        ob_nr = runs2;
        ob_lo = l2;
        ob_hi = h2;
        return;
      }
      close_open();
    }
    ob = true;
    ob_v0 = v0;
    ob_r0 = r0;
    ob_nv = nv;
    ob_nr = nruns;
    ob_lo = lo;
    ob_hi = hi;
  }

  // The chain runs in mask m (each lane: first value s relative to
  // `produced`, take k, payload offset / RLE value pay, bp): their RunEnts,
  // and the batch as one block.  Returns the values taken.
  __device__ __forceinline__ uint32_t emit(uint64_t m, uint32_t s, uint32_t k, bool bp, uint32_t pay) {
    const int lane = lane_id();
    const bool mine = ((m >> lane) & 1) && k > 0;
    const uint64_t mm = __ballot(mine);
    if (!mm) return 0;
    const int rank = __popcll(mm & ((1ull << lane) - 1));
    if (mine) stg8((uintptr_t)(R + 2 * (nr + (uint32_t)rank)), (produced + s) | (bp ? kRunBP : 0u), pay);
    const int ll = 63 - __builtin_clzll(mm);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)(s + k), ll);
    const uint64_t pend = bp ? (((uint64_t)pay * 8 + (uint64_t)k * (uint32_t)iw.w + 7) >> 3) : 0ull;
    const uint32_t lo = (uint32_t)wave_min((int64_t)(mine && bp ? pay : 0xffffffffu));
    const uint32_t hi = (uint32_t)-wave_min(-(int64_t)(mine && bp ? (pend > 0xffffffffull ? 0xffffffffu : (uint32_t)pend) : 0u));
    const uint32_t nruns = (uint32_t)__popcll(mm);
    add(produced, nr, total, nruns, lo, hi, false);
    nr += nruns;
    return total;
  }

  // One run of `take` values alone (longer than a batch, or a > 4-byte header):
  // its RunEnt, blocks of K values (bit-packed) or kHBlock values (RLE), the
  // last of them left open.
  __device__ __forceinline__ void long_run(bool bp, uint32_t pay, uint32_t take) {
    const int lane = lane_id();
    if (lane == 0) stg8((uintptr_t)(R + 2 * nr), produced | (bp ? kRunBP : 0u), pay);
    const uint32_t per = bp ? K : (uint32_t)kHBlock;
    const uint32_t np = (take + per - 1) / per;
    // the first piece may join the open block (the run is new there)
    auto piece = [&](uint32_t j, uint32_t& lo, uint32_t& hi, uint32_t& nv) {
      const uint32_t a = j * per;
      nv = take - a < per ? take - a : per;
      if (bp) {
        const uint64_t b0 = (uint64_t)pay * 8 + (uint64_t)a * (uint32_t)iw.w;
        lo = (uint32_t)(b0 >> 3);
        const uint64_t e = (b0 + (uint64_t)nv * (uint32_t)iw.w + 7) >> 3;
        hi = e > 0xffffffffull ? 0xffffffffu : (uint32_t)e;
      } else {
        lo = 0xffffffffu;
        hi = 0u;
      }
    };
    uint32_t lo, hi, nv;
    piece(0, lo, hi, nv);
    add(produced, nr, nv, 1u, lo, hi, false);
    if (np > 1) {
      close_open();
      // pieces 1 .. np - 2 closed here, by the lanes; np - 1 stays open
      for (uint32_t j = 1 + (uint32_t)lane; j + 1 < np; j += 64) {
        uint32_t l2, h2, n2;
        piece(j, l2, h2, n2);
        const bool pay2 = l2 != 0xffffffffu;
        stg16((uintptr_t)(B + 4 * (nb + j - 1)),
              make_uint4(produced + j * per, nr, pay2 ? l2 : 0u, ((pay2 ? h2 - l2 : 0u) & 0xffffu) | (1u << 16)));
      }
      nb += np - 2;
      piece(np - 1, lo, hi, nv);
      ob = true;
      ob_v0 = produced + (np - 1) * per;
      ob_r0 = nr;
      ob_nv = nv;
      ob_nr = 1;
      ob_lo = lo;
      ob_hi = hi;
    }
    nr++;
    produced += take;
  }

  // A run met alone: its take (short bit-packed reads end the stream), its
  // tables, then pos.  Returns true when the stream ends here.
  __device__ __forceinline__ bool single_run(bool bp, uint32_t cnt, uint32_t pay, uint32_t nx, uint32_t& pos) {
    const uint32_t left = count - produced;
    uint32_t take = cnt < left ? cnt : left;
    int e = kOK;
    if (bp) {
      const uint64_t need = (take + 7) >> 3;
      if ((uint64_t)pay + (need - 1) * (uint32_t)iw.w >= iw.n) {
        const uint32_t ok = pay < iw.n ? (iw.n - pay + (uint32_t)iw.w - 1) / (uint32_t)iw.w : 0u;
        take = ok * 8;
        e = kEOF;
      }
    }
    if (take) long_run(bp, pay, take);
    if (e != kOK) {
      status = e;
      return true;
    }
    pos = nx;
    return false;
  }

  // The header at q byte by byte (binary.ReadUvarint + the MaxInt32 check),
  // then its run.  Returns true when the stream ends.
  __device__ __forceinline__ bool serial_run(uint32_t q, uint32_t& pos) {
    const uint32_t n = iw.n;
    const int w = iw.w;
    uint64_t v = 0;
    unsigned sft = 0;
    uint32_t hl = 0;
    int e = kOK;
    for (uint32_t i = 0;; i++) {
      if (q + i >= n) { e = kEOF; break; }
      const uint32_t b = iw.byte_at(q + i);
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
    if (e != kOK) {
      status = e;
      return true;
    }
    const uint32_t h = (uint32_t)v, g = h >> 1;
    if (g == 0) {
      status = kRLE;
      return true;
    }
    if (h & 1) {
      const uint64_t nx = (uint64_t)q + hl + (uint64_t)g * (uint32_t)w;
      return single_run(true, g > 0x1fffffffu ? 0xffffffffu : g * 8, q + hl, nx > 0xffffffffull ? 0xffffffffu : (uint32_t)nx,
                        pos);
    }
    const uint32_t rb = ((uint32_t)w + 7) >> 3, vp = q + hl;
    if ((uint64_t)vp + rb > n) {
      status = kEOF;
      return true;
    }
    uint32_t val = 0;
    for (uint32_t k = 0; k < rb; k++) val |= iw.byte_at(vp + k) << (8 * k);
    if (w < 32 && (val >> w) != 0) {
      status = kRLE;
      return true;
    }
    return single_run(false, g, val, vp + rb, pos);
  }

  __device__ __forceinline__ void walk() {
    const int lane = lane_id();
    const uint32_t n = iw.n;
    const int w = iw.w;
    uint32_t pos = 0;
    while (produced < count) {
      if (pos >= n) {
        status = kEOF;
        break;
      }
      iw.ensure(pos);
      const uint32_t left = count - produced;
      // ---- speculative headers and the chain (IdxWalk's)
      const IRun r = iw.parse(pos + (uint32_t)lane);
      const int nx = iw.succ(r, pos);
      uint64_t cm = 1;
      if (__builtin_amdgcn_readfirstlane(nx) < kIPos) cm = chain_marks64(nx, lds_ptr(iw.sh->cflag));
      const bool on = (cm >> lane) & 1;
      const uint32_t c = on ? r.cnt : 0u;
      const uint32_t st = cm == 1 ? 0u : dpp_incl_add_sat(c) - c;
      int e = kOK;
      uint32_t take = 0;
      const bool need = on && st < left;
      if (need) {
        if (r.cplx) e = kCOMPLEX;
        else if (r.err != kOK) e = r.err;
        else {
          take = r.cnt < left - st ? r.cnt : left - st;
          if (r.bp) {
            const uint64_t ng = (take + 7) >> 3;
            if ((uint64_t)r.pay + (ng - 1) * (uint32_t)w >= n) {
              const uint32_t ok = r.pay < n ? (n - r.pay + (uint32_t)w - 1) / (uint32_t)w : 0u;
              take = ok * 8;
              e = kEOF;
            }
          }
        }
      }
      // ---- the batch: at most kHBlock values, payload within kHBlockBytes
      const uint32_t pend = (need && r.bp) ? (uint32_t)min((((uint64_t)r.pay * 8 + (uint64_t)take * (uint32_t)w + 7) >> 3),
                                                          (uint64_t)0xffffffffu)
                                           : 0u;
      const uint32_t minpay = ldpp_incl_min_u32(need && r.bp ? r.pay : 0xffffffffu);
      const bool cut = need && e == kOK &&
                       ((uint64_t)st + take > (uint64_t)kHBlock || (r.bp && pend - minpay > (uint32_t)kHBlockBytes));
      const uint64_t eb = __ballot(e != kOK), xb = __ballot(cut), nb_ = __ballot(need);
      const int first_err = eb ? __ffsll((long long)eb) - 1 : kIPos;
      const int first_cut = xb ? __ffsll((long long)xb) - 1 : kIPos;
      auto below = [](int lim) { return lim >= 64 ? ~0ull : ((1ull << lim) - 1); };
      auto next_of = [&](uint64_t m) {
        const int ll = 63 - __builtin_clzll(m);
        return (uint32_t)__builtin_amdgcn_readlane((int)r.next, ll);
      };
      if (first_cut < kIPos && first_cut <= first_err) {
        if (first_cut == 0) {  // run 0 alone passes a batch
          if (single_run(__builtin_amdgcn_readfirstlane((int)r.bp) != 0, (uint32_t)__builtin_amdgcn_readfirstlane((int)r.cnt),
                         (uint32_t)__builtin_amdgcn_readfirstlane((int)r.pay),
                         (uint32_t)__builtin_amdgcn_readfirstlane((int)r.next), pos))
            break;
          continue;
        }
        const uint64_t m = nb_ & below(first_cut);
        produced += emit(m, st, take, r.bp, r.pay);
        pos = next_of(m);
        continue;
      }
      if (first_err < kIPos) {
        const int ee = __builtin_amdgcn_readlane(e, first_err);
        if (ee == kCOMPLEX) {  // the runs before it, then its header byte by byte
          const uint64_t m = nb_ & below(first_err);
          if (m) produced += emit(m, st, take, r.bp, r.pay);
          if (serial_run(pos + (uint32_t)first_err, pos)) break;
          continue;
        }
        // the runs before the failing one, then its own take (a short
        // bit-packed run keeps the groups that start in the stream) alone
        const uint64_t m = nb_ & below(first_err);
        if (m) produced += emit(m, st, take, r.bp, r.pay);
        const uint32_t tf = (uint32_t)__builtin_amdgcn_readlane((int)take, first_err);
        if (tf) long_run(__builtin_amdgcn_readlane((int)r.bp, first_err) != 0, (uint32_t)__builtin_amdgcn_readlane((int)r.pay, first_err), tf);
        status = ee;
        break;
      }
      produced += emit(nb_, st, take, r.bp, r.pay);
      pos = next_of(nb_);
    }
    close_open();
  }
};

// One wave per value stream of the page list (pages pulled from a queue).
__global__ void __launch_bounds__(64) k_walk_wave(const PageDev* pages, const int* list, const int* total, int* queue,
                                                  HStream* streams, RunEnt* runs, BlockDesc* blks, int skip_dict_small) {
  __shared__ __attribute__((aligned(16))) WalkShared sh;
  const int lane = lane_id();
  for (;;) {
    const int t = queue_next(queue);
    if (t >= *total) return;
    const PageDev& pg = pages[__builtin_amdgcn_readfirstlane(list[t])];
    const int hs = __builtin_amdgcn_readfirstlane(pg.hs_val);
    if (hs < 0 || (skip_dict_small && dict_walk_page(pg))) continue;  // no stream, or walked in k_dict_walk
    HStream& S = streams[hs];
    const gcu8 p = gconst(S.p);
    const int w = S.w;
    TableWalk tw{IdxWalk<GlobalDict, false>{p, (uint32_t)S.n, w, (uint32_t)S.count, nullptr, 0u, GlobalDict{nullptr}, &sh,
                                             (uint32_t)((uintptr_t)p & (kIWin - 1))},
                 (PQG_G uint32_t*)(gmut(runs) + S.run_base), (PQG_G uint32_t*)(gmut(blks) + S.blk_base),
                 (uint32_t)S.count, min((uint32_t)kHBlock, ((8u * kHBlockBytes - 14u) / (uint32_t)w) & ~7u)};
    tw.walk();
    if (lane == 0) {
      S.n_runs = (int32_t)tw.nr;
      S.produced = (int32_t)tw.produced;
      S.status = tw.status;
      S.n_blocks = (int32_t)tw.nb;
    }
  }
}

}  // namespace pqg
