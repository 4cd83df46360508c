// pqg_values.hip — K4: values[:notNull] of every data page, K5: chunk status.
//
//   K4 k_values    one wave per data page: valuesDecoder.init (read phase) and
//                  decodeValues (chunk_reader.go:143-196 dispatch): PLAIN
//                  fixed-width copies (type_int32.go:12-37, type_int64.go:12-37,
//                  type_int96.go:21-42, type_float.go:23-33, type_double.go:22-32,
//                  type_boolean.go:10-69), RLE_DICTIONARY gather through the
//                  index run table (type_dict.go:39-59), DELTA_BINARY_PACKED
//                  (deltabp_decoder.go:14-334), RLE booleans
//   K5 k_finalize  chunk status in reference order
#include <hip/hip_runtime.h>

#include "pqg_common.h"
#include "pqg_device.h"
#include "pqg_hybrid.h"

namespace pqg {

#ifndef PQG_DBP_WPE
#define PQG_DBP_WPE 4  // the same for the DELTA_BINARY_PACKED stage
#endif
#ifndef PQG_VALUES_WPE
#define PQG_VALUES_WPE 1  // minimum waves per SIMD the register allocation must allow
#endif

#ifdef PQG_PROFILE
// host reader of this translation unit's phase counters (see pqg_debug_counters)
int prof_read_values(unsigned long long* out) {
  unsigned long long z[64] = {0};
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pqg_prof), sizeof(z)) != hipSuccess) return -1;
  hipMemcpyToSymbol(HIP_SYMBOL(pqg_prof), z, sizeof(z));
  return 0;
}
#endif

// ============================================================================
// K4: values — one wave per data page.
// ============================================================================
// dictDecoder.decodeValues (type_dict.go:39-59): dst[i] = values[key],
// "dict: invalid index" when key >= len(values).  W bytes per entry (W == 0:
// runtime width `w`, a byte-copy path for FLBA / INT96 dictionaries).  All the
// gathers of a group are issued before its stores (see pqg_hybrid.h).
template <int W>
struct DictSink {
  gu8 out;
  gcu8 dict;        // never null (a safe base when the chunk has no dictionary)
  int64_t count;
  int64_t bad;      // first index with an invalid key
  int64_t nil_key;  // INT96 partial final entry (-1: none): its value reads as zero bytes (Q8)
  int w;
  // W == 4, every key of the group valid (checked with one max + one ballot
  // instead of per value): the gathers issued by prepare(), stored by group()
  bool fast = false;
  uint32_t gv4[kGroup][8];
  __device__ __forceinline__ void prepare(const uint32_t (&v)[kGroup][8], const uint32_t (&i0)[kGroup],
                                          const int (&cnt)[kGroup]) {
    if (W != 4) return;
    uint32_t mx = 0;
#pragma unroll
    for (int b = 0; b < kGroup; b++)
#pragma unroll
      for (int q = 0; q < 8; q++) mx = q < cnt[b] && v[b][q] > mx ? v[b][q] : mx;
    fast = !__ballot((int64_t)mx >= count);
    if (!fast) return;
    const PQG_G uint32_t* d = (const PQG_G uint32_t*)dict;
#ifdef PQG_EXP_NOGATHER
#pragma unroll
    for (int b = 0; b < kGroup; b++)
#pragma unroll
      for (int q = 0; q < 8; q++) gv4[b][q] = v[b][q];
    (void)d;
#else
#pragma unroll
    for (int b = 0; b < kGroup; b++)
#pragma unroll
      for (int q = 0; q < 8; q++) gv4[b][q] = d[q < cnt[b] ? v[b][q] : 0u];
#endif
  }
  __device__ __forceinline__ void group(const uint32_t (&v)[kGroup][8], const uint32_t (&i0)[kGroup],
                                        const int (&cnt)[kGroup]) {
    if (W == 4 && fast) {
#ifdef PQG_EXP_NOSTORE
      uint32_t x = 0;
#pragma unroll
      for (int b = 0; b < kGroup; b++)
#pragma unroll
        for (int q = 0; q < 8; q++) x ^= gv4[b][q];
      if (x == 0x9e3779b9u) *(PQG_G uint32_t*)out = x;  // keeps the gathers alive
      return;
#endif
      // aligned 16-byte stores whatever the page's alignment (store_run_aligned)
#pragma unroll
      for (int b = 0; b < kGroup; b++) {
        if (!__ballot(cnt[b] > 0)) continue;
        const uint32_t v0 = (uint32_t)__builtin_amdgcn_readfirstlane(i0[b]);
        // dictionaries larger than 256 KiB: non-temporal stores keep the
        // output from evicting dictionary lines (b = 20: -5 %)
        if (count > 65536) store_run_aligned<8, true>((uintptr_t)(out + (int64_t)v0 * 4), gv4[b], cnt[b]);
        else
          store_run_aligned<8>((uintptr_t)(out + (int64_t)v0 * 4), gv4[b], cnt[b]);
      }
      return;
    }
    bool ok[kGroup][8];
#pragma unroll
    for (int b = 0; b < kGroup; b++)
#pragma unroll
      for (int q = 0; q < 8; q++) {
        ok[b][q] = q < cnt[b] && (int64_t)v[b][q] < count;
        if (q < cnt[b] && !ok[b][q]) bad = (int64_t)(i0[b] + q) < bad ? (int64_t)(i0[b] + q) : bad;
      }
    if (W == 4) {
      uint32_t gv[kGroup][8];
      const PQG_G uint32_t* d = (const PQG_G uint32_t*)dict;
#pragma unroll
      for (int b = 0; b < kGroup; b++)
#pragma unroll
        for (int q = 0; q < 8; q++) gv[b][q] = d[ok[b][q] ? v[b][q] : 0u];
#pragma unroll
      for (int b = 0; b < kGroup; b++) {
        if (cnt[b] == 0) continue;
        const uintptr_t o = (uintptr_t)(out + (int64_t)i0[b] * 4);
        if (cnt[b] == 8 && (o & 15) == 0 && ok[b][0] && ok[b][1] && ok[b][2] && ok[b][3] && ok[b][4] && ok[b][5] &&
            ok[b][6] && ok[b][7]) {
          stg16o(o, make_uint4(gv[b][0], gv[b][1], gv[b][2], gv[b][3]));
          stg16o(o + 16, make_uint4(gv[b][4], gv[b][5], gv[b][6], gv[b][7]));
        } else {
#pragma unroll
          for (int q = 0; q < 8; q++)
            if (ok[b][q]) ((PQG_G uint32_t*)o)[q] = gv[b][q];
        }
      }
    } else if (W == 8) {
      u32x2_t gv[kGroup][8];
      const PQG_G u32x2_t* d = (const PQG_G u32x2_t*)dict;
#pragma unroll
      for (int b = 0; b < kGroup; b++)
#pragma unroll
        for (int q = 0; q < 8; q++) gv[b][q] = d[ok[b][q] ? v[b][q] : 0u];
#pragma unroll
      for (int b = 0; b < kGroup; b++) {
        if (cnt[b] == 0) continue;
        const uintptr_t o = (uintptr_t)(out + (int64_t)i0[b] * 8);
#pragma unroll
        for (int q = 0; q < 8; q++)
          if (ok[b][q]) stg8(o + 8 * q, gv[b][q].x, gv[b][q].y);
      }
    } else {
#pragma unroll
      for (int b = 0; b < kGroup; b++)
#pragma unroll
        for (int q = 0; q < 8; q++) {
          if (!ok[b][q]) continue;
          const int64_t key = v[b][q], i = (int64_t)i0[b] + q;
          gcu8 s = dict + key * w;
          for (int c = 0; c < w; c++) out[i * w + c] = (key == nil_key) ? 0 : s[c];
        }
    }
  }
};

// booleanRLEDecoder (type_boolean.go:100-120): value == 1
struct BoolSink {
  gu8 out;
  __device__ __forceinline__ void prepare(const uint32_t (&)[kGroup][8], const uint32_t (&)[kGroup], const int (&)[kGroup]) {}
  __device__ __forceinline__ void group(const uint32_t (&v)[kGroup][8], const uint32_t (&i0)[kGroup],
                                        const int (&cnt)[kGroup]) {
    for (int b = 0; b < kGroup; b++)
      for (int q = 0; q < cnt[b]; q++) out[i0[b] + q] = v[b][q] == 1;
  }
};

// ---- DELTA_BINARY_PACKED (deltabp_decoder.go) ------------------------------
constexpr int kBlocks = 64;
constexpr int kMaxMb = 8;

#ifndef PQG_DBP_STAGE
#define PQG_DBP_STAGE 4096
#endif
constexpr int kDStage = PQG_DBP_STAGE;  // staged bytes of the regular path (a multiple of 1024)
struct DbpShared {
  uint8_t stage[kDStage + 32];          // regular path: block headers and bodies
  uint8_t win[kWin];
  int64_t body[kBlocks];                // stream offset of the block's first miniblock
  uint64_t mind[kBlocks];               // min delta (as unsigned for wrapping adds)
  uint64_t wpk[kBlocks];                // staged path: the block's miniblock widths, one per byte
  uint32_t sbody[kBlocks];              // staged path: stage byte of the block's first miniblock
  uint8_t widths[kBlocks][kMaxMb];
  int64_t mb_off[kBlocks][kMaxMb];      // stream offset of each miniblock
  uint8_t gwidths[256];                 // generic path: miniblock widths of the block
  uint64_t gvals[8];                    // generic path: current 8-group
};

// Stage [at, at + kDStage) of a DBP stream (from a 16-byte aligned address;
// bytes at or past n read as zero) into LDS with one round of loads.
__device__ __forceinline__ void dbp_restage(gcu8 s, int64_t n, PQG_L uint8_t* stb, int64_t at, int64_t& st_lo,
                                            int64_t& st_hi) {
  const int lane = lane_id();
  st_lo = at - (int64_t)(((uintptr_t)(s + at)) & 15);
  uint4 g[kDStage / 1024];
  // every load unconditional (a granule holding no stream byte reads the
  // stream's first one and is zeroed after all are issued: a load under a
  // branch is waited for inside it)
  const uintptr_t safe = (uintptr_t)s & ~(uintptr_t)15;
#pragma unroll
  for (int k = 0; k < kDStage / 1024; k++) {
    const int64_t o = st_lo + 16 * (int64_t)(lane + 64 * k);
    g[k] = ldg16((o < n && o + 16 > 0) ? (uintptr_t)(s + o) : safe);
  }
#pragma unroll
  for (int k = 0; k < kDStage / 1024; k++) {
    const int64_t o = st_lo + 16 * (int64_t)(lane + 64 * k);
    sts16(stb + 16 * (lane + 64 * k), (o < n && o + 16 > 0) ? mask_tail(g[k], o, n) : make_uint4(0u, 0u, 0u, 0u));
  }
  st_hi = st_lo + kDStage;
  __builtin_amdgcn_wave_barrier();
}
// binary.ReadUvarint over the stage (bytes at or past n: EOF)
__device__ __forceinline__ int dbp_st_uvarint(const PQG_L uint8_t* stb, int64_t st_lo, int64_t n, int64_t& q,
                                              uint64_t* out) {
  uint64_t x = 0;
  unsigned sft = 0;
  for (int i = 0;; i++) {
    if (q >= n) return kEOF;
    const uint32_t bt = stb[q - st_lo];
    q++;
    if (bt < 0x80) {
      if (i > 9 || (i == 9 && bt > 1)) return kRLE;
      *out = x | (sft < 64 ? (uint64_t)bt << sft : 0);
      return kOK;
    }
    if (sft < 64) x |= (uint64_t)(bt & 0x7f) << sft;
    sft += 7;
  }
}

// The regular-layout block walk through a Window, resuming at position p0 /
// block header blk_pos / value carry: for blocks too large for dbp_decode's
// stage (the fast path's fallback; the same semantics).
__device__ __forceinline__ int dbp_decode_rest(gcu8 s, int64_t n, int64_t readable, bool is64, int64_t nn, gu8 out, DbpShared& sh,
                               int64_t P, int64_t p0, int64_t blk_pos, uint64_t carry, int32_t bs, int32_t mbc,
                               int32_t mbvc, int32_t total, bool pow2, int bs_sh, int mb_sh) {
  const int lane = lane_id();
  const int maxw = is64 ? 64 : 32;
  Window win{s, n, kFarAway, lds_ptr(sh.win)};
  int e;
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
    // unpack + wrapping prefix over positions [p0, p_end): value(p) = carry + Σ deltas.
    // A lane's 4 positions share one miniblock (mbvc % 8 == 0), so the block /
    // miniblock split is done once per lane, by shifts for power-of-two sizes.
    for (int64_t t0 = p0; t0 < p_end; t0 += 256) {
      uint64_t d[4];
      uint64_t local = 0;
      const int64_t pb = t0 + lane * 4;
      const uint32_t rel = (uint32_t)(pb - p0);  // < kBlocks * bs <= 2^31 (regular)
      uint32_t b, r2, m, j;
      if (pow2) {
        b = rel >> bs_sh;
        r2 = rel & (uint32_t)(bs - 1);
        m = r2 >> mb_sh;
        j = r2 & (uint32_t)(mbvc - 1);
      } else {
        b = rel / (uint32_t)bs;
        r2 = rel - b * (uint32_t)bs;
        m = r2 / (uint32_t)mbvc;
        j = r2 - m * (uint32_t)mbvc;
      }
      const bool any = pb < p_end;
      const int wv = any ? sh.widths[b][m] : 0;
      const int64_t bit0 = any ? sh.mb_off[b][m] * 8 + (int64_t)j * wv : 0;
      const uint64_t mnd = any ? sh.mind[b] : 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        uint64_t dv = 0;
        if (pb + k < p_end) dv = extract_bits64(s, readable, n, bit0 + (int64_t)k * wv, wv) + mnd;
        d[k] = dv;
        local += dv;
      }
      uint64_t incl = wave_incl_scan_u64(local);
      uint64_t run = carry + (incl - local);
      const int nvp = pb >= p_end ? 0 : (p_end - pb >= 4 ? 4 : (int)(p_end - pb));
      if (is64) {
        uint32_t dw[8];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          dw[2 * k] = (uint32_t)run;
          dw[2 * k + 1] = (uint32_t)(run >> 32);
          run += d[k];
        }
        store_run_aligned<8>((uintptr_t)(out + t0 * 8), dw, 2 * nvp);
      } else {
        uint32_t dw[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          dw[k] = (uint32_t)run;
          run += d[k];
        }
        store_run_aligned<4>((uintptr_t)(out + t0 * 4), dw, nvp);
      }
      carry += __shfl(incl, 63, 64);
    }
    __builtin_amdgcn_wave_barrier();
    p0 = p_end;
  }
  if (nn > total) return kEOF;
  return kOK;
}

// Eight-byte values at base + 8 (4 L + k), k < nv (4 except at the ragged
// end), as aligned 16-byte granules: base is 8-byte aligned, so the run
// starts 0 or 8 bytes before a granule; at 8, lane L stores its values 1..3
// and lane L + 1's value 0 (DPP wave_shl:1), lane 0 its value 0 alone.
// Plain (write-back) stores: each instruction writes every other 16-byte
// granule of the wave's 2 KiB, and non-temporal stores sent those half lines
// out unmerged (C3 k_values<3>: WRITE_SIZE 2.09 GB for 1.6 GB of int64,
// 0.64 ms; write-back: 1.60 GB, 0.48 ms).
template <bool Full>
__device__ __forceinline__ void store_run64(uintptr_t base, const uint64_t (&v)[4], int nv) {
  const int lane = lane_id();
  const bool shifted = __builtin_amdgcn_readfirstlane((int)(base & 8)) != 0;
  const uintptr_t o = base + 32 * (uintptr_t)lane;
  if (!shifted) {
    if (Full || nv == 4) {
      stg16(o, make_uint4((uint32_t)v[0], (uint32_t)(v[0] >> 32), (uint32_t)v[1], (uint32_t)(v[1] >> 32)));
      stg16(o + 16, make_uint4((uint32_t)v[2], (uint32_t)(v[2] >> 32), (uint32_t)v[3], (uint32_t)(v[3] >> 32)));
    } else {
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (k < nv) stg8(o + 8 * k, (uint32_t)v[k], (uint32_t)(v[k] >> 32));
    }
    return;
  }
  const uint32_t n0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v[0], 0x130, 0xf, 0xf, true);
  const uint32_t n1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v[0] >> 32), 0x130, 0xf, 0xf, true);
  const int nxv = Full ? 4 : __builtin_amdgcn_update_dpp(0, nv, 0x130, 0xf, 0xf, true);
  if (Full ? lane < 63 : (nv == 4 && nxv >= 1)) {
    stg16(o + 8, make_uint4((uint32_t)v[1], (uint32_t)(v[1] >> 32), (uint32_t)v[2], (uint32_t)(v[2] >> 32)));
    stg16(o + 24, make_uint4((uint32_t)v[3], (uint32_t)(v[3] >> 32), n0, n1));
  } else {
#pragma unroll
    for (int k = 1; k < 4; k++)
      if (k < nv) stg8(o + 8 * k, (uint32_t)v[k], (uint32_t)(v[k] >> 32));
    if (nxv >= 1 && (Full || nv == 4) && lane < 63) stg8(o + 32, n0, n1);
  }
  if (lane == 0 && nv >= 1) stg8(o, (uint32_t)v[0], (uint32_t)(v[0] >> 32));
}

// One tile of the staged DBP path: positions [t0, t0 + 256) of the batch
// starting at p0 (4 consecutive positions per lane, all below p_end when
// Full), unpacked from the stage and prefix-summed on top of carry; returns
// the value after the tile.
template <bool Full>
__device__ __forceinline__ uint64_t dbp_tile(const DbpShared& sh, const PQG_L uint32_t* stw, int64_t t0, int64_t p0,
                                             int64_t p_end, bool pow2, int bs_sh, int mb_sh, int32_t bs, int32_t mbvc,
                                             uint64_t carry, bool is64, gu8 out) {
  const int lane = lane_id();
  const int64_t pb = t0 + lane * 4;
  const int nvp = Full ? 4 : (pb >= p_end ? 0 : (p_end - pb >= 4 ? 4 : (int)(p_end - pb)));
  const uint32_t rl = Full || nvp > 0 ? (uint32_t)(pb - p0) : 0u;  // < kBlocks * bs <= 2^31 (regular)
  uint32_t b, r2, m, j;
  if (pow2) {
    b = rl >> bs_sh;
    r2 = rl & (uint32_t)(bs - 1);
    m = r2 >> mb_sh;
    j = r2 & (uint32_t)(mbvc - 1);
  } else {
    b = rl / (uint32_t)bs;
    r2 = rl - b * (uint32_t)bs;
    m = r2 / (uint32_t)mbvc;
    j = r2 - m * (uint32_t)mbvc;
  }
  const PQG_L DbpShared* S = lds_ptr(&sh);
  const uint64_t wpk = S->wpk[b];
  const int wv = (int)(wpk >> (8 * m)) & 0xff;
  // bytes of the miniblocks before m: sum of widths below m, times mbvc / 8
  uint64_t lw = wpk & ((1ull << (8 * m)) - 1);  // m < 8
  lw = (lw & 0x00ff00ff00ff00ffull) + ((lw >> 8) & 0x00ff00ff00ff00ffull);
  lw += lw >> 16;
  lw += lw >> 32;
  const uint32_t bit0 = (S->sbody[b] + (uint32_t)(mbvc / 8) * ((uint32_t)lw & 0xffff)) * 8 + j * (uint32_t)wv;
  const uint64_t mnd = S->mind[b];
  const uint64_t wmask = wv == 64 ? ~0ull : ((1ull << wv) - 1);  // wv == 0: 0
  uint64_t d[4], local = 0;
  if (!__ballot(wv > 32)) {
    // widths <= 32 (every INT32 page, most INT64 ones): a value's bits lie in
    // two dwords, so two LDS reads per value instead of three
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t bt = bit0 + (uint32_t)(k * wv);
      const uint32_t dw = bt >> 5, sh5 = bt & 31;
      const uint64_t lo = (uint64_t)stw[dw] | ((uint64_t)stw[dw + 1] << 32);
      const uint64_t dv = ((lo >> sh5) & wmask) + mnd;
      d[k] = Full || k < nvp ? dv : 0;
      local += d[k];
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t bt = bit0 + (uint32_t)(k * wv);
      const uint32_t dw = bt >> 5, sh5 = bt & 31;
      const uint64_t lo = (uint64_t)stw[dw] | ((uint64_t)stw[dw + 1] << 32);
      const uint64_t x = (lo >> sh5) | (((uint64_t)stw[dw + 2] << (63 - sh5)) << 1);
      const uint64_t dv = (x & wmask) + mnd;
      d[k] = Full || k < nvp ? dv : 0;
      local += d[k];
    }
  }
  const uint64_t incl = wave_incl_scan_u64(local);
  uint64_t run = carry + (incl - local);
  if (is64) {
    uint64_t v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      v[k] = run;
      run += d[k];
    }
    store_run64<Full>((uintptr_t)(out + t0 * 8), v, nvp);
  } else {
    uint32_t dw4[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      dw4[k] = (uint32_t)run;
      run += d[k];
    }
    store_run_aligned<4>((uintptr_t)(out + t0 * 4), dw4, nvp);
  }
  const uint64_t tot = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)incl, 63) |
                       (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(incl >> 32), 63) << 32;
  return carry + tot;
}

// Values of a DBP page: emulates deltaBitPackDecoder{32,64}.next for positions
// [0, nn).  Regular layout (miniblock value count a multiple of 8, <= kMaxMb
// miniblocks): wave-parallel unpack + wrapping scan; otherwise one lane.
__device__ __forceinline__ int dbp_decode(gcu8 s, int64_t n, int64_t readable, bool is64, int64_t nn, gu8 out,
                          DbpShared& sh, int stage /*0 = header only (read phase), 1 = decode*/) {
  const int lane = lane_id();
  Window win{s, n, kFarAway, lds_ptr(sh.win)};
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
  // wave-uniform from here on (scalar registers, uniform branches)
  bs = __builtin_amdgcn_readfirstlane(bs);
  mbc = __builtin_amdgcn_readfirstlane(mbc);
  mbvc = __builtin_amdgcn_readfirstlane(mbvc);
  total = __builtin_amdgcn_readfirstlane(total);
  pos = (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)pos) |
                  (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)pos >> 32)) << 32);
  first = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)first) |
          (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(first >> 32)) << 32;
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
  const bool regular = (mbvc % 8 == 0) && mbc <= kMaxMb && bs <= (1 << 24);
  const bool pow2 = (bs & (bs - 1)) == 0 && (mbvc & (mbvc - 1)) == 0;
  const int bs_sh = __builtin_ctz((uint32_t)bs), mb_sh = __builtin_ctz((uint32_t)mbvc);
  if (!regular) {
    // ---- generic single-lane emulation of next() (rare layouts)
    int64_t rp = pos;
    int32_t cur_mb = mbc;  // force header read at position 0 semantics below
    uint64_t mind = 0, prev = first;
    uint8_t* widths = sh.gwidths;  // LDS: wave-uniform values (no scratch)
    uint64_t* vals = sh.gvals;
    int32_t cw = 0, mbpos = 0;
    for (int k = 0; k < 8; k++) vals[k] = 0;
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
        if (is64) stg8((uintptr_t)(out + p * 8), (uint32_t)prev, (uint32_t)(prev >> 32));
        else *(PQG_G uint32_t*)(out + p * 4) = (uint32_t)prev;
      }
      prev = prev + vals[p % 8] + mind;
      if (!is64) prev = (uint32_t)prev;
    }
    return kOK;
  }
  // ---- regular layout: block headers and bodies read from an LDS stage of
  // kDStage bytes, refilled with one round of loads whenever the next block is
  // not inside it; blocks walked in batches of <= kBlocks, then every position
  // of the batch unpacked from the stage and scanned.
  uint64_t carry = first;  // value at the first position of the next tile
  int64_t blk_pos = pos;   // stream offset of the next block header
  int64_t p0 = 0;          // first position of the current batch
  int64_t st_lo = kFarAway, st_hi = kFarAway;  // staged stream range (st_lo: a 16-byte aligned address)
  PQG_L uint8_t* const stb = lds_ptr(sh.stage);
  const PQG_L uint32_t* const stw = (const PQG_L uint32_t*)stb;
  const uint64_t wmask_mbc = mbc >= 8 ? ~0ull : (1ull << (8 * mbc)) - 1;
  const uint64_t wadd = 0x0101010101010101ull * (uint64_t)(127 - maxw);
  const int32_t mb_bytes_per_w = mbvc / 8;  // bytes of a miniblock per bit of width
  int64_t spec_len = 0;  // length of the last block walked one at a time (0: none, or a partial one)
#ifdef PQG_PROFILE
  uint64_t pf_rs = 0, pf_walk = 0, pf_tile = 0, pf_nrs = 0, pf_nb = 0;
#define PQG_DBP_RS(...) { PQG_T(ra_); __VA_ARGS__; PQG_T(rb_); pf_rs += rb_ - ra_; pf_nrs++; }
#else
#define PQG_DBP_RS(...) { __VA_ARGS__; }
#endif
  while (p0 < P) {
#ifdef PQG_PROFILE
    PQG_T(tw0_);
    const uint64_t rs0_ = pf_rs;
#endif
    int nb = 0;
    int64_t p_end = p0;
    bool fresh = false;  // the stage was just filled at blk_pos
    while (nb < kBlocks && p_end < P) {
      // the header (<= 10 varint bytes + mbc widths) must be staged
      if (!(blk_pos >= st_lo && blk_pos + 10 + mbc <= st_hi)) {
        if (nb > 0) break;  // decode the batch so far, then restage here
        PQG_DBP_RS(dbp_restage(s, n, stb, blk_pos, st_lo, st_hi));
        fresh = true;
      }
      // Speculative headers: lane i reads a header at blk_pos + i * spec_len
      // (spec_len: the length of the last block walked one at a time; the
      // blocks of a page are usually all the same length).  The blocks before
      // the first lane whose guess fails — a length other than spec_len, a
      // header or body not staged, a header the exact walk below would reject,
      // the batch's or the positions' end — are taken at once; a failed first
      // lane leaves that block to the exact walk.
      if (spec_len > 0) {
        const int64_t q = blk_pos + (int64_t)lane * spec_len;
        bool ok = q + spec_len <= st_hi && q + 10 + mbc <= st_hi && q + spec_len <= n && nb + lane < kBlocks &&
                  p_end + (int64_t)(lane + 1) * bs <= P;
        const uint32_t hr = (uint32_t)((ok ? q : blk_pos) - st_lo);
        uint32_t h[7];
#pragma unroll
        for (int k = 0; k < 7; k++) h[k] = stw[(hr >> 2) + k];
        const uint32_t hs = (hr & 3) * 8;
        uint64_t x0 = (uint64_t)h[0] | (uint64_t)h[1] << 32, x1 = (uint64_t)h[2] | (uint64_t)h[3] << 32;
        const uint64_t x2 = (uint64_t)h[4] | (uint64_t)h[5] << 32;
        if (hs) {
          x0 = (x0 >> hs) | (x1 << (64 - hs));
          x1 = (x1 >> hs) | (x2 << (64 - hs));
        }
        const uint64_t cont = ~x0 & 0x8080808080808080ull;
        ok = ok && cont != 0;  // a varint of <= 8 bytes
        const int vl = cont ? (int)(__builtin_ctzll(cont) >> 3) + 1 : 1;
        uint64_t t = x0 & 0x7f7f7f7f7f7f7f7full;
        t = (t & 0x007f007f007f007full) | ((t & 0x7f007f007f007f00ull) >> 1);
        t = (t & 0x00003fff00003fffull) | ((t & 0x3fff00003fff0000ull) >> 2);
        t = (t & 0x000000000fffffffull) | ((t & 0x0fffffff00000000ull) >> 4);
        const uint64_t ux = vl == 8 ? t : t & ((1ull << (7 * vl)) - 1);
        int64_t mdv = (int64_t)(ux >> 1);
        if (ux & 1) mdv = ~mdv;
        if (!is64 && (mdv > 2147483647LL || mdv < -2147483648LL)) ok = false;
        const uint32_t vs = (uint32_t)vl * 8;  // 8..64
        uint64_t wpk = vs < 64 ? (x0 >> vs) | (x1 << (64 - vs)) : x1;
        wpk &= wmask_mbc;
        if (((wpk | ((wpk & 0x7f7f7f7f7f7f7f7full) + wadd)) & 0x8080808080808080ull) != 0) ok = false;
        uint64_t sw = (wpk & 0x00ff00ff00ff00ffull) + ((wpk >> 8) & 0x00ff00ff00ff00ffull);
        sw += sw >> 16;
        sw += sw >> 32;
        const int64_t body = q + vl + mbc;
        ok = ok && body + (int64_t)mb_bytes_per_w * (int64_t)((uint32_t)sw & 0xffff) == q + spec_len;
        const uint64_t fail = __ballot(!ok);
        const int k = fail ? __ffsll((long long)fail) - 1 : 64;
        if (k > 0) {
          if (lane < k) {
            sh.mind[nb + lane] = (uint64_t)mdv;
            sh.wpk[nb + lane] = wpk;
            sh.sbody[nb + lane] = (uint32_t)(body - st_lo);
          }
          nb += k;
          p_end += (int64_t)k * bs;
          blk_pos += (int64_t)k * spec_len;
          continue;
        }
      }
      // block header (readMiniBlockHeader): its <= 10 varint bytes and <= 8
      // widths come from one read of 7 stage dwords, made wave-uniform
      const uint32_t hr = (uint32_t)(blk_pos - st_lo);
      uint32_t h[7];
#pragma unroll
      for (int k = 0; k < 7; k++) h[k] = __builtin_amdgcn_readfirstlane(stw[(hr >> 2) + k]);
      const uint32_t hs = (hr & 3) * 8;
      uint64_t x0 = (uint64_t)h[0] | (uint64_t)h[1] << 32, x1 = (uint64_t)h[2] | (uint64_t)h[3] << 32;
      uint64_t x2 = (uint64_t)h[4] | (uint64_t)h[5] << 32;
      if (hs) {
        x0 = (x0 >> hs) | (x1 << (64 - hs));
        x1 = (x1 >> hs) | (x2 << (64 - hs));
        x2 = (x2 >> hs) | ((uint64_t)h[6] << (64 - hs));
      }
      // binary.ReadUvarint: bytes at or past n are EOF; a terminator after 9
      // continuation bytes overflows (kDELTA).  Headers of <= 8 bytes (every
      // int64 delta below 2^55) are decoded branch-free from x0.
      uint64_t ux = 0;
      int vl = 0;
      const uint64_t cont = ~x0 & 0x8080808080808080ull;
      if (cont) {
        vl = (int)(__builtin_ctzll(cont) >> 3) + 1;
        if (blk_pos + vl > n) return kEOF;
        uint64_t t = x0 & 0x7f7f7f7f7f7f7f7full;
        t = (t & 0x007f007f007f007full) | ((t & 0x7f007f007f007f00ull) >> 1);
        t = (t & 0x00003fff00003fffull) | ((t & 0x3fff00003fff0000ull) >> 2);
        t = (t & 0x000000000fffffffull) | ((t & 0x0fffffff00000000ull) >> 4);
        ux = vl == 8 ? t : t & ((1ull << (7 * vl)) - 1);
      } else {
        for (;; vl++) {
          if (vl == 10) break;  // >= 10 continuation bytes: the exact walk decides
          if (blk_pos + vl >= n) return kEOF;
          const uint32_t bt = (uint32_t)((vl < 8 ? x0 >> (8 * vl) : x1 >> (8 * (vl - 8))) & 0xff);
          if (bt < 0x80) {
            if (vl == 9 && bt > 1) return kDELTA;
            ux |= (uint64_t)bt << (7 * vl);
            vl++;
            break;
          }
          ux |= (uint64_t)(bt & 0x7f) << (7 * vl);
        }
        if (vl == 10 && ((x1 >> 8) & 0x80)) {
          if (nb > 0) break;
          return dbp_decode_rest(s, n, readable, is64, nn, out, sh, P, p0, blk_pos, carry, bs, mbc, mbvc, total,
                                 pow2, bs_sh, mb_sh);
        }
      }
      int64_t mdv = (int64_t)(ux >> 1);
      if (ux & 1) mdv = ~mdv;
      if (!is64 && (mdv > 2147483647LL || mdv < -2147483648LL)) return kDELTA;
      const uint64_t md = (uint64_t)mdv;
      const int64_t hp = blk_pos + vl;
      if (n - hp < mbc) return kEOF;
      const uint32_t vs = (uint32_t)vl * 8;
      uint64_t wpk = vs == 0 ? x0 : vs < 64 ? (x0 >> vs) | (x1 << (64 - vs)) : vs == 64 ? x1
                                                                          : (x1 >> (vs - 64)) | (x2 << (128 - vs));
      wpk &= wmask_mbc;
      // a width above maxw (< 128): the byte's top bit, or its low 7 bits + (127 - maxw) carry into it
      if (((wpk | ((wpk & 0x7f7f7f7f7f7f7f7full) + wadd)) & 0x8080808080808080ull) != 0) return kBIT_WIDTH;
      uint64_t sw = (wpk & 0x00ff00ff00ff00ffull) + ((wpk >> 8) & 0x00ff00ff00ff00ffull);
      sw += sw >> 16;
      sw += sw >> 32;
      const uint32_t sumw = (uint32_t)sw & 0xffff;
      const int64_t body = hp + mbc;
      const int64_t off = body + (int64_t)mb_bytes_per_w * sumw;
      // groups of this block that positions < P read: each must be whole
      const int64_t bp0 = p_end;
      const int64_t bp1 = bp0 + bs < P ? bp0 + bs : P;
      int64_t g_end = off;
      if (bp1 - bp0 < bs) {
        const int64_t rel = ((bp1 - 1) / 8) * 8 - bp0;  // the last group read
        const int m_last = (int)(rel / mbvc);
        const int64_t g_in_mb = (rel % mbvc) / 8;
        int64_t mo = body;
        for (int m = 0; m < m_last; m++) mo += (int64_t)(mbvc / 8) * ((wpk >> (8 * m)) & 0xff);
        g_end = mo + (g_in_mb + 1) * (int64_t)((wpk >> (8 * m_last)) & 0xff);
      }
      if (g_end > n) return kEOF;
      if (g_end > st_hi) {  // the block's body is not staged
        if (nb > 0) break;
        if (fresh) return dbp_decode_rest(s, n, readable, is64, nn, out, sh, P, p0, blk_pos, carry, bs, mbc, mbvc,
                                          total, pow2, bs_sh, mb_sh);
        PQG_DBP_RS(dbp_restage(s, n, stb, blk_pos, st_lo, st_hi));
        fresh = true;
        continue;
      }
      if (lane == 0) {
        sh.mind[nb] = md;
        sh.wpk[nb] = wpk;
        sh.sbody[nb] = (uint32_t)(body - st_lo);  // stage byte of the first miniblock
      }
      nb++;
      spec_len = bp1 - bp0 == bs ? off - blk_pos : 0;
      p_end = bp1;
      blk_pos = off;
    }
    __builtin_amdgcn_wave_barrier();
#ifdef PQG_PROFILE
    PQG_T(tw1_);
    pf_walk += (tw1_ - tw0_) - (pf_rs - rs0_);
    pf_nb += nb;
#endif
    // unpack + wrapping prefix over positions [p0, p_end): value(p) = carry + sum of deltas.
    // A lane's 4 positions share one miniblock (mbvc % 8 == 0): the block /
    // miniblock split once per lane, by shifts for power-of-two sizes.
    int64_t t0 = p0;
    for (; t0 + 256 <= p_end; t0 += 256)
      carry = dbp_tile<true>(sh, stw, t0, p0, p_end, pow2, bs_sh, mb_sh, bs, mbvc, carry, is64, out);
    if (t0 < p_end) carry = dbp_tile<false>(sh, stw, t0, p0, p_end, pow2, bs_sh, mb_sh, bs, mbvc, carry, is64, out);
    __builtin_amdgcn_wave_barrier();
#ifdef PQG_PROFILE
    PQG_T(tw2_);
    pf_tile += tw2_ - tw1_;
#endif
    p0 = p_end;
  }
#ifdef PQG_PROFILE
  PQG_ACC(20, 0, pf_walk);
  PQG_ACC(21, 0, pf_rs);
  PQG_ACC(22, 0, pf_tile);
  PQG_ACC(23, 0, pf_nrs);
  PQG_ACC(24, 0, pf_nb);
#endif
#undef PQG_DBP_RS
  if (nn > total) return kEOF;
  return kOK;
}

union ValuesShared {
  ExpandShared ex;
  DbpShared dbp;
};

// Mode 1: pages of 4-byte dictionary columns only (the C2 hot path, kept
// apart so that its register budget is not the union of every encoding's);
// mode 0: every other fixed-width page; mode 3: DELTA_BINARY_PACKED.  Work
// items are the pages' parts (k_part_plan): a big page (parquet-go's writer: a
// whole chunk in one page) is decoded by many waves, one part each.
template <int Mode>
__global__ void __launch_bounds__(64, Mode == 3 ? PQG_DBP_WPE : PQG_VALUES_WPE) k_values(JobDev* jobs, PageDev* pages, const PartRec* parts, const int* total,
                                               int* queue, uint8_t* value_arena, const HStream* streams,
                                               const RunEnt* runs, const BlockDesc* blks) {
  __shared__ __attribute__((aligned(16))) ValuesShared sh;
  const int lane = lane_id();
  if (total[kModePresentOff + Mode] == 0) return;  // no page of this stage
  const int n_items = min(total[kCtrItems], total[kCtrPartsCap]);
  for (;;) {
    PQG_T(tp0);
    const int t = queue_next(queue);
    if (t >= n_items) return;
    // wave-uniform: part, page and job records are read once, by scalar loads,
    // into locals; results are written back at the end
    const PartRec pr = parts[t];
    if (pr.vmode != Mode) continue;
    const int pidx = __builtin_amdgcn_readfirstlane(pr.pidx);
    const PageDev pg = pages[pidx];
    // every data page of the list is set up by k_page_levels, which also
    // chose its values stage (vmode)
    if (pg.read_status != kOK || (pg.page_type != 0 && pg.page_type != 3) || pg.vmode != Mode) continue;
    const JobDev job = jobs[pg.job];
    if (job.status == kCAPACITY) continue;
    const bool last = pr.p + 1 >= pr.np;
    const uint32_t nx_v0 = last ? 0u : parts[t + 1].v0;
    const int nx_b0 = last ? -1 : parts[t + 1].b0;
    const gcu8 val = gconst(pg.val);
    const int64_t vn = pg.val_n;
    // readable bytes from val (for wide loads)
    int64_t readable = (pg.scratch_offset >= 0) ? vn : job.data_len - (pg.val - job.data);
    const int enc = pg.encoding;
    const int64_t nn = pg.not_null;
    // the part's values [v_lo, v_hi) (the whole page: [0, nn))
    const int64_t v_lo = pr.v0, v_hi = last ? nn : (int64_t)nx_v0;
    PQG_T(tpa);
    PQG_ACC(10 + Mode, tp0, tpa);
    const int w = job.value_width;
    const gu8 out = gmut(value_arena) + job.value_base + pg.value_offset * (int64_t)w;
    // ---- valuesDecoder.init (read phase; every part finds the same)
    int re = kOK;
    int dict_w = 0;
    if ((Mode == 0 || Mode == 1) && enc == 8) {
      if (vn < 1) re = kEOF;
      else {
        dict_w = val[0];
        if (dict_w > 32) re = kBIT_WIDTH;
      }
    } else if (Mode == 3 && enc == 5) {
      re = dbp_decode(val, vn, readable, job.type == 2, 0, nullptr, sh.dbp, 0);
    } else if (Mode == 0 && enc == 3 && job.type == 0) {
      if (vn < 4) re = kEOF;
    }
    if (re != kOK) {
      if (lane == 0) pages[pidx].read_status = re;
      continue;
    }
    if (pg.decode_status != kOK || nn == 0) continue;
    // ---- decodeValues(val[:nn]) (decode phase)
    int de = kOK;
    if (Mode == 0 && enc == 0) {
      if (job.type == 0) {  // booleanPlainDecoder: one byte per 8 values
        if ((nn + 7) / 8 > vn) de = kEOF;
        else
          for (int64_t i = v_lo + lane; i < v_hi; i += 64) out[i] = (val[i >> 3] >> (i & 7)) & 1;
      } else if (job.type == 3) {  // INT96 (type_int96.go:21-42)
        int64_t full = vn / 12, rem = vn % 12;
        if (nn > full + (rem > 0 ? 1 : 0)) de = kEOF;
        else {
          // a partial final value is left nil (Q8): its bytes are zero
          const int64_t whole = nn < full ? nn : full;
          const int64_t w_hi = v_hi < whole ? v_hi : whole;
          if (nn == full + 1 && rem > 0 && lane == 0 && whole >= v_lo && whole < v_hi) atomicOr(&pages[pidx].flags, 1);
          if (w_hi > v_lo) wave_copy(out + v_lo * 12, val + v_lo * 12, (w_hi - v_lo) * 12);
          if (whole >= v_lo && whole < v_hi && lane < 12) out[whole * 12 + lane] = 0;
        }
      } else if (w > 0) {  // INT32 / INT64 / FLOAT / DOUBLE / FLBA: little-endian bit copies
        if (nn * w > vn) de = kEOF;
        else wave_copy(out + v_lo * w, val + v_lo * w, (v_hi - v_lo) * w);
      } else {
        de = kUNSUPPORTED;  // variable length: pqg_strings.hip
      }
    } else if ((Mode == 0 || Mode == 1) && enc == 8) {
      const gcu8 dict = gconst(job.dict_data);
      const int64_t dcount = job.dict_data ? job.dict_count : 0;
      const int64_t nil_key = (job.flags & 1) ? dcount - 1 : -1;
      if (w == 0) {
        de = kUNSUPPORTED;  // variable-length dictionaries: pqg_strings.hip
      } else if (dict_w == 0) {
        // a zero-width decoder yields key 0 forever, reading nothing (hybrid_decoder.go:84-86)
        if (dcount < 1) de = kDICT_INDEX;
        else
          for (int64_t b = lane; b < nn * w; b += 64) out[b] = (0 == nil_key) ? 0 : dict[b % w];
      } else {
        const HStream S = streams[pg.hs_val];
        const int serr = (S.status != kOK && S.produced < nn) ? S.status : kOK;
        int64_t bad = nn;
        const gcu8 dsafe = dict ? dict : (gcu8)out;  // never dereferenced for a valid key when null
        const int blo = pr.b0, bhi = nx_b0;
        if (Mode == 1 || w == 4) {
          DictSink<4> sk{out, dsafe, dcount, nn, nil_key, 4};
          hybrid_expand(S, runs, blks, v_hi, sh.ex, sk, blo, bhi);
          bad = wave_min(sk.bad);
        } else if (Mode == 0 && w == 8) {
          DictSink<8> sk{out, dsafe, dcount, nn, nil_key, 8};
          hybrid_expand(S, runs, blks, v_hi, sh.ex, sk, blo, bhi);
          bad = wave_min(sk.bad);
        } else if (Mode == 0) {
          DictSink<0> sk{out, dsafe, dcount, nn, nil_key, w};
          hybrid_expand(S, runs, blks, v_hi, sh.ex, sk, blo, bhi);
          bad = wave_min(sk.bad);
        }
        // a bad key found lies before the stream's end (the expander stops
        // there): "dict: invalid index" wins over the stream's own error
        // (kDICT_INDEX is below kEOF / kRLE, so the parts' atomicMin agrees)
        if (bad < nn && (serr == kOK || bad < S.produced)) de = kDICT_INDEX;
        else de = serr;
      }
    } else if (Mode == 3 && enc == 5) {
      de = dbp_decode(val, vn, readable, job.type == 2, nn, out, sh.dbp, 1);
    } else if (Mode == 0 && enc == 3 && job.type == 0) {  // booleanRLEDecoder: hybrid w=1 after a u32 length
      const HStream S = streams[pg.hs_val];
      BoolSink sk{out};
      hybrid_expand(S, runs, blks, v_hi, sh.ex, sk, pr.b0, nx_b0);
      de = (S.status != kOK && S.produced < nn) ? S.status : kOK;
    } else {
      de = kUNSUPPORTED;
    }
    if (lane == 0 && de != kOK) atomicMin(&pages[pidx].decode_status, de);
    PQG_T(tp1);
    PQG_ACC(8 + Mode, tp0, tp1);
  }
}

template __global__ void k_values<0>(JobDev*, PageDev*, const PartRec*, const int*, int*, uint8_t*, const HStream*,
                                    const RunEnt*, const BlockDesc*);
template __global__ void k_values<1>(JobDev*, PageDev*, const PartRec*, const int*, int*, uint8_t*, const HStream*,
                                    const RunEnt*, const BlockDesc*);
template __global__ void k_values<3>(JobDev*, PageDev*, const PartRec*, const int*, int*, uint8_t*, const HStream*,
                                    const RunEnt*, const BlockDesc*);

// ============================================================================
// K5: chunk status in reference order (readPages errors first, then
// readPageData errors) — one 256-lane block per job, min-reductions over pages.
// ============================================================================
__global__ void __launch_bounds__(1024) k_finalize(JobDev* jobs, int n_jobs, PageDev* pages) {
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
#pragma unroll 8
  for (int i = threadIdx.x; i < np; i += 1024) {
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

