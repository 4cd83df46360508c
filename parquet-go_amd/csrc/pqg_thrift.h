// pqg_thrift.h — thrift compact-protocol PageHeader reader (host + device).
//
// Replaces readThrift(ph, r) (helpers.go:101-107) → PageHeader.Read
// (parquet/parquet.go:5885-6008, DataPageHeader.Read :3993-4090,
// DictionaryPageHeader.Read :4333-4400, DataPageHeaderV2.Read :4585-4722) over
// the vendored compact protocol (vendor/github.com/apache/thrift/lib/go/thrift/
// compact_protocol.go: ReadFieldBegin :385-424, readVarint64 :715-731,
// ReadListBegin :461-485; protocol.go Skip :92-176).
//
// The generic Skip is iterative (explicit frame stack) so it can run in one
// GPU lane without recursion.  Go-semantics preserved: ReadFieldBegin errors
// inside a skipped struct end that struct; a MAP value is skipped with a fresh
// depth and its error is ignored; the lastField stack is not unwound on errors.
// Limits (documented divergence for adversarial input only): 96 skip frames,
// 192 lastField entries — exceeding either is reported as a thrift error.
#pragma once
#include "pqg_common.h"

// Every method is force-inlined: a parser object whose address escapes into
// an out-of-line call lives in scratch memory on the GPU, and every byte read
// then round-trips through it.
#if defined(__HIPCC__)
#define PQG_TINLINE __host__ __device__ __attribute__((always_inline)) inline
#else
#define PQG_TINLINE inline
#endif

namespace pqg {

// the end-of-bytes shortcut of skip() (diagnostic builds may turn it off)
#ifdef PQG_NO_EOF_SKIP
constexpr bool kEofSkip = false;
#else
constexpr bool kEofSkip = true;
#endif

enum : int { T_STOP = 0, T_BOOL = 2, T_BYTE = 3, T_DOUBLE = 4, T_I16 = 6, T_I32 = 8, T_I64 = 10,
             T_STRING = 11, T_STRUCT = 12, T_MAP = 13, T_SET = 14, T_LIST = 15 };

struct SkipFrame {
  int32_t remaining;
  uint8_t kind, et, kt, vt;
  uint8_t phase;
  int8_t depth;
  uint8_t pad0, pad1;
};

constexpr int kMaxFrames = 96;
constexpr int kMaxLast = 192;

// Src must provide: int get(int64_t pos) -> byte or -1 past the end.
template <class Src>
struct Compact {
  Src src;
  int64_t pos;
  SkipFrame* frames;   // kMaxFrames
  int16_t* last;       // kMaxLast
  int nlast;
  int16_t last_id;
  bool bool_set, bool_val;
  // Stack capacities.  The serial walk uses the full kMax* limits (hitting
  // them is a thrift error); the speculative per-lane candidate parse
  // (k_page_cands) uses small stacks and reports `overflow` instead, so the
  // page is re-parsed by the serial walk rather than misclassified.
  int fcap = kMaxFrames;
  int lcap = kMaxLast;
  bool overflow = false;
  // Loop steps left (fields read plus container elements skipped): the
  // speculative candidate parse bounds its work with it (running out is
  // `overflow`, like the small stacks); the serial walk never runs out.
  int budget = 0x7fffffff;

  PQG_TINLINE int byte(uint8_t* b) {
    int v = src.get(pos);
    if (v < 0) return -1;
    pos++;
    *b = (uint8_t)v;
    return 0;
  }
  PQG_TINLINE int varint64(int64_t* out) {
    unsigned shift = 0;
    uint64_t r = 0;
    for (;;) {
      uint8_t b;
      if (byte(&b)) return -1;
      if (shift < 64) r |= (uint64_t)(b & 0x7f) << shift;
      if (!(b & 0x80)) break;
      shift += 7;
    }
    *out = (int64_t)r;
    return 0;
  }
  PQG_TINLINE int i32(int32_t* out) {
    int64_t v;
    if (varint64(&v)) return -1;
    int32_t n = (int32_t)v;
    *out = (int32_t)((uint32_t)n >> 1) ^ -(n & 1);
    return 0;
  }
  PQG_TINLINE int i64(int64_t* out) {
    int64_t v;
    if (varint64(&v)) return -1;
    *out = (int64_t)((uint64_t)v >> 1) ^ -(v & 1);
    return 0;
  }
  PQG_TINLINE static int ttype(int t) {  // getTType; -1 = unknown
    switch (t & 0x0f) {
      case 0: return T_STOP;
      case 1: case 2: return T_BOOL;
      case 3: return T_BYTE;
      case 4: return T_I16;
      case 5: return T_I32;
      case 6: return T_I64;
      case 7: return T_DOUBLE;
      case 8: return T_STRING;
      case 9: return T_LIST;
      case 10: return T_SET;
      case 11: return T_MAP;
      case 12: return T_STRUCT;
    }
    return -1;
  }
  PQG_TINLINE int struct_begin() {
    if (nlast >= lcap) {
      if (lcap < kMaxLast) overflow = true;
      return -1;
    }
    last[nlast++] = last_id;
    last_id = 0;
    return 0;
  }
  PQG_TINLINE void struct_end() {
    if (nlast > 0) last_id = last[--nlast];
  }
  // ReadFieldBegin: returns 0 ok / -1 error; *type = T_STOP on error.
  PQG_TINLINE int field_begin(int* type, int* id) {
    *type = T_STOP;
    *id = 0;
    uint8_t t;
    if (byte(&t)) return -1;
    if ((t & 0x0f) == 0) return 0;
    int16_t mod = (int16_t)((t & 0xf0) >> 4);
    int16_t fid;
    if (mod == 0) {
      int32_t v;
      if (i32(&v)) return -1;
      fid = (int16_t)v;
    } else {
      fid = (int16_t)(last_id + mod);
    }
    int tt = ttype(t);
    if (tt < 0) {
      *id = fid;
      return -1;
    }
    if ((t & 0x0f) == 1 || (t & 0x0f) == 2) {
      bool_val = (t & 0x0f) == 1;
      bool_set = true;
    }
    last_id = fid;
    *type = tt;
    *id = fid;
    return 0;
  }
  PQG_TINLINE int read_bool(bool* v) {
    if (bool_set) {
      bool_set = false;
      *v = bool_val;
      return 0;
    }
    uint8_t b;
    if (byte(&b)) return -1;
    *v = b == 1;
    return 0;
  }
  PQG_TINLINE int binary_skip() {
    int64_t v;
    if (varint64(&v)) return -1;
    int32_t len = (int32_t)v;
    if (len < 0) return -1;
    if (len == 0) return 0;
    if (src.get(pos + len - 1) < 0) {  // io.ReadFull short
      pos += len;
      return -1;
    }
    pos += len;
    return 0;
  }
  // Start processing one value of `type` at `depth`: primitives complete
  // immediately; containers push a frame.  Returns 0 / -1.
  PQG_TINLINE int start_value(int type, int depth, int* nf) {
    if (depth <= 0) return -1;
    switch (type) {
      case T_BOOL: { bool b; return read_bool(&b); }
      case T_BYTE: { uint8_t b; return byte(&b); }
      case T_I16: case T_I32: { int32_t v; return i32(&v); }
      case T_I64: { int64_t v; return i64(&v); }
      case T_DOUBLE:
        if (src.get(pos + 7) < 0) { pos += 8; return -1; }
        pos += 8;
        return 0;
      case T_STRING: return binary_skip();
      case T_STRUCT: {
        if (*nf >= fcap) { if (fcap < kMaxFrames) overflow = true; return -1; }
        if (struct_begin()) return -1;
        SkipFrame& f = frames[(*nf)++];
        f.kind = T_STRUCT;
        f.depth = (int8_t)depth;
        f.remaining = 0;
        f.phase = 0;
        return 0;
      }
      case T_MAP: {
        int64_t v;
        if (varint64(&v)) return -1;
        int32_t size = (int32_t)v;
        if (size < 0) return -1;
        uint8_t kv = 0;
        if (size != 0 && byte(&kv)) return -1;
        if (*nf >= fcap) { if (fcap < kMaxFrames) overflow = true; return -1; }
        SkipFrame& f = frames[(*nf)++];
        f.kind = T_MAP;
        f.depth = (int8_t)depth;
        f.remaining = size;
        int kt = ttype(kv >> 4), vt = ttype(kv & 0xf);
        f.kt = (uint8_t)(kt < 0 ? T_STOP : kt);
        f.vt = (uint8_t)(vt < 0 ? T_STOP : vt);
        f.phase = 0;
        return 0;
      }
      case T_SET: case T_LIST: {
        uint8_t st;
        if (byte(&st)) return -1;
        int32_t size = (st >> 4) & 0x0f;
        if (size == 15) {
          int64_t v;
          if (varint64(&v)) return -1;
          size = (int32_t)v;
          if (size < 0) return -1;
        }
        int et = ttype(st);
        if (et < 0) return -1;
        if (*nf >= fcap) { if (fcap < kMaxFrames) overflow = true; return -1; }
        SkipFrame& f = frames[(*nf)++];
        f.kind = T_LIST;
        f.depth = (int8_t)depth;
        f.remaining = size;
        f.et = (uint8_t)et;
        f.phase = 0;
        return 0;
      }
    }
    return -1;  // STOP / unknown: "Unknown data type"
  }
  // protocol.go Skip(fieldType, depth) — iterative: start_value, then
  // skip_step until the value's frames are all closed.
  PQG_TINLINE int skip(int type, int depth) {
    int nf = 0;
    int e = start_value(type, depth, &nf);
    for (;;) {
      const int r = skip_step(nf, e);
      if (r <= 0) return r;
    }
  }
  // One step of Skip: 1 = more to do, 0 = the value is skipped, -1 = error.
  // `e`: the error of the previous step's start_value (unwinds to the nearest
  // MAP frame whose value is in flight: that error is ignored).
  PQG_TINLINE int skip_step(int& nf, int& e) {
    if (--budget < 0) {
      overflow = true;
      return -1;
    }
    if (e) {
      while (nf > 0 && !(frames[nf - 1].kind == T_MAP && frames[nf - 1].phase == 2)) nf--;
      if (nf == 0) return -1;
      e = 0;
    }
    if (nf == 0) return 0;
    SkipFrame& f = frames[nf - 1];
    if (f.kind == T_STRUCT) {
      int t, id;
      field_begin(&t, &id);  // error => STOP
      if (t == T_STOP) {
        struct_end();
        nf--;
        return 1;
      }
      e = start_value(t, f.depth - 1, &nf);
    } else if (f.kind == T_LIST) {
      if (f.remaining <= 0) {
        nf--;
        return 1;
      }
      // At the end of the bytes a STRUCT element is a no-op (its
      // ReadFieldBegin fails, the error is ignored: STOP), and so is every
      // element after it: the rest of the list is skipped in one step
      // instead of up to 2^31 (a garbage header with a huge list size would
      // otherwise spin one lane for seconds).  Only where the element would
      // have pushed its frame and lastField entry without hitting a limit.
      if (kEofSkip && f.et == T_STRUCT && f.depth > 1 && nf < fcap && nlast < lcap && src.get(pos) < 0) {
        nf--;
        return 1;
      }
      f.remaining--;
      e = start_value(f.et, f.depth - 1, &nf);
    } else {  // MAP
      if (f.phase == 2) f.phase = 0;
      if (f.phase == 0) {
        if (f.remaining <= 0) {
          nf--;
          return 1;
        }
        // the same for STRUCT keys at the end of the bytes when the value is
        // not a container (its error is ignored, it leaves no state)
        if (kEofSkip && f.kt == T_STRUCT && f.vt != T_STRUCT && f.vt != T_MAP && f.vt != T_SET && f.vt != T_LIST &&
            f.depth > 1 && nf < fcap && nlast < lcap && src.get(pos) < 0) {
          nf--;
          return 1;
        }
        f.remaining--;
        f.phase = 1;
        e = start_value(f.kt, f.depth - 1, &nf);
      } else {
        f.phase = 2;
        e = start_value(f.vt, 64, &nf);  // self.Skip(valueType): fresh depth, error ignored
        if (e) e = 0;                    // a direct primitive error is swallowed here
      }
    }
    return 1;
  }
  // PageHeader.Read (parquet.go:5885-6008) with the nested readers it calls —
  // DataPageHeader.Read :3993-4090, IndexPageHeader (no fields),
  // DictionaryPageHeader.Read :4333-4400, DataPageHeaderV2.Read :4585-4722 and
  // Statistics.Read — as ONE loop over a stack of known structs.  Every
  // field of every known struct goes through the same field_begin / read /
  // skip code, so the generic skip() is inlined once (nested readers with a
  // skip() each made k_cand_parse ~100K instructions: the instruction cache,
  // not the bytes, set its speed).  Per known struct: a field of the
  // expected id and type is read (i32 kept, bool / i64 / binary read and
  // dropped), any other field is skipped; ReadFieldBegin errors, read errors
  // and skip errors fail the header; at STOP the struct's required fields
  // must have been seen ("Required field ... is not set").
  enum : int { S_PH = 0, S_DPH = 1, S_IDX = 2, S_DICT = 3, S_V2 = 4, S_STAT = 5 };
  enum : int { A_SKIP = 0, A_I32 = 1, A_BOOL = 2, A_I64 = 3, A_BIN = 4, A_STRUCT = 5 };
  PQG_TINLINE int read_page_header(PageHdr* h) {
    int64_t start = pos;
    h->type = h->usize = h->csize = 0;
    h->num_values = h->encoding = h->def_enc = h->rep_enc = 0;
    h->v2_def_len = h->v2_rep_len = 0;
    h->has_dph = h->has_dict = h->has_v2 = 0;
    // known-struct stack (PageHeader -> DPH / V2 -> Statistics: depth <= 3),
    // held as packed scalars (no dynamically indexed local arrays)
    uint32_t schs = S_PH;  // 4 bits per level
    uint32_t seen = 0;     // required fields of the innermost struct
    uint32_t seen_up = 0;  // 8 bits per enclosing level
    int depth = 1;
    // a field being skipped: its frames and pending error (skip_step)
    int nf = 0, se = 0;
    bool skipping = false;
    if (struct_begin()) return kTHRIFT;
    // ONE loop for both kinds of step: lanes of a wave parsing different
    // candidates then step together (nested loops would run one lane's skip
    // while the others wait, and the next lane's after it)
    for (;;) {
      if (skipping) {
        const int r = skip_step(nf, se);
        if (r < 0) return kTHRIFT;
        skipping = r > 0;
        continue;
      }
      int t, id;
      if (--budget < 0) {
        overflow = true;
        return kTHRIFT;
      }
      if (field_begin(&t, &id)) return kTHRIFT;
      const int sc = (int)((schs >> (4 * (depth - 1))) & 0xf);
      if (t == T_STOP) {
        struct_end();
        const uint32_t need = sc == S_PH ? 7u : sc == S_DPH ? 15u : sc == S_DICT ? 3u : sc == S_V2 ? 63u : 0u;
        if ((seen & need) != need) return kTHRIFT;
        if (--depth == 0) break;
        seen = seen_up & 0xff;
        seen_up >>= 8;
        continue;
      }
      // the field's action in its struct: A_I32 into slot `slot` (required
      // bit `bit`), A_STRUCT into schema `child`, or a read / skip
      int act = A_SKIP, slot = -1, child = 0;
      uint32_t bit = 0;
      if (sc == S_PH) {
        if (id >= 1 && id <= 4 && t == T_I32) { act = A_I32; slot = id - 1; bit = id <= 3 ? 1u << (id - 1) : 0u; }
        else if (id == 5 && t == T_STRUCT) { act = A_STRUCT; child = S_DPH; }
        else if (id == 6 && t == T_STRUCT) { act = A_STRUCT; child = S_IDX; }
        else if (id == 7 && t == T_STRUCT) { act = A_STRUCT; child = S_DICT; }
        else if (id == 8 && t == T_STRUCT) { act = A_STRUCT; child = S_V2; }
      } else if (sc == S_DPH) {
        if (id >= 1 && id <= 4 && t == T_I32) { act = A_I32; slot = 3 + id; bit = 1u << (id - 1); }
        else if (id == 5 && t == T_STRUCT) { act = A_STRUCT; child = S_STAT; }
      } else if (sc == S_DICT) {
        if (id >= 1 && id <= 2 && t == T_I32) { act = A_I32; slot = 3 + id; bit = 1u << (id - 1); }
        else if (id == 3 && t == T_BOOL) act = A_BOOL;
      } else if (sc == S_V2) {
        if (id >= 1 && id <= 6 && t == T_I32) { act = A_I32; slot = 8 + id; bit = 1u << (id - 1); }
        else if (id == 7 && t == T_BOOL) act = A_BOOL;  // IsCompressed: ignored (Q4)
        else if (id == 8 && t == T_STRUCT) { act = A_STRUCT; child = S_STAT; }
      } else if (sc == S_STAT) {
        if ((id == 1 || id == 2 || id == 5 || id == 6) && t == T_STRING) act = A_BIN;
        else if ((id == 3 || id == 4) && t == T_I64) act = A_I64;
      }
      if (act == A_STRUCT) {
        if (struct_begin()) return kTHRIFT;
        if (child == S_DPH) h->has_dph = 1;
        if (child == S_DICT) h->has_dict = 1;
        if (child == S_V2) h->has_v2 = 1;
        schs = (schs & ~(0xfu << (4 * depth))) | ((uint32_t)child << (4 * depth));
        seen_up = (seen_up << 8) | (seen & 0xff);
        seen = 0;
        depth++;
        continue;
      }
      int e;
      if (act == A_I32) {
        int32_t v = 0;
        e = i32(&v);
        seen |= bit;
        if (!e) switch (slot) {  // a failed read leaves the field as it was  // 0-3 PageHeader, 4-7 DPH, 5-6 dictionary, 9-14 V2
          case 0: h->type = v; break;
          case 1: h->usize = v; break;
          case 2: h->csize = v; break;
          case 4: case 9: h->num_values = v; break;
          case 5: case 12: h->encoding = v; break;
          case 6: h->def_enc = v; break;
          case 7: h->rep_enc = v; break;
          case 13: h->v2_def_len = v; break;
          case 14: h->v2_rep_len = v; break;
          default: break;  // crc, num_nulls, num_rows
        }
      } else if (act == A_BOOL) {
        bool b;
        e = read_bool(&b);
      } else if (act == A_I64) {
        int64_t v;
        e = i64(&v);
      } else if (act == A_BIN) {
        e = binary_skip();
      } else {
        // Skip(t): a primitive is read here; a container's frames are
        // stepped by the loop (a failed start pushes no frame: error)
        nf = 0;
        se = start_value(t, 64, &nf);
        if (se) return kTHRIFT;
        skipping = nf > 0;
        continue;
      }
      if (e) return kTHRIFT;
    }
    h->hlen = (int32_t)(pos - start);
    return kOK;
  }
};

}  // namespace pqg
