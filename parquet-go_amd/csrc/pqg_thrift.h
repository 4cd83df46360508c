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
  // protocol.go Skip(fieldType, depth) — iterative.
  PQG_TINLINE int skip(int type, int depth) {
    int nf = 0;
    int e = start_value(type, depth, &nf);
    for (;;) {
      if (e) {  // unwind to the nearest MAP frame whose value is in flight
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
          continue;
        }
        e = start_value(t, f.depth - 1, &nf);
      } else if (f.kind == T_LIST) {
        if (f.remaining <= 0) {
          nf--;
          continue;
        }
        f.remaining--;
        e = start_value(f.et, f.depth - 1, &nf);
      } else {  // MAP
        if (f.phase == 2) f.phase = 0;
        if (f.phase == 0) {
          if (f.remaining <= 0) {
            nf--;
            continue;
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
    }
  }
  // Statistics.Read: binary 1,2,5,6; i64 3,4.
  PQG_TINLINE int read_statistics() {
    if (struct_begin()) return -1;
    for (;;) {
      int t, id;
      if (field_begin(&t, &id)) return -1;
      if (t == T_STOP) break;
      int e;
      if ((id == 1 || id == 2 || id == 5 || id == 6) && t == T_STRING) {
        e = binary_skip();
      } else if ((id == 3 || id == 4) && t == T_I64) {
        int64_t v;
        e = i64(&v);
      } else {
        e = skip(t, 64);
      }
      if (e) return -1;
    }
    struct_end();
    return 0;
  }
  PQG_TINLINE int read_page_header(PageHdr* h) {
    int64_t start = pos;
    h->type = h->usize = h->csize = 0;
    h->num_values = h->encoding = h->def_enc = h->rep_enc = 0;
    h->v2_def_len = h->v2_rep_len = 0;
    h->has_dph = h->has_dict = h->has_v2 = 0;
    bool st = false, su = false, sc = false;
    if (struct_begin()) return kTHRIFT;
    for (;;) {
      int t, id;
      if (field_begin(&t, &id)) return kTHRIFT;
      if (t == T_STOP) break;
      int e = 0;
      bool handled = false;
      switch (id) {
        case 1: if (t == T_I32) { handled = true; st = true; e = i32(&h->type); } break;
        case 2: if (t == T_I32) { handled = true; su = true; e = i32(&h->usize); } break;
        case 3: if (t == T_I32) { handled = true; sc = true; e = i32(&h->csize); } break;
        case 4: if (t == T_I32) { handled = true; int32_t crc; e = i32(&crc); } break;
        case 5:
          if (t == T_STRUCT) {
            handled = true;
            h->has_dph = 1;
            e = read_dph(h);
          }
          break;
        case 6:
          if (t == T_STRUCT) {  // IndexPageHeader has no fields: every field is skipped
            handled = true;
            if (struct_begin()) return kTHRIFT;
            for (;;) {
              int t2, id2;
              if (field_begin(&t2, &id2)) return kTHRIFT;
              if (t2 == T_STOP) break;
              if (skip(t2, 64)) return kTHRIFT;
            }
            struct_end();
          }
          break;
        case 7:
          if (t == T_STRUCT) {
            handled = true;
            h->has_dict = 1;
            e = read_dict(h);
          }
          break;
        case 8:
          if (t == T_STRUCT) {
            handled = true;
            h->has_v2 = 1;
            e = read_v2(h);
          }
          break;
      }
      if (!handled) e = skip(t, 64);
      if (e) return kTHRIFT;
    }
    struct_end();
    if (!st || !su || !sc) return kTHRIFT;  // "Required field ... is not set"
    h->hlen = (int32_t)(pos - start);
    return kOK;
  }
  PQG_TINLINE int read_dph(PageHdr* h) {
    if (struct_begin()) return -1;
    bool a = false, b = false, c = false, d = false;
    for (;;) {
      int t, id;
      if (field_begin(&t, &id)) return -1;
      if (t == T_STOP) break;
      int e;
      if (id == 1 && t == T_I32) { a = true; e = i32(&h->num_values); }
      else if (id == 2 && t == T_I32) { b = true; e = i32(&h->encoding); }
      else if (id == 3 && t == T_I32) { c = true; e = i32(&h->def_enc); }
      else if (id == 4 && t == T_I32) { d = true; e = i32(&h->rep_enc); }
      else if (id == 5 && t == T_STRUCT) e = read_statistics();
      else e = skip(t, 64);
      if (e) return -1;
    }
    struct_end();
    return (a && b && c && d) ? 0 : -1;
  }
  PQG_TINLINE int read_dict(PageHdr* h) {
    if (struct_begin()) return -1;
    bool a = false, b = false;
    for (;;) {
      int t, id;
      if (field_begin(&t, &id)) return -1;
      if (t == T_STOP) break;
      int e;
      if (id == 1 && t == T_I32) { a = true; e = i32(&h->num_values); }
      else if (id == 2 && t == T_I32) { b = true; e = i32(&h->encoding); }
      else if (id == 3 && t == T_BOOL) { bool s; e = read_bool(&s); }
      else e = skip(t, 64);
      if (e) return -1;
    }
    struct_end();
    return (a && b) ? 0 : -1;
  }
  PQG_TINLINE int read_v2(PageHdr* h) {
    if (struct_begin()) return -1;
    unsigned seen = 0;
    for (;;) {
      int t, id;
      if (field_begin(&t, &id)) return -1;
      if (t == T_STOP) break;
      int e;
      int32_t dummy;
      if (id == 1 && t == T_I32) { seen |= 1; e = i32(&h->num_values); }
      else if (id == 2 && t == T_I32) { seen |= 2; e = i32(&dummy); }
      else if (id == 3 && t == T_I32) { seen |= 4; e = i32(&dummy); }
      else if (id == 4 && t == T_I32) { seen |= 8; e = i32(&h->encoding); }
      else if (id == 5 && t == T_I32) { seen |= 16; e = i32(&h->v2_def_len); }
      else if (id == 6 && t == T_I32) { seen |= 32; e = i32(&h->v2_rep_len); }
      else if (id == 7 && t == T_BOOL) { bool s; e = read_bool(&s); }  // IsCompressed: ignored (Q4)
      else if (id == 8 && t == T_STRUCT) e = read_statistics();
      else e = skip(t, 64);
      if (e) return -1;
    }
    struct_end();
    return seen == 63 ? 0 : -1;
  }
};

}  // namespace pqg
