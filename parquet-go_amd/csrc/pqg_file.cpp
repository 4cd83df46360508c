// pqg_file.cpp — host-side planner: footer + schema → column-chunk jobs.
//
// Replaces readFileMetaData (file_meta.go:14-62) and makeSchema / readSchema /
// readGroupSchema / readColumnSchema (schema.go:789-919, 996-1025): PAR1 magic
// at both ends, i32 LE footer length (> 0), thrift FileMetaData, then leaf
// columns in depth-first order with maxD (+1 per non-REQUIRED element) and maxR
// (+1 per REPEATED element).  Row group r's chunk for leaf i is
// RowGroup.columns[i] (readRowGroup chunk_reader.go:404-431).
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/pqgpu.h"
#include "pqg_thrift.h"

using namespace pqg;

namespace {

struct MemSrc {
  const uint8_t* p;
  int64_t n;
  int get(int64_t i) const { return (i >= 0 && i < n) ? p[i] : -1; }
};

struct Elem {
  bool has_type = false, has_tl = false, has_rep = false, has_nc = false, has_ct = false;
  int32_t type = 0, type_length = 0, rep = 0, num_children = 0, converted = 0;
  bool unsigned_int = false;
  std::string name;
};

struct ChunkM {
  bool has_meta = false, has_path = false, has_dict = false;
  int32_t type = 0, codec = 0;
  int64_t num_values = 0, tus = 0, tcs = 0, data_off = 0, dict_off = 0;
};

struct Leaf {
  pqg_column_desc desc;
  std::string path;
};

struct Parser {
  Compact<MemSrc> c;
  SkipFrame frames[kMaxFrames];
  int16_t last[kMaxLast];
  explicit Parser(const uint8_t* p, int64_t n) {
    c.src = MemSrc{p, n};
    c.pos = 0;
    c.frames = frames;
    c.last = last;
    c.nlast = 0;
    c.last_id = 0;
    c.bool_set = c.bool_val = false;
  }
  bool str(std::string* out) {
    int64_t v;
    if (c.varint64(&v)) return false;
    int32_t len = (int32_t)v;
    if (len < 0) return false;
    if (len == 0) {
      out->clear();
      return true;
    }
    if (c.src.get(c.pos + len - 1) < 0) return false;
    out->assign((const char*)c.src.p + c.pos, (size_t)len);
    c.pos += len;
    return true;
  }
  bool list(int* et, int32_t* size) {
    uint8_t st;
    if (c.byte(&st)) return false;
    int32_t sz = (st >> 4) & 0x0f;
    if (sz == 15) {
      int64_t v;
      if (c.varint64(&v)) return false;
      sz = (int32_t)v;
      if (sz < 0) return false;
    }
    int t = Compact<MemSrc>::ttype(st);
    if (t < 0) return false;
    *et = t;
    *size = sz;
    return true;
  }
  // generic field loop
  template <class F>
  bool fields(F&& f) {
    if (c.struct_begin()) return false;
    for (;;) {
      int t, id;
      if (c.field_begin(&t, &id)) return false;
      if (t == T_STOP) break;
      int r = f(t, id);  // 1 handled ok, 0 not handled, -1 error
      if (r < 0) return false;
      if (r == 0 && c.skip(t, 64)) return false;
    }
    c.struct_end();
    return true;
  }
  bool logical_unsigned(bool* uns) {
    // LogicalType union; INTEGER = field 10: IntType{1: bitWidth byte, 2: isSigned bool}
    return fields([&](int t, int id) -> int {
      if (id == 10 && t == T_STRUCT) {
        bool ok = fields([&](int t2, int id2) -> int {
          if (id2 == 2 && t2 == T_BOOL) {
            bool s;
            if (c.read_bool(&s)) return -1;
            *uns = !s;
            return 1;
          }
          return 0;
        });
        return ok ? 1 : -1;
      }
      return 0;
    });
  }
  bool elem(Elem* e) {
    return fields([&](int t, int id) -> int {
      int32_t v;
      switch (id) {
        case 1: if (t == T_I32) { if (c.i32(&v)) return -1; e->type = v; e->has_type = true; return 1; } break;
        case 2: if (t == T_I32) { if (c.i32(&v)) return -1; e->type_length = v; e->has_tl = true; return 1; } break;
        case 3: if (t == T_I32) { if (c.i32(&v)) return -1; e->rep = v; e->has_rep = true; return 1; } break;
        case 4: if (t == T_STRING) { return str(&e->name) ? 1 : -1; } break;
        case 5: if (t == T_I32) { if (c.i32(&v)) return -1; e->num_children = v; e->has_nc = true; return 1; } break;
        case 6: if (t == T_I32) { if (c.i32(&v)) return -1; e->converted = v; e->has_ct = true; return 1; } break;
        case 10: if (t == T_STRUCT) { return logical_unsigned(&e->unsigned_int) ? 1 : -1; } break;
      }
      return 0;
    });
  }
  bool meta(ChunkM* m) {
    return fields([&](int t, int id) -> int {
      int32_t v;
      int64_t w;
      switch (id) {
        case 1: if (t == T_I32) { if (c.i32(&v)) return -1; m->type = v; return 1; } break;
        case 4: if (t == T_I32) { if (c.i32(&v)) return -1; m->codec = v; return 1; } break;
        case 5: if (t == T_I64) { if (c.i64(&w)) return -1; m->num_values = w; return 1; } break;
        case 6: if (t == T_I64) { if (c.i64(&w)) return -1; m->tus = w; return 1; } break;
        case 7: if (t == T_I64) { if (c.i64(&w)) return -1; m->tcs = w; return 1; } break;
        case 9: if (t == T_I64) { if (c.i64(&w)) return -1; m->data_off = w; return 1; } break;
        case 11: if (t == T_I64) { if (c.i64(&w)) return -1; m->dict_off = w; m->has_dict = true; return 1; } break;
      }
      return 0;
    });
  }
  bool chunk(ChunkM* m) {
    return fields([&](int t, int id) -> int {
      if (id == 1 && t == T_STRING) {
        std::string s;
        if (!str(&s)) return -1;
        m->has_path = true;
        return 1;
      }
      if (id == 3 && t == T_STRUCT) {
        m->has_meta = true;
        return meta(m) ? 1 : -1;
      }
      return 0;
    });
  }
};

}  // namespace

struct SNode {
  std::string name;
  int32_t rep, num_children, leaf, max_def, max_rep;
};

struct pqg_file {
  std::vector<Leaf> leaves;
  std::vector<SNode> nodes;  // schema tree below the root, depth first
  std::vector<std::vector<ChunkM>> rgs;
  std::vector<int64_t> rg_rows;
  int64_t num_rows = 0;
};

namespace {

// schema.go:789-894 (readColumnSchema / readGroupSchema), depth-first.
bool read_schema(const std::vector<Elem>& s, size_t& idx, const std::string& name, int d, int r,
                 std::vector<Leaf>& out, int depth, std::vector<SNode>& nodes) {
  if (depth > 256 || idx >= s.size()) return false;
  const Elem& e = s[idx];
  if (!e.has_type) {  // group
    if (!e.has_nc || e.num_children <= 0) return false;
    if (s.size() <= idx + (size_t)e.num_children) return false;
    if (e.has_rep && e.rep != 0) d++;
    if (e.has_rep && e.rep == 2) r++;
    std::string nm = name.empty() ? e.name : name + "." + e.name;
    nodes.push_back(SNode{e.name, e.has_rep ? e.rep : 0, e.num_children, -1, d, r});
    idx++;
    for (int i = 0; i < e.num_children; i++)
      if (!read_schema(s, idx, nm, d, r, out, depth + 1, nodes)) return false;
    return true;
  }
  if (e.name.empty() || !e.has_rep) return false;
  if (e.rep != 0) d++;
  if (e.rep == 2) r++;
  if (e.type == 7 && !e.has_tl) return false;  // getValuesStore: nil type len
  if (e.type < 0 || e.type > 7) return false;
  Leaf l;
  memset(&l.desc, 0, sizeof(l.desc));
  l.desc.physical_type = e.type;
  l.desc.type_length = e.has_tl ? e.type_length : -1;
  l.desc.max_def = d;
  l.desc.max_rep = r;
  bool uns = e.unsigned_int;
  if (e.has_ct && ((e.type == 1 && (e.converted == 11 || e.converted == 12 || e.converted == 13)) ||
                   (e.type == 2 && e.converted == 14)))
    uns = true;
  l.desc.flags = uns ? 1 : 0;
  l.path = name.empty() ? e.name : name + "." + e.name;
  nodes.push_back(SNode{e.name, e.rep, 0, (int32_t)out.size(), d, r});
  out.push_back(l);
  idx++;
  return true;
}

}  // namespace

extern "C" {

static int open_footer(const uint8_t* footer, int32_t fl, pqg_file** out);

int pqg_file_open(const uint8_t* file, int64_t len, pqg_file** out) {
  if (!file || !out || len < 0) return PQG_ERR_INVALID_ARG;
  return pqg_file_open_tail(file, len, file, len, len, out);
}

// readFileMetaData (file_meta.go:14-62) from the file's first bytes and its
// last tail_len bytes only: what a range reader fetches before planning.
int pqg_file_open_tail(const uint8_t* head, int64_t head_len, const uint8_t* tail, int64_t tail_len, int64_t file_len,
                       pqg_file** out) {
  if (!head || !tail || !out || head_len < 0 || tail_len < 0 || file_len < 0 || tail_len > file_len)
    return PQG_ERR_INVALID_ARG;
  *out = nullptr;
  if (head_len < 4 || memcmp(head, "PAR1", 4) != 0) return PQG_ERR_METADATA;
  if (tail_len < 8 || memcmp(tail + tail_len - 4, "PAR1", 4) != 0) return PQG_ERR_METADATA;
  int32_t fl;
  memcpy(&fl, tail + tail_len - 8, 4);
  if (fl <= 0) return PQG_ERR_METADATA;
  if ((int64_t)fl + 8 > file_len) return PQG_ERR_METADATA;
  if ((int64_t)fl + 8 > tail_len) return PQG_ERR_INVALID_ARG;  // fetch the last fl + 8 bytes
  return open_footer(tail + tail_len - 8 - fl, fl, out);
}

static int open_footer(const uint8_t* footer, int32_t fl, pqg_file** out) {
  Parser P(footer, fl);
  std::vector<Elem> schema;
  std::vector<std::vector<ChunkM>> rgs;
  std::vector<int64_t> rg_rows;
  int64_t num_rows = 0;
  bool ok = P.fields([&](int t, int id) -> int {
    if (id == 2 && t == T_LIST) {
      int et;
      int32_t n;
      if (!P.list(&et, &n) || et != T_STRUCT) return -1;
      for (int32_t i = 0; i < n; i++) {
        Elem e;
        if (!P.elem(&e)) return -1;
        schema.push_back(e);
      }
      return 1;
    }
    if (id == 3 && t == T_I64) return P.c.i64(&num_rows) ? -1 : 1;
    if (id == 4 && t == T_LIST) {
      int et;
      int32_t n;
      if (!P.list(&et, &n) || et != T_STRUCT) return -1;
      for (int32_t i = 0; i < n; i++) {
        std::vector<ChunkM> cols;
        int64_t rows = 0;
        bool okr = P.fields([&](int t2, int id2) -> int {
          if (id2 == 1 && t2 == T_LIST) {
            int et2;
            int32_t n2;
            if (!P.list(&et2, &n2) || et2 != T_STRUCT) return -1;
            for (int32_t k = 0; k < n2; k++) {
              ChunkM m;
              if (!P.chunk(&m)) return -1;
              cols.push_back(m);
            }
            return 1;
          }
          if (id2 == 3 && t2 == T_I64) return P.c.i64(&rows) ? -1 : 1;
          return 0;
        });
        if (!okr) return -1;
        rgs.push_back(cols);
        rg_rows.push_back(rows);
      }
      return 1;
    }
    return 0;
  });
  if (!ok || schema.empty()) return PQG_ERR_METADATA;
  pqg_file* f = new pqg_file();
  size_t idx = 1;  // makeSchema: readSchema(meta.Schema[1:])
  while (idx < schema.size()) {
    if (!read_schema(schema, idx, "", 0, 0, f->leaves, 0, f->nodes)) {
      delete f;
      return PQG_ERR_METADATA;
    }
  }
  f->rgs = rgs;
  f->rg_rows = rg_rows;
  f->num_rows = num_rows;
  *out = f;
  return PQG_OK;
}

void pqg_file_close(pqg_file* f) { delete f; }
int pqg_file_num_columns(const pqg_file* f) { return f ? (int)f->leaves.size() : 0; }
int pqg_file_num_row_groups(const pqg_file* f) { return f ? (int)f->rgs.size() : 0; }
int64_t pqg_file_num_rows(const pqg_file* f) { return f ? f->num_rows : 0; }
int64_t pqg_file_row_group_rows(const pqg_file* f, int rg) {
  if (!f || rg < 0 || rg >= (int)f->rgs.size()) return -1;
  return f->rg_rows[(size_t)rg];
}

int pqg_file_num_schema_nodes(const pqg_file* f) { return f ? (int)f->nodes.size() : PQG_ERR_INVALID_ARG; }

int pqg_file_schema_node(const pqg_file* f, int i, pqg_schema_node* out) {
  if (!f || !out || i < 0 || i >= (int)f->nodes.size()) return PQG_ERR_INVALID_ARG;
  memset(out, 0, sizeof(*out));
  const SNode& n = f->nodes[(size_t)i];
  // the name is the row's map key (Column.name): never hand out a truncated one
  if (n.name.size() >= sizeof(out->name)) return PQG_ERR_METADATA;
  snprintf(out->name, sizeof(out->name), "%s", n.name.c_str());
  out->repetition = n.rep;
  out->num_children = n.num_children;
  out->leaf = n.leaf;
  out->max_def = n.max_def;
  out->max_rep = n.max_rep;
  return PQG_OK;
}

int pqg_file_column(const pqg_file* f, int col, pqg_column_info* out) {
  if (!f || !out || col < 0 || col >= (int)f->leaves.size()) return PQG_ERR_INVALID_ARG;
  memset(out, 0, sizeof(*out));
  if (f->leaves[(size_t)col].path.size() >= sizeof(out->path)) return PQG_ERR_METADATA;  // no truncated paths
  out->desc = f->leaves[(size_t)col].desc;
  strncpy(out->path, f->leaves[(size_t)col].path.c_str(), sizeof(out->path) - 1);
  return PQG_OK;
}

// readChunk chunk_reader.go:314-340: FilePath must be nil, MetaData present,
// type must match the schema; start = DictionaryPageOffset if set.
int pqg_file_chunk(const pqg_file* f, int rg, int col, pqg_chunk_meta* out) {
  if (!f || !out || rg < 0 || rg >= (int)f->rgs.size() || col < 0 || col >= (int)f->leaves.size())
    return PQG_ERR_INVALID_ARG;
  memset(out, 0, sizeof(*out));
  const std::vector<ChunkM>& cols = f->rgs[(size_t)rg];
  if ((int)cols.size() <= col) return PQG_ERR_METADATA;  // "column index %d is out of bounds"
  const ChunkM& m = cols[(size_t)col];
  if (m.has_path || !m.has_meta) return PQG_ERR_METADATA;
  if (m.type != f->leaves[(size_t)col].desc.physical_type) return PQG_ERR_METADATA;
  out->start = m.has_dict ? m.dict_off : m.data_off;
  out->total_compressed_size = m.tcs;
  out->total_uncompressed_size = m.tus;
  out->data_page_offset = m.data_off;
  out->num_values = m.num_values;
  out->has_dict_page_offset = m.has_dict ? 1 : 0;
  out->codec = m.codec;
  out->type = m.type;
  return PQG_OK;
}

}  // extern "C"
