// pqwrite.cpp — synthetic Parquet file writer (TEST / BENCH INPUT GENERATOR).
//
// Writes the BASELINE configs' files (C1..C5) and the parity-test files.  It
// is modelled on the page layout rules of parquet writers (arrow-style
// RLE/bit-pack hybrid with aligned literal groups, 20 000 rows per page, a
// dictionary page followed by data pages, DELTA_BINARY_PACKED with 128-value
// blocks of 4 x 32 miniblocks, snappy per page) and is independent of the
// reference's writer.  Not part of the decode product.
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <vector>
#include <zlib.h>

namespace {

typedef std::vector<uint8_t> Buf;

// ---------------------------------------------------------------- varints
void put_uvarint(Buf& b, uint64_t v) {
  while (v >= 0x80) {
    b.push_back((uint8_t)(v | 0x80));
    v >>= 7;
  }
  b.push_back((uint8_t)v);
}
void put_zigzag(Buf& b, int64_t v) { put_uvarint(b, ((uint64_t)v << 1) ^ (uint64_t)(v >> 63)); }
void put_u32(Buf& b, uint32_t v) {
  for (int i = 0; i < 4; i++) b.push_back((uint8_t)(v >> (8 * i)));
}

// ---------------------------------------------------------------- thrift compact writer
struct TW {
  Buf& b;
  std::vector<int> stack;
  int last = 0;
  explicit TW(Buf& buf) : b(buf) {}
  void field(int id, int ctype) {
    int d = id - last;
    if (d > 0 && d <= 15) {
      b.push_back((uint8_t)(d << 4 | ctype));
    } else {
      b.push_back((uint8_t)ctype);
      put_zigzag(b, id);
    }
    last = id;
  }
  void i32(int id, int32_t v) { field(id, 5); put_zigzag(b, v); }
  void i64(int id, int64_t v) { field(id, 6); put_zigzag(b, v); }
  void boolean(int id, bool v) { field(id, v ? 1 : 2); }
  void str(int id, const std::string& s) {
    field(id, 8);
    put_uvarint(b, s.size());
    b.insert(b.end(), s.begin(), s.end());
  }
  void begin_struct(int id) {
    field(id, 12);
    stack.push_back(last);
    last = 0;
  }
  void begin_struct_elem() {  // struct inside a list
    stack.push_back(last);
    last = 0;
  }
  void end_struct() {
    b.push_back(0);
    last = stack.back();
    stack.pop_back();
  }
  void list(int id, int etype, int64_t n) {
    field(id, 9);
    if (n < 15) {
      b.push_back((uint8_t)(n << 4 | etype));
    } else {
      b.push_back((uint8_t)(0xf0 | etype));
      put_uvarint(b, (uint64_t)n);
    }
  }
  void stop() { b.push_back(0); }
};

// ---------------------------------------------------------------- bit packing
// Append `n` values of width w as an LSB-first bitstream.
void bitpack(Buf& b, const uint64_t* v, int64_t n, int w) {
  if (w == 0) return;
  size_t base = b.size();
  b.resize(base + (size_t)((n * w + 7) / 8), 0);
  uint8_t* p = b.data() + base;
  for (int64_t i = 0; i < n; i++) {
    uint64_t x = w == 64 ? v[i] : (v[i] & ((1ULL << w) - 1));
    int64_t bit = i * (int64_t)w;
    int sh = (int)(bit & 7);
    unsigned __int128 y = (unsigned __int128)x << sh;
    int nb = (sh + w + 7) / 8;
    for (int k = 0; k < nb; k++) p[(bit >> 3) + k] |= (uint8_t)(y >> (8 * k));
  }
}

// RLE / bit-packing hybrid encoder: literal groups of 8 aligned to the start
// of the literal segment; a run of >= min_rle equal values starting at an
// aligned position becomes an RLE run; literal runs <= 64 groups.
// max_groups < 0: parquet-go's own hybridEncoder (hybrid_encoder.go:59-99):
// the whole stream is ONE bit-packed run (bpEncode: header (groups << 1) | 1,
// the values padded to a multiple of 8), nothing for a zero width.
void hybrid_encode(Buf& out, const uint32_t* v, int64_t n, int w, int min_rle = 8, int max_groups = 64) {
  if (max_groups < 0) {
    if (w == 0 || n == 0) return;
    const int64_t groups = (n + 7) / 8;
    put_uvarint(out, (uint64_t)(groups << 1 | 1));
    std::vector<uint64_t> tmp((size_t)(groups * 8), 0);
    for (int64_t k = 0; k < n; k++) tmp[(size_t)k] = v[k];
    bitpack(out, tmp.data(), groups * 8, w);
    return;
  }
  if (max_groups == 0) max_groups = 64;
  if (w == 0) {  // one RLE run without value bytes (readers other than parquet-go read it)
    if (n > 0) put_uvarint(out, (uint64_t)n << 1);
    return;
  }
  int64_t i = 0, lit = 0;
  std::vector<uint64_t> tmp;
  auto flush_lit = [&](int64_t end) {
    int64_t s = lit;
    while (s < end) {
      int64_t cnt = end - s;
      int64_t maxv = (int64_t)max_groups * 8;
      if (cnt > maxv) cnt = maxv;
      int64_t groups = (cnt + 7) / 8;
      put_uvarint(out, (uint64_t)(groups << 1 | 1));
      tmp.assign((size_t)(groups * 8), 0);
      for (int64_t k = 0; k < cnt; k++) tmp[(size_t)k] = v[s + k];
      bitpack(out, tmp.data(), groups * 8, w);
      s += cnt;
    }
  };
  while (i < n) {
    int64_t r = 1;
    while (i + r < n && v[i + r] == v[i]) r++;
    if (r >= min_rle) {
      flush_lit(i);
      put_uvarint(out, (uint64_t)(r << 1));
      int nbytes = (w + 7) / 8;
      for (int k = 0; k < nbytes; k++) out.push_back((uint8_t)(v[i] >> (8 * k)));
      i += r;
      lit = i;
    } else {
      i += 8;
      if (i > n) i = n;
    }
  }
  flush_lit(n);
}

int bits_len(uint64_t v) {
  int n = 0;
  while (v) {
    n++;
    v >>= 1;
  }
  return n;
}
int ceil_log2(uint64_t d) {  // bits to index d entries
  if (d <= 1) return 0;
  return bits_len(d - 1);
}

// DELTA_BINARY_PACKED encoder (block 128, 4 miniblocks of 32).
template <typename T>
void dbp_encode(Buf& out, const T* v, int64_t n, int block = 128, int mbc = 4) {
  typedef typename std::conditional<sizeof(T) == 8, uint64_t, uint32_t>::type U;
  int mbv = block / mbc;
  put_uvarint(out, (uint64_t)block);
  put_uvarint(out, (uint64_t)mbc);
  put_uvarint(out, (uint64_t)n);
  put_zigzag(out, n ? (int64_t)v[0] : 0);
  if (n <= 1) return;
  std::vector<U> deltas((size_t)(n - 1));
  for (int64_t i = 1; i < n; i++) deltas[(size_t)(i - 1)] = (U)((U)v[i] - (U)v[i - 1]);
  std::vector<uint64_t> tmp;
  for (int64_t s = 0; s < n - 1; s += block) {
    int64_t e = s + block < n - 1 ? s + block : n - 1;
    T mind = (T)deltas[(size_t)s];
    for (int64_t k = s; k < e; k++)
      if ((T)deltas[(size_t)k] < mind) mind = (T)deltas[(size_t)k];
    put_zigzag(out, (int64_t)mind);
    uint8_t widths[64];
    std::vector<std::vector<uint64_t>> mbs((size_t)mbc);
    for (int m = 0; m < mbc; m++) {
      int64_t ms = s + (int64_t)m * mbv;
      if (ms >= e) {
        widths[m] = 0;
        continue;
      }
      int64_t me = ms + mbv < e ? ms + mbv : e;
      U mx = 0;
      mbs[(size_t)m].assign((size_t)mbv, 0);
      for (int64_t k = ms; k < me; k++) {
        U x = (U)(deltas[(size_t)k] - (U)mind);
        mbs[(size_t)m][(size_t)(k - ms)] = (uint64_t)x;
        if (x > mx) mx = x;
      }
      widths[m] = (uint8_t)bits_len((uint64_t)mx);
    }
    for (int m = 0; m < mbc; m++) out.push_back(widths[m]);
    for (int m = 0; m < mbc; m++) {
      if ((int64_t)s + (int64_t)m * mbv >= e) break;
      bitpack(out, mbs[(size_t)m].data(), mbv, widths[m]);
    }
  }
}

// DELTA_LENGTH_BYTE_ARRAY: DBP lengths, then the bytes (byteArrayDeltaLengthEncoder,
// type_bytearray.go:142-187); DELTA_BYTE_ARRAY: DBP lengths of the prefix each
// value shares with the previous one, then the suffixes as
// DELTA_LENGTH_BYTE_ARRAY (byteArrayDeltaEncoder, type_bytearray.go:242-300).
void delta_byte_array(Buf& out, const uint8_t* vals, const int64_t* offs, int64_t vs, int64_t ve, bool dba) {
  const int64_t n = ve - vs;
  std::vector<int32_t> lens, pre;
  Buf chars;
  const uint8_t* prev = nullptr;
  int64_t plen = 0;
  for (int64_t i = vs; i < ve; i++) {
    const uint8_t* p = vals + offs[i];
    const int64_t l = offs[i + 1] - offs[i];
    int64_t k = 0;
    if (dba)
      while (k < l && k < plen && prev[k] == p[k]) k++;
    pre.push_back((int32_t)k);
    lens.push_back((int32_t)(l - k));
    chars.insert(chars.end(), p + k, p + l);
    prev = p;
    plen = l;
  }
  if (dba) dbp_encode<int32_t>(out, pre.data(), n);
  dbp_encode<int32_t>(out, lens.data(), n);
  out.insert(out.end(), chars.begin(), chars.end());
}

// ---------------------------------------------------------------- snappy compressor
void snappy_literal(Buf& o, const uint8_t* p, int64_t n) {
  while (n > 0) {
    int64_t len = n > 65536 ? 65536 : n;
    int64_t l1 = len - 1;
    if (l1 < 60) {
      o.push_back((uint8_t)(l1 << 2));
    } else if (l1 < 256) {
      o.push_back(60 << 2);
      o.push_back((uint8_t)l1);
    } else {
      o.push_back(61 << 2);
      o.push_back((uint8_t)l1);
      o.push_back((uint8_t)(l1 >> 8));
    }
    o.insert(o.end(), p, p + len);
    p += len;
    n -= len;
  }
}
void snappy_copy(Buf& o, int64_t off, int64_t len) {
  while (len > 0) {
    int64_t l = len;
    if (l > 64) l = 64;
    if (l >= 4 && l <= 11 && off < 2048) {
      o.push_back((uint8_t)(1 | ((l - 4) << 2) | ((off >> 8) << 5)));
      o.push_back((uint8_t)off);
    } else {
      o.push_back((uint8_t)(2 | ((l - 1) << 2)));
      o.push_back((uint8_t)off);
      o.push_back((uint8_t)(off >> 8));
    }
    len -= l;
  }
}
// Like golang/snappy's Encode (the reference writer's snappyCompressor,
// compress.go:42-44 -> vendor/github.com/golang/snappy/encode.go:18-41): the
// input is cut into independent blocks of maxBlockSize = 65536 bytes
// (snappy.go:72), each encoded with a fresh match table, so no copy reaches
// into an earlier block.  g_snappy_block = 0 encodes the page as one block
// (copies up to 65535 bytes back across any 64 KiB boundary: still a valid
// stream, which the decoder must handle without the block structure).
static int64_t g_snappy_block = 65536;
Buf snappy_compress(const uint8_t* src, int64_t n) {
  Buf o;
  put_uvarint(o, (uint64_t)n);
  const int HB = 14;
  std::vector<int64_t> table((size_t)1 << HB, -1);
  const int64_t bs = g_snappy_block > 0 ? g_snappy_block : (n > 0 ? n : 1);
  for (int64_t b0 = 0; b0 < n || (n == 0 && b0 == 0); b0 += bs) {
    if (n == 0) break;
    const int64_t b1 = b0 + bs < n ? b0 + bs : n;
    std::fill(table.begin(), table.end(), (int64_t)-1);
    int64_t i = b0, lit = b0;
    while (i + 4 <= b1) {
      uint32_t x;
      memcpy(&x, src + i, 4);
      uint32_t h = (x * 0x1e35a7bdU) >> (32 - HB);
      int64_t cand = table[h];
      table[h] = i;
      if (cand >= 0 && i - cand <= 65535 && memcmp(src + cand, src + i, 4) == 0) {
        int64_t len = 4;
        while (i + len < b1 && src[cand + len] == src[i + len]) len++;
        snappy_literal(o, src + lit, i - lit);
        snappy_copy(o, i - cand, len);
        i += len;
        lit = i;
      } else {
        i++;
      }
    }
    snappy_literal(o, src + lit, b1 - lit);
  }
  return o;
}

// ---------------------------------------------------------------- column writer
struct ColSpec {
  std::string name;
  int type, type_length, repetition;  // repetition: 0 required, 1 optional, 2 LIST (3-level, optional list + optional element)
  int encoding, codec, page_version, rows_per_page;
  int64_t dict_limit;  // bytes of dictionary before PLAIN fallback (<=0: no limit)
  const uint8_t* values;
  const int64_t* offsets;
  const uint8_t* def_levels;
  const uint8_t* rep_levels;
  int64_t num_slots, num_values;
  int min_rle;
  int v2_uncompressed_flag;  // write is_compressed=false on V2 pages (Q4 probe)
  int hybrid_groups;         // literal groups per bit-packed run (0: 64; < 0: one run per stream, parquet-go's writer)
};

int type_width(int type, int tl) {
  switch (type) {
    case 0: return 1;
    case 1: case 4: return 4;
    case 2: case 5: return 8;
    case 3: return 12;
    case 7: return tl;
  }
  return 0;
}

struct ChunkOut {
  int64_t start = 0, dict_off = -1, data_off = 0, tcs = 0, tus = 0, num_values = 0;
  std::vector<int> encodings;
};

void write_page_header(Buf& out, int type, int32_t usize, int32_t csize, int32_t nvals, int enc, int32_t nulls,
                       int32_t nrows, int32_t def_len, int32_t rep_len, bool v2_comp) {
  TW t(out);
  t.i32(1, type);
  t.i32(2, usize);
  t.i32(3, csize);
  if (type == 0) {
    t.begin_struct(5);
    t.i32(1, nvals);
    t.i32(2, enc);
    t.i32(3, 3);
    t.i32(4, 3);
    t.end_struct();
  } else if (type == 2) {
    t.begin_struct(7);
    t.i32(1, nvals);
    t.i32(2, 0);  // PLAIN
    t.end_struct();
  } else if (type == 3) {
    t.begin_struct(8);
    t.i32(1, nvals);
    t.i32(2, nulls);
    t.i32(3, nrows);
    t.i32(4, enc);
    t.i32(5, def_len);
    t.i32(6, rep_len);
    t.boolean(7, v2_comp);
    t.end_struct();
  }
  t.stop();
}

// GZIP (codec 2): one gzip member at zlib's default level, as Go's
// gzip.NewWriter (compress.go:63-76 writes through compress/gzip's default).
Buf gzip_compress(const uint8_t* src, int64_t n) {
  z_stream z{};
  if (deflateInit2(&z, Z_DEFAULT_COMPRESSION, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) != Z_OK) return Buf();
  Buf out(deflateBound(&z, (uLong)n) + 64);
  z.next_in = const_cast<uint8_t*>(src);
  z.avail_in = (uInt)n;
  z.next_out = out.data();
  z.avail_out = (uInt)out.size();
  const int r = deflate(&z, Z_FINISH);
  out.resize(r == Z_STREAM_END ? z.total_out : 0);
  deflateEnd(&z);
  return out;
}

Buf compress(int codec, const Buf& raw) {
  if (codec == 1) return snappy_compress(raw.data(), (int64_t)raw.size());
  if (codec == 2) return gzip_compress(raw.data(), (int64_t)raw.size());
  return raw;
}

// Encode PLAIN values [vs, ve) of the column into b.
void plain_values(Buf& b, const ColSpec& c, int64_t vs, int64_t ve) {
  int w = type_width(c.type, c.type_length);
  if (c.type == 0) {  // boolean bit-packed
    int64_t n = ve - vs;
    for (int64_t i = 0; i < n; i += 8) {
      uint8_t x = 0;
      for (int j = 0; j < 8 && i + j < n; j++) x |= (uint8_t)((c.values[vs + i + j] & 1) << j);
      b.push_back(x);
    }
  } else if (w > 0) {
    b.insert(b.end(), c.values + vs * w, c.values + ve * w);
  } else {
    for (int64_t i = vs; i < ve; i++) {
      int64_t a = c.offsets[i], e = c.offsets[i + 1];
      put_u32(b, (uint32_t)(e - a));
      b.insert(b.end(), c.values + a, c.values + e);
    }
  }
}

struct Key {
  const uint8_t* p;
  int64_t n;
  bool operator==(const Key& o) const { return n == o.n && memcmp(p, o.p, (size_t)n) == 0; }
};
struct KeyHash {
  size_t operator()(const Key& k) const {
    uint64_t h = 1469598103934665603ULL;
    for (int64_t i = 0; i < k.n; i++) h = (h ^ k.p[i]) * 1099511628211ULL;
    return (size_t)h;
  }
};

// Write one column chunk covering slots [s0, s1) / values [v0, v1) / rows.
ChunkOut write_chunk(Buf& file, const ColSpec& c, int64_t s0, int64_t s1, int64_t v0, int64_t v1,
                     const std::vector<int64_t>& row_starts /* slot index of each row start within [s0,s1) */) {
  ChunkOut co;
  co.start = (int64_t)file.size();
  int maxd = c.repetition == 0 ? 0 : (c.repetition == 1 ? 1 : 3);
  int maxr = c.repetition == 2 ? 1 : 0;
  int dw = bits_len((uint64_t)maxd), rw = bits_len((uint64_t)maxr);
  int w = type_width(c.type, c.type_length);

  // page boundaries in rows
  std::vector<int64_t> pstarts;  // slot starts
  int64_t nrows = (int64_t)row_starts.size();
  for (int64_t r = 0; r < nrows; r += c.rows_per_page) pstarts.push_back(row_starts[(size_t)r]);
  if (pstarts.empty()) pstarts.push_back(s0);
  pstarts.push_back(s1);

  // dictionary: built over the chunk's values, up to dict_limit bytes; pages
  // whose values all fall before the fallback point are dictionary pages.
  bool use_dict = c.encoding == 8;
  std::vector<uint32_t> idx;
  int64_t dict_values_end = v1;  // values [v0, dict_values_end) are dictionary-encoded candidates
  Buf dict_plain;
  int64_t dict_count = 0;
  if (use_dict) {
    std::unordered_map<Key, uint32_t, KeyHash> m;
    idx.resize((size_t)(v1 - v0));
    int64_t bytes = 0;
    for (int64_t i = v0; i < v1; i++) {
      Key k = w > 0 ? Key{c.values + i * w, w} : Key{c.values + c.offsets[i], c.offsets[i + 1] - c.offsets[i]};
      auto it = m.find(k);
      if (it == m.end()) {
        int64_t add = w > 0 ? w : 4 + k.n;
        if (c.dict_limit > 0 && bytes + add > c.dict_limit) {
          dict_values_end = i;
          break;
        }
        uint32_t id = (uint32_t)m.size();
        m.emplace(k, id);
        bytes += add;
        if (w > 0) {
          dict_plain.insert(dict_plain.end(), k.p, k.p + k.n);
        } else {
          put_u32(dict_plain, (uint32_t)k.n);
          dict_plain.insert(dict_plain.end(), k.p, k.p + k.n);
        }
        idx[(size_t)(i - v0)] = id;
      } else {
        idx[(size_t)(i - v0)] = it->second;
      }
    }
    dict_count = (int64_t)m.size();
    if (c.type == 0) use_dict = false;  // boolean: no dictionary
  }
  int idx_w = ceil_log2((uint64_t)dict_count);

  if (use_dict) {
    Buf comp = compress(c.codec, dict_plain);
    co.dict_off = (int64_t)file.size();
    Buf hdr;
    write_page_header(hdr, 2, (int32_t)dict_plain.size(), (int32_t)comp.size(), (int32_t)dict_count, 0, 0, 0, 0, 0,
                      true);
    file.insert(file.end(), hdr.begin(), hdr.end());
    file.insert(file.end(), comp.begin(), comp.end());
    co.tus += (int64_t)(hdr.size() + dict_plain.size());
    co.encodings.push_back(0);
  }
  co.data_off = (int64_t)file.size();

  // walk pages
  int64_t vcur = v0;
  std::vector<uint32_t> lv;
  bool any_plain = false, any_dict = false;
  for (size_t p = 0; p + 1 < pstarts.size(); p++) {
    int64_t ps = pstarts[p], pe = pstarts[p + 1];
    int64_t n = pe - ps;
    int64_t nn = 0;
    for (int64_t i = ps; i < pe; i++)
      if (!c.def_levels || c.def_levels[i] == maxd) nn++;
    int64_t vs = vcur, ve = vcur + nn;
    vcur = ve;
    Buf rep, def, vals;
    if (maxr > 0) {
      lv.assign((size_t)n, 0);
      for (int64_t i = 0; i < n; i++) lv[(size_t)i] = c.rep_levels[ps + i];
      hybrid_encode(rep, lv.data(), n, rw, c.min_rle, c.hybrid_groups);
    }
    if (maxd > 0) {
      lv.assign((size_t)n, 0);
      for (int64_t i = 0; i < n; i++) lv[(size_t)i] = c.def_levels[ps + i];
      hybrid_encode(def, lv.data(), n, dw, c.min_rle, c.hybrid_groups);
    }
    int enc = c.encoding;
    if (enc == 8 && (!use_dict || ve > dict_values_end)) enc = 0;  // PLAIN fallback
    if (enc == 8) {
      vals.push_back((uint8_t)idx_w);
      hybrid_encode(vals, idx.data() + (vs - v0), nn, idx_w, c.min_rle, c.hybrid_groups);
      any_dict = true;
    } else if (enc == 6 || enc == 7) {
      if (c.offsets) {
        delta_byte_array(vals, c.values, c.offsets, vs, ve, enc == 7);
      } else {  // FIXED_LEN_BYTE_ARRAY: values of type_length bytes
        std::vector<int64_t> fo((size_t)(ve + 1));
        for (int64_t i = 0; i <= ve; i++) fo[(size_t)i] = i * c.type_length;
        delta_byte_array(vals, c.values, fo.data(), vs, ve, enc == 7);
      }
    } else if (enc == 5) {
      if (c.type == 1)
        dbp_encode<int32_t>(vals, (const int32_t*)c.values + vs, nn);
      else
        dbp_encode<int64_t>(vals, (const int64_t*)c.values + vs, nn);
    } else {
      plain_values(vals, c, vs, ve);
      any_plain = true;
    }
    int64_t nrows_page = 0;
    for (int64_t i = ps; i < pe; i++)
      if (!c.rep_levels || c.rep_levels[i] == 0) nrows_page++;
    Buf hdr, body;
    int32_t usize, csize;
    if (c.page_version == 2) {
      Buf comp = compress(c.codec, vals);
      bool is_comp = !c.v2_uncompressed_flag;
      body.insert(body.end(), rep.begin(), rep.end());
      body.insert(body.end(), def.begin(), def.end());
      body.insert(body.end(), comp.begin(), comp.end());
      usize = (int32_t)(rep.size() + def.size() + vals.size());
      csize = (int32_t)body.size();
      write_page_header(hdr, 3, usize, csize, (int32_t)n, enc, (int32_t)(n - nn), (int32_t)nrows_page,
                        (int32_t)def.size(), (int32_t)rep.size(), is_comp);
    } else {
      Buf raw;
      if (maxr > 0) {
        put_u32(raw, (uint32_t)rep.size());
        raw.insert(raw.end(), rep.begin(), rep.end());
      }
      if (maxd > 0) {
        put_u32(raw, (uint32_t)def.size());
        raw.insert(raw.end(), def.begin(), def.end());
      }
      raw.insert(raw.end(), vals.begin(), vals.end());
      body = compress(c.codec, raw);
      usize = (int32_t)raw.size();
      csize = (int32_t)body.size();
      write_page_header(hdr, 0, usize, csize, (int32_t)n, enc, 0, 0, 0, 0, true);
    }
    file.insert(file.end(), hdr.begin(), hdr.end());
    file.insert(file.end(), body.begin(), body.end());
    co.tus += (int64_t)hdr.size() + usize;
  }
  if (any_dict) co.encodings.push_back(8);
  if (any_plain || c.encoding == 0) co.encodings.push_back(0);
  if (c.encoding == 5 || c.encoding == 6 || c.encoding == 7) co.encodings.push_back(c.encoding);
  co.encodings.push_back(3);
  co.tcs = (int64_t)file.size() - co.start;
  co.num_values = s1 - s0;
  return co;
}

}  // namespace

extern "C" {

typedef struct pqw_column {
  const char* name;
  int32_t type, type_length, repetition, encoding, codec, page_version, rows_per_page, min_rle;
  int32_t v2_uncompressed_flag, hybrid_groups;
  int64_t dict_limit;
  const uint8_t* values;
  const int64_t* offsets;
  const uint8_t* def_levels;
  const uint8_t* rep_levels;
  int64_t num_slots, num_values;
} pqw_column;

}  // extern "C"

namespace {
// An open file: the bytes so far, the column specs (metadata only: their
// array pointers are not kept past the call that wrote them) and every row
// group's chunk records, for the footer.
struct Writer {
  // the bytes so far, in one malloc'ed block grown by realloc (large blocks
  // are remapped, not copied), handed to the caller as the file at the end
  uint8_t* mem = nullptr;
  size_t len = 0, cap = 0;
  std::vector<ColSpec> cs;
  std::vector<std::vector<ChunkOut>> rgs;
  std::vector<int64_t> rg_rows;
  int64_t num_rows = 0;
  Buf tail;  // footer + length + magic (build_tail)
  ~Writer() { free(mem); }
  bool append(const uint8_t* p, size_t n) {
    if (len + n > cap) {
      size_t nc = cap ? cap : 1 << 20;
      while (nc < len + n) nc += nc / 2 + (1 << 20);
      uint8_t* m = (uint8_t*)realloc(mem, nc);
      if (!m) return false;
      mem = m;
      cap = nc;
    }
    memcpy(mem + len, p, n);
    len += n;
    return true;
  }
};

// Append `row_groups` row groups of equal row counts holding the `ncols`
// columns' `num_rows` rows.  A later call must pass the same columns (name,
// type, repetition, codec).
int add_row_groups(Writer& w, const pqw_column* cols, int ncols, int64_t num_rows, int row_groups) {
  if (row_groups < 1) row_groups = 1;
  if (!w.cs.empty() && (int)w.cs.size() != ncols) return -3;
  std::vector<ColSpec> cs((size_t)ncols);
  std::vector<std::vector<int64_t>> row_start_slots((size_t)ncols);
  std::vector<std::vector<int64_t>> value_before_slot((size_t)ncols);
  for (int k = 0; k < ncols; k++) {
    const pqw_column& p = cols[k];
    ColSpec& c = cs[(size_t)k];
    c.name = p.name;
    c.type = p.type;
    c.type_length = p.type_length;
    c.repetition = p.repetition;
    c.encoding = p.encoding;
    c.codec = p.codec;
    c.page_version = p.page_version;
    c.rows_per_page = p.rows_per_page > 0 ? p.rows_per_page : 20000;
    c.dict_limit = p.dict_limit;
    c.values = p.values;
    c.offsets = p.offsets;
    c.def_levels = p.def_levels;
    c.rep_levels = p.rep_levels;
    c.num_slots = p.num_slots;
    c.num_values = p.num_values;
    c.min_rle = p.min_rle > 0 ? p.min_rle : 8;
    c.v2_uncompressed_flag = p.v2_uncompressed_flag;
    c.hybrid_groups = p.hybrid_groups;
    if (!w.cs.empty()) {
      const ColSpec& o = w.cs[(size_t)k];
      if (o.name != c.name || o.type != c.type || o.repetition != c.repetition || o.codec != c.codec) return -3;
    }
    int maxd = c.repetition == 0 ? 0 : (c.repetition == 1 ? 1 : 3);
    auto& rs = row_start_slots[(size_t)k];
    for (int64_t i = 0; i < c.num_slots; i++)
      if (!c.rep_levels || c.rep_levels[i] == 0) rs.push_back(i);
    if ((int64_t)rs.size() != num_rows) return -1;
    auto& vb = value_before_slot[(size_t)k];
    vb.resize((size_t)c.num_slots + 1);
    int64_t acc = 0;
    for (int64_t i = 0; i < c.num_slots; i++) {
      vb[(size_t)i] = acc;
      if (!c.def_levels || c.def_levels[i] == maxd) acc++;
    }
    vb[(size_t)c.num_slots] = acc;
    if (acc != c.num_values) return -2;
  }
  int64_t per = (num_rows + row_groups - 1) / row_groups;
  Buf rg;  // one row group's chunks (offsets rebased onto the file below)
  for (int g = 0; g < row_groups; g++) {
    int64_t r0 = g * per, r1 = (g + 1) * per < num_rows ? (g + 1) * per : num_rows;
    if (r0 > r1) r0 = r1;
    w.rg_rows.push_back(r1 - r0);
    w.rgs.emplace_back();
    rg.clear();
    for (int k = 0; k < ncols; k++) {
      auto& rs = row_start_slots[(size_t)k];
      int64_t s0 = r0 < (int64_t)rs.size() ? rs[(size_t)r0] : cs[(size_t)k].num_slots;
      int64_t s1 = r1 < (int64_t)rs.size() ? rs[(size_t)r1] : cs[(size_t)k].num_slots;
      std::vector<int64_t> starts(rs.begin() + r0, rs.begin() + r1);
      auto& vb = value_before_slot[(size_t)k];
      ChunkOut co = write_chunk(rg, cs[(size_t)k], s0, s1, vb[(size_t)s0], vb[(size_t)s1], starts);
      co.start += (int64_t)w.len;
      co.data_off += (int64_t)w.len;
      if (co.dict_off >= 0) co.dict_off += (int64_t)w.len;
      w.rgs.back().push_back(co);
    }
    if (!w.append(rg.data(), rg.size())) return -4;
  }
  w.num_rows += num_rows;
  if (w.cs.empty()) {
    for (ColSpec& c : cs) c.values = nullptr, c.offsets = nullptr, c.def_levels = c.rep_levels = nullptr;
    w.cs = cs;
  }
  return 0;
}

// The footer (FileMetaData), its length and the closing magic into w.tail.
void build_tail(Writer& w) {
  const std::vector<ColSpec>& cs = w.cs;
  const int ncols = (int)cs.size();
  const int row_groups = (int)w.rgs.size();
  Buf meta;
  TW t(meta);
  t.i32(1, 1);
  // schema: root + leaves (LIST columns expand to 3 elements + the leaf)
  int64_t n_elems = 1;
  for (const auto& c : cs) n_elems += c.repetition == 2 ? 3 : 1;
  t.list(2, 12, n_elems);
  t.begin_struct_elem();
  t.str(4, "schema");
  t.i32(5, ncols);
  t.end_struct();
  for (const auto& c : cs) {
    if (c.repetition == 2) {
      t.begin_struct_elem();
      t.i32(3, 1);  // OPTIONAL
      t.str(4, c.name);
      t.i32(5, 1);
      t.i32(6, 3);  // ConvertedType LIST
      t.end_struct();
      t.begin_struct_elem();
      t.i32(3, 2);  // REPEATED
      t.str(4, "list");
      t.i32(5, 1);
      t.end_struct();
      t.begin_struct_elem();
      t.i32(1, c.type);
      if (c.type == 7) t.i32(2, c.type_length);
      t.i32(3, 1);
      t.str(4, "element");
      t.end_struct();
    } else {
      t.begin_struct_elem();
      t.i32(1, c.type);
      if (c.type == 7) t.i32(2, c.type_length);
      t.i32(3, c.repetition == 0 ? 0 : 1);
      t.str(4, c.name);
      if (c.type == 6) t.i32(6, 0);  // UTF8
      t.end_struct();
    }
  }
  t.i64(3, w.num_rows);
  t.list(4, 12, row_groups);
  for (int g = 0; g < row_groups; g++) {
    t.begin_struct_elem();
    t.list(1, 12, ncols);
    int64_t total = 0;
    for (int k = 0; k < ncols; k++) {
      const ChunkOut& co = w.rgs[(size_t)g][(size_t)k];
      const ColSpec& c = cs[(size_t)k];
      total += co.tus;
      t.begin_struct_elem();
      t.i64(2, co.start);
      t.begin_struct(3);
      t.i32(1, c.type);
      t.list(2, 5, (int64_t)co.encodings.size());
      for (int e : co.encodings) put_zigzag(meta, e);
      if (c.repetition == 2) {
        t.list(3, 8, 3);
        for (const std::string& s : {c.name, std::string("list"), std::string("element")}) {
          put_uvarint(meta, s.size());
          meta.insert(meta.end(), s.begin(), s.end());
        }
      } else {
        t.list(3, 8, 1);
        put_uvarint(meta, c.name.size());
        meta.insert(meta.end(), c.name.begin(), c.name.end());
      }
      t.i32(4, c.codec);
      t.i64(5, co.num_values);
      t.i64(6, co.tus);
      t.i64(7, co.tcs);
      t.i64(9, co.data_off);
      if (co.dict_off >= 0) t.i64(11, co.dict_off);
      t.end_struct();
      t.end_struct();
    }
    t.i64(2, total);
    t.i64(3, w.rg_rows[(size_t)g]);
    t.end_struct();
  }
  t.str(6, "pqgpu-gen");
  t.stop();
  w.tail = meta;
  put_u32(w.tail, (uint32_t)meta.size());
  w.tail.insert(w.tail.end(), {'P', 'A', 'R', '1'});
}
}  // namespace

extern "C" {

// Write a whole file: `ncols` columns of `num_rows` rows split into
// `row_groups` row groups of equal row counts.  Returns 0 and a malloc'ed
// buffer in *out.
int pqw_write_file(const pqw_column* cols, int ncols, int64_t num_rows, int row_groups, uint8_t** out,
                   int64_t* out_len) {
  Writer w;
  const uint8_t magic[4] = {'P', 'A', 'R', '1'};
  if (!w.append(magic, 4)) return -4;
  const int rc = add_row_groups(w, cols, ncols, num_rows, row_groups);
  if (rc) return rc;
  build_tail(w);
  if (!w.append(w.tail.data(), w.tail.size())) return -4;
  *out = w.mem;
  *out_len = (int64_t)w.len;
  w.mem = nullptr;
  return 0;
}

// A file written one row group at a time, so a caller never holds more than
// one row group's column arrays (the C5 shard: 8 row groups per rank):
// pqw_writer_new, pqw_writer_add (one call per row group, the same columns
// each time), pqw_writer_finish (the footer; the file's malloc'ed bytes are
// handed over, free them with pqw_free; the writer is freed).
void* pqw_writer_new() {
  Writer* w = new Writer();
  const uint8_t magic[4] = {'P', 'A', 'R', '1'};
  if (!w->append(magic, 4)) {
    delete w;
    return nullptr;
  }
  return w;
}
int pqw_writer_add(void* h, const pqw_column* cols, int ncols, int64_t num_rows) {
  return add_row_groups(*(Writer*)h, cols, ncols, num_rows, 1);
}
int pqw_writer_finish(void* h, uint8_t** out, int64_t* out_len) {
  Writer* w = (Writer*)h;
  build_tail(*w);
  if (!w->append(w->tail.data(), w->tail.size())) {
    delete w;
    return -4;
  }
  *out = (uint8_t*)realloc(w->mem, w->len);  // shrink to the file
  if (!*out) *out = w->mem;
  *out_len = (int64_t)w->len;
  w->mem = nullptr;
  delete w;
  return 0;
}
void pqw_writer_free(void* h) { delete (Writer*)h; }

void pqw_free(uint8_t* p) { free(p); }

// Raw encoders exposed for unit tests.
int64_t pqw_hybrid_encode(const uint32_t* v, int64_t n, int w, int min_rle, uint8_t* out, int64_t cap) {
  Buf b;
  hybrid_encode(b, v, n, w, min_rle);
  if ((int64_t)b.size() > cap) return -(int64_t)b.size();
  memcpy(out, b.data(), b.size());
  return (int64_t)b.size();
}
int64_t pqw_dbp_encode64(const int64_t* v, int64_t n, uint8_t* out, int64_t cap) {
  Buf b;
  dbp_encode<int64_t>(b, v, n);
  if ((int64_t)b.size() > cap) return -(int64_t)b.size();
  memcpy(out, b.data(), b.size());
  return (int64_t)b.size();
}
int64_t pqw_dbp_encode32(const int32_t* v, int64_t n, uint8_t* out, int64_t cap) {
  Buf b;
  dbp_encode<int32_t>(b, v, n);
  if ((int64_t)b.size() > cap) return -(int64_t)b.size();
  memcpy(out, b.data(), b.size());
  return (int64_t)b.size();
}
// 65536 (default): golang/snappy's independent 64 KiB blocks; 0: one block
void pqw_set_snappy_block(int64_t bs) { g_snappy_block = bs; }
int64_t pqw_snappy_compress(const uint8_t* src, int64_t n, uint8_t* out, int64_t cap) {
  Buf b = snappy_compress(src, n);
  if ((int64_t)b.size() > cap) return -(int64_t)b.size();
  memcpy(out, b.data(), b.size());
  return (int64_t)b.size();
}

}  // extern "C"
