/*
 * pqgpu.h — C ABI of the MI355X (gfx950) Parquet column-chunk decoder.
 *
 * This is the drop-in boundary for parquet-go's page-decode path
 * (fraugster/parquet-go v0.2.1, mounted read-only at /root/reference).  Every
 * entry point below names the reference interface it replaces.  Signatures use
 * plain pointers and sizes only (no torch / HIP types), so a cgo, ctypes or
 * JNI binding can call them directly.
 *
 * Two libraries implement (parts of) this header:
 *   libpqgpu.so   (parquet-go_amd/csrc)  the product: HIP kernels + host runtime
 *   liboracle.so  (oracle/)              TEST INFRASTRUCTURE ONLY: the CPU
 *                                        restatement of the reference algorithm
 *                                        (pqo_* symbols), used as the parity checker.
 *
 * Semantics: a "chunk job" is one column chunk (ColumnChunk / ColumnMetaData of
 * one row group).  Decoding a job is what the reference does in
 *   readChunk      chunk_reader.go:314-378   (seek, level-decoder factories)
 *   readPages      chunk_reader.go:206-284   (page-header walk, dict page, V1/V2)
 *   readPageData   chunk_reader.go:380-402   (per page readValues)
 * and the per-page outputs are exactly pageReader.readValues
 * (interfaces.go:10-17; page_v1.go:27-55, page_v2.go:26-54):
 *   rLevels[numValues], dLevels[numValues], values[:notNull]
 * concatenated over the data pages of the chunk in file order (spec-correct
 * stitching; see DESIGN.md "Quirk policy" for the reference's Q1/Q2 defects).
 */
#ifndef PQGPU_H
#define PQGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- parquet.thrift enums (reference parquet/parquet.go: Type, Encoding :343,
 *      CompressionCodec :442, PageType :525) ------------------------------- */
enum {
  PQG_BOOLEAN = 0,
  PQG_INT32 = 1,
  PQG_INT64 = 2,
  PQG_INT96 = 3,
  PQG_FLOAT = 4,
  PQG_DOUBLE = 5,
  PQG_BYTE_ARRAY = 6,
  PQG_FIXED_LEN_BYTE_ARRAY = 7
};
enum {
  PQG_ENC_PLAIN = 0,
  PQG_ENC_PLAIN_DICTIONARY = 2,
  PQG_ENC_RLE = 3,
  PQG_ENC_BIT_PACKED = 4,
  PQG_ENC_DELTA_BINARY_PACKED = 5,
  PQG_ENC_DELTA_LENGTH_BYTE_ARRAY = 6,
  PQG_ENC_DELTA_BYTE_ARRAY = 7,
  PQG_ENC_RLE_DICTIONARY = 8
};
enum {
  PQG_CODEC_UNCOMPRESSED = 0,
  PQG_CODEC_SNAPPY = 1,
  PQG_CODEC_GZIP = 2
};
enum {
  PQG_PAGE_DATA = 0,
  PQG_PAGE_INDEX = 1,
  PQG_PAGE_DICTIONARY = 2,
  PQG_PAGE_DATA_V2 = 3
};

/* ---- status codes --------------------------------------------------------
 * The reference returns a Go error (wrapped with github.com/pkg/errors) and
 * treats ANY error inside readPages/readPageData as fatal for the row group.
 * Parity is defined on error/no-error per page and per chunk; the class below
 * is this library's own classification, identical between libpqgpu and the
 * oracle (both follow the same cited reference lines). */
enum {
  PQG_OK = 0,
  PQG_ERR_EOF = -1,           /* io.EOF / io.ErrUnexpectedEOF inside a stream       */
  PQG_ERR_THRIFT = -2,        /* PageHeader thrift-compact decode failed            */
  PQG_ERR_PAGE_HEADER = -3,   /* missing sub-header, negative count/size            */
  PQG_ERR_SIZE = -4,          /* block shorter than compressed size / size mismatch */
  PQG_ERR_SNAPPY = -5,        /* snappy: corrupt input                              */
  PQG_ERR_RLE = -6,           /* hybrid: empty run, RLE value too large, bad varint */
  PQG_ERR_DICT_INDEX = -7,    /* dict: invalid index                                */
  PQG_ERR_BIT_WIDTH = -8,     /* dict/delta: invalid bit width                      */
  PQG_ERR_DELTA = -9,         /* DELTA_BINARY_PACKED header/stream invalid          */
  PQG_ERR_UNSUPPORTED = -10,  /* encoding / codec / type / page type                */
  PQG_ERR_DICT_PAGE = -11,    /* second dictionary page                             */
  PQG_ERR_BYTE_ARRAY = -12,   /* bytearray/plain: negative length                   */
  PQG_ERR_LEVELS = -13,       /* level decoder not initialised (V2, zero length)    */
  PQG_ERR_GZIP = -15,         /* gzip: invalid header / data / checksum (compress.go:63-76) */
  PQG_ERR_FIXED_LEN = -14,    /* DELTA_BYTE_ARRAY on FIXED_LEN_BYTE_ARRAY: a value  */
                              /* whose length is not type_length (the reference     */
                              /* returns it; the fixed-width output cannot hold it) */
  PQG_ERR_CAPACITY = -20,     /* internal: arena too small; host grows and retries  */
  PQG_ERR_INVALID_ARG = -21,
  PQG_ERR_HIP = -22,
  PQG_ERR_METADATA = -23,     /* footer / FileMetaData problems                      */
  PQG_ERR_NOT_BUILT = -24
};

/* page_info.flags */
enum {
  PQG_PAGE_FLAG_INT96_NIL = 1,  /* Q8: truncated final INT96 value left nil by the
                                   reference (type_int96.go:21-42); bytes are 0 */
  PQG_PAGE_FLAG_SNAPPY_SERIAL = 2, /* libpqgpu diagnostic: the page's snappy block was
                                   decoded whole by one wave (its 64 KiB sub-block
                                   split failed: a copy across a 64 KiB block
                                   boundary, or a corrupt block) */
  PQG_PAGE_FLAG_INFLATE_REDO = 64 /* libpqgpu diagnostic: the page's GZIP stream was
                                   decoded again with the full 32 KiB window ring
                                   (a match reached back past the 8 KiB ring to
                                   bytes past the page's size) */
};

/* ---- column / chunk description ----------------------------------------- */

/* What readChunk learns from the schema (schema.go:789-894) and the chunk's
 * ColumnMetaData (parquet.go ColumnMetaData). */
typedef struct pqg_column_desc {
  int32_t physical_type; /* PQG_INT32 ...                                        */
  int32_t type_length;   /* FIXED_LEN_BYTE_ARRAY length; -1 = unset (nil)        */
  int32_t max_def;       /* Column.MaxDefinitionLevel()  (0..255)                */
  int32_t max_rep;       /* Column.MaxRepetitionLevel()  (0..255)                */
  int32_t codec;         /* ColumnMetaData.codec                                 */
  int32_t flags;         /* bit0: unsigned (uint32/uint64 Go type; bits identical) */
} pqg_column_desc;

/* One column chunk to decode.  `data` points at the chunk's first page
 * (DictionaryPageOffset when set, else DataPageOffset — chunk_reader.go:332-340).
 * For pqg_decode_chunks it is a DEVICE pointer (bytes resident in HBM); for the
 * oracle it is a host pointer. */
typedef struct pqg_chunk_job {
  pqg_column_desc col;
  const uint8_t* data;
  int64_t data_len;              /* readable bytes at data (>= total_compressed_size) */
  int64_t total_compressed_size; /* ColumnMetaData.total_compressed_size              */
  int64_t data_page_offset;      /* DataPageOffset - first-page offset (>= 0)          */
  int64_t num_values_hint;       /* ColumnMetaData.num_values (capacity hint only)     */
  int64_t total_uncompressed_size; /* ColumnMetaData.total_uncompressed_size (hint)     */
  int32_t has_dict_page_offset;  /* ColumnMetaData.DictionaryPageOffset != nil         */
  int32_t quirks;                /* PQG_QUIRK_* mask; libpqgpu decodes spec-correctly
                                    and rejects a non-zero mask (PQG_ERR_INVALID_ARG):
                                    quirk reproduction is the oracle's triage mode
                                    (pqo_decode_column_store)                        */
} pqg_chunk_job;

/* The reference's caller-side stitching defects (DESIGN.md "Quirk
 * policy").  Q1: readPageData appends each page's whole numValues-long slice,
 * numValues - notNull trailing nils included (chunk_reader.go:394-397).  Q2:
 * from the second row group on, the dictionary page decodes into the column
 * store's reused backing array (chunk_reader.go:235, page_dict.go:50-53), which
 * the first data page's append then overwrites (type_dict.go:72-79). */
enum {
  PQG_QUIRK_Q1_PAGE_NILS = 1,
  PQG_QUIRK_Q2_DICT_ALIAS = 2
};

/* Decoded column chunk.  Fixed-width physical types (INT32/INT64/INT96/FLOAT/
 * DOUBLE/FLBA>0/BOOLEAN) store values densely, little endian, `value_width`
 * bytes each (BOOLEAN: one byte 0/1).  BYTE_ARRAY (and FLBA with length 0)
 * store the value bytes back to back in `values` (values_bytes = chars) and
 * num_values+1 int64 `offsets` (offsets[0] = 0, value i = chars
 * [offsets[i], offsets[i+1]); Arrow large-binary layout).  Pointers are DEVICE
 * pointers for libpqgpu (owned by the ctx, valid until the next decode on that
 * ctx or pqg_ctx_destroy) and malloc'ed host pointers for the oracle. */
typedef struct pqg_chunk_result {
  int32_t status;      /* first error in reference order (read phase, then decode) */
  int32_t error_page;  /* index into the page list of the failing page, -1 if none */
  int32_t num_pages;   /* pages seen (dictionary page included)                    */
  int32_t value_width; /* bytes per value; 0 = variable length (offsets)           */
  int32_t col_flags;   /* the job's pqg_column_desc.flags, echoed: bit0 unsigned   */
                       /* (the Go adapter boxes uint32/uint64 from it, as          */
                       /* int32PlainDecoder.unSigned does, type_int32.go:29-33)    */
  int32_t reserved;
  int64_t num_slots;   /* Σ data-page num_values  (= level entries)                */
  int64_t num_values;  /* Σ notNull                                                */
  int64_t values_bytes;
  uint8_t* def_levels; /* num_slots bytes, NULL when max_def == 0                  */
  uint8_t* rep_levels; /* num_slots bytes, NULL when max_rep == 0                  */
  uint8_t* values;
  int64_t* offsets;    /* variable-length values only                              */
} pqg_chunk_result;

/* Per page bookkeeping (dictionary page included, in file order). */
typedef struct pqg_page_info {
  int64_t header_offset;     /* relative to job.data                    */
  int64_t payload_offset;    /* first byte after the thrift header      */
  int64_t slot_offset;       /* Σ num_values of preceding data pages    */
  int64_t value_offset;      /* Σ not_null  of preceding data pages     */
  int32_t page_type;
  int32_t encoding;
  int32_t num_values;        /* header NumValues                        */
  int32_t not_null;          /* #(dLevel == maxD)                        */
  int32_t compressed_size;
  int32_t uncompressed_size;
  int32_t def_len;           /* V2 DefinitionLevelsByteLength           */
  int32_t rep_len;           /* V2 RepetitionLevelsByteLength           */
  int32_t def_encoding;      /* V1 definition_level_encoding            */
  int32_t rep_encoding;
  int32_t status;
  int32_t flags;             /* PQG_PAGE_FLAG_*                          */
} pqg_page_info;

/* ======================= libpqgpu (product) =============================== */

typedef struct pqg_ctx pqg_ctx;

/* One context per GPU; owns a HIP stream and grow-only device arenas.
 * (No reference counterpart: parquet-go's reader is one goroutine per FileReader.) */
int pqg_ctx_create(int device, pqg_ctx** out);
void pqg_ctx_destroy(pqg_ctx* ctx);
const char* pqg_status_string(int status);

/* Device memory helpers for callers without their own allocator (cgo). */
int pqg_device_alloc(pqg_ctx* ctx, int64_t bytes, void** dptr);
int pqg_device_free(pqg_ctx* ctx, void* dptr);
int pqg_memcpy_h2d(pqg_ctx* ctx, void* dst, const void* src, int64_t bytes);
int pqg_memcpy_d2h(pqg_ctx* ctx, void* dst, const void* src, int64_t bytes);

/* Decode a batch of column chunks already resident in HBM.  Replaces, for
 * every job, readChunk+readPages+readPageData (chunk_reader.go:206-402) and the
 * valuesDecoder / levelDecoder implementations they call (interfaces.go:28-38,
 * hybrid_decoder.go:17-28).  Enqueues work on the ctx stream and returns;
 * pqg_sync waits and fills `results` (n_jobs entries). */
int pqg_decode_chunks_async(pqg_ctx* ctx, const pqg_chunk_job* jobs, int n_jobs);
int pqg_sync(pqg_ctx* ctx, pqg_chunk_result* results, int n_jobs);
/* Convenience: async + sync. */
int pqg_decode_chunks(pqg_ctx* ctx, const pqg_chunk_job* jobs, int n_jobs,
                      pqg_chunk_result* results);

/* ---- page-level and codec-level entries ------------------------------------ */

/* One data page (and optionally its chunk's dictionary page), both DEVICE
 * pointers to a thrift PageHeader followed by the page body.  Decoding it is
 * pageReader.read + readValues (interfaces.go:10-17; page_v1.go:27-108,
 * page_v2.go:26-129, dictionary: page_dict.go:30-64): the result holds that
 * page's rLevels, dLevels and values[:notNull] (or chars + offsets), the page
 * table lists the dictionary page (if any) and the data page. */
typedef struct pqg_page_job {
  pqg_column_desc col;
  const uint8_t* page;       /* DEVICE: PageHeader + body of a DATA_PAGE / DATA_PAGE_V2 */
  int64_t page_len;
  const uint8_t* dict_page;  /* DEVICE: PageHeader + body of the DICTIONARY_PAGE, or NULL */
  int64_t dict_page_len;
} pqg_page_job;
int pqg_decode_page(pqg_ctx* ctx, const pqg_page_job* job, pqg_chunk_result* result);

/* BlockCompressor.DecompressBlock (compress.go:24-27, 46-48, registered with
 * RegisterBlockCompressor compress.go:124-135): decompress one HOST block
 * synchronously on the GPU.  codec SNAPPY (snappy.Decode semantics: decoded
 * length from the block's varint header, ErrCorrupt -> PQG_ERR_SNAPPY), GZIP
 * (gzipCompressor.DecompressBlock, compress.go:63-76: multistream members,
 * a bad header / block / CRC / ISIZE or trailing bytes -> PQG_ERR_GZIP) or
 * UNCOMPRESSED (a copy).  *out_len is the decoded length; PQG_ERR_CAPACITY
 * when it exceeds `cap` (nothing written). */
int pqg_block_decompress(pqg_ctx* ctx, int codec, const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap,
                         int64_t* out_len);

/* ColumnStore refill (the Go adapter's half of the drop-in): pack `n` levels
 * (u8, DEVICE) the way packedArray stores them (packed_array.go:34-101): width
 * bw = bits.Len16(max_level), each group of 8 levels in bw bytes in the
 * unpack8int32 layout (LSB first, bitbacking32.go), the last group zero padded
 * (packedArray.flush).  `packed` (DEVICE) receives ceil(n/8) * bw bytes; a
 * packedArray refill takes the floor(n/8) * bw bytes as `data` and the last
 * n % 8 levels as its pending buffer. */
int pqg_pack_levels(pqg_ctx* ctx, const uint8_t* levels, int64_t n, int max_level, uint8_t* packed);

/* After pqg_sync: page table of job `job` (host copy).  Returns pages written
 * or a negative status. */
int pqg_get_pages(pqg_ctx* ctx, int job, pqg_page_info* out, int cap);

/* Kernel timing of the last decode (HIP events on the ctx stream), in ms:
 * out[0] = whole pipeline, out[1..] = per stage. Returns the
 * number of entries written. */
int pqg_last_timings(pqg_ctx* ctx, float* out, int cap);

/* Per-stage HIP events on the ctx stream (on by default): `on` = 0 records
 * none (pqg_last_timings then returns 0 entries until a timed decode), 1
 * records them.  The
 * events are instrumentation: each costs a few microseconds of stream time,
 * which matters for small batches. */
int pqg_set_timing(pqg_ctx* ctx, int on);

/* Optional: run `iters` back-to-back decodes of the same jobs on the ctx
 * stream and return the device time in ms (used by bench.py).  */
int pqg_bench_decode(pqg_ctx* ctx, const pqg_chunk_job* jobs, int n_jobs, int iters,
                     float* ms_total, float* ms_stage, int stage_cap);

/* Diagnostics of the last decode for job `job` (after pqg_sync): out[0] = 1
 * when its page list came from the serial header walk (K1e) instead of the
 * speculative parallel scan, out[1] = header candidates found, out[2] =
 * pages, out[3] = decompressed scratch bytes, out[4] = pipeline launches of
 * the whole last decode call (1 unless an arena had to grow; grown capacities
 * are remembered per chunk for later calls).  Returns entries written. */
int pqg_debug_job(pqg_ctx* ctx, int job, int64_t* out, int cap);

/* Diagnostic builds only (compiled with -DPQG_PROFILE): in-kernel phase cycle
 * counters accumulated since the last call, then reset.  Returns the number of
 * counters written (0 in normal builds). */
int pqg_debug_counters(pqg_ctx* ctx, uint64_t* out, int cap);

/* ---- K8: level assembly (null scatter / record and list offsets) ----------
 * Replaces the per-slot cursor walk of ColumnStore.get (data_store.go:158-203)
 * and Column.getData (schema.go:235-264): a slot with dLevel < maxD is a null
 * (level cursor advances, value cursor does not); a slot with rLevel <
 * maxR ends the current repeated object.  Evaluated for every slot at once:
 *   valid(i)    = def[i] == max_def          (def_levels NULL → all valid)
 *   boundary(i) = rep[i] <= boundary_level   (rep_levels NULL → every slot)
 * boundary_level 0 = record starts (rLevel 0 → new row); max_rep-1 = the
 * objects ColumnStore.get returns.  All pointers are DEVICE pointers (e.g. a
 * pqg_chunk_result's def_levels/rep_levels/values); any output may be NULL. */
typedef struct pqg_assemble_args {
  const uint8_t* def_levels; /* num_slots bytes or NULL                          */
  const uint8_t* rep_levels; /* num_slots bytes or NULL                          */
  const uint8_t* values;     /* dense fixed-width values (num_valid × width)     */
  int64_t num_slots;
  int32_t max_def;
  int32_t boundary_level;
  int32_t value_width;       /* bytes per value; needed when values_spaced set   */
  int32_t reserved;
  uint8_t* validity;         /* out: ceil(num_slots/8) bytes, LSB-first bits     */
  uint8_t* values_spaced;    /* out: num_slots × value_width, nulls zeroed       */
  int64_t* offsets;          /* out: num_boundaries+1 entries (cap num_slots+1): */
                             /* the SLOT index of each boundary, then num_slots  */
                             /* (a null or empty list still takes its slot; for  */
                             /* Arrow LIST element offsets: pqg_assemble_list)   */
  int64_t num_valid;         /* out: #valid slots (= notNull total)              */
  int64_t null_count;        /* out: num_slots - num_valid                       */
  int64_t num_boundaries;    /* out: #boundary slots (rows / objects)            */
} pqg_assemble_args;

/* Enqueue K8 on the ctx stream and wait; fills the three counts. */
int pqg_assemble(pqg_ctx* ctx, pqg_assemble_args* args);

/* ---- K8 list export: Arrow LIST layout of a repeated leaf (max_rep == 1) ----
 * The record assembly of a LIST column (Column.getData schema.go:235-264 over
 * ColumnStore.get data_store.go:158-203) evaluated for every slot at once:
 *   row start     rep[i] == 0 (rep_levels NULL: every slot)
 *   element slot  def[i] >= elem_def          (the repeated group is present)
 *   valid element def[i] == max_def           (consumes the next dense value)
 *   row validity  def[row start] >= list_def  (else the list itself is null)
 * For the 3-level LIST<T> written by parquet-mr / pyarrow (optional group (LIST)
 * { repeated group list { optional T element } }: maxD = 3, maxR = 1):
 * list_def = 1, elem_def = 2 — def 0 null list, 1 empty list, 2 null element,
 * 3 value.  Outputs (DEVICE pointers, any may be NULL):
 *   list_validity  one bit per row, LSB first           (zeroed by the call)
 *   list_offsets   int32[rows + 1]: elements before each row, then the total
 *   elem_validity  one bit per element, LSB first       (zeroed by the call)
 *   elem_values    elements x value_width, null elements zeroed
 * Buffers must hold rows / elements <= num_slots entries; the two bitmaps are
 * written as whole dwords: give them 4 * ceil(num_slots / 32) bytes. */
typedef struct pqg_list_args {
  const uint8_t* def_levels; /* num_slots bytes (required)                        */
  const uint8_t* rep_levels; /* num_slots bytes or NULL                           */
  const uint8_t* values;     /* dense values (num_valid x value_width)            */
  int64_t num_slots;
  int32_t max_def;
  int32_t list_def;
  int32_t elem_def;
  int32_t value_width;
  uint8_t* list_validity;
  int32_t* list_offsets;
  uint8_t* elem_validity;
  uint8_t* elem_values;
  int64_t num_rows;          /* out */
  int64_t num_elements;      /* out */
  int64_t num_valid;         /* out: valid elements (= dense values consumed)     */
  int64_t null_lists;        /* out */
} pqg_list_args;

/* Enqueue the list export on the ctx stream and wait; fills the counts.
 * PQG_ERR_INVALID_ARG when elements exceed int32 offsets. */
int pqg_assemble_list(pqg_ctx* ctx, pqg_list_args* args);

/* Device time (ms) of the K8 kernels of the last pqg_assemble /
 * pqg_assemble_list call: HIP events on the ctx stream around its kernel
 * launches (the count read-back and host syncs excluded). */
int pqg_last_assemble_ms(pqg_ctx* ctx, float* ms);

/* ---- host-side planner: footer / schema (file_meta.go:14-62, schema.go) --- */
typedef struct pqg_file pqg_file;

typedef struct pqg_column_info {
  pqg_column_desc desc;
  char path[256];        /* dotted flat name (schema.go flatName) */
} pqg_column_info;

typedef struct pqg_chunk_meta {
  int64_t start;                 /* DictionaryPageOffset if set else DataPageOffset */
  int64_t total_compressed_size;
  int64_t total_uncompressed_size;
  int64_t data_page_offset;      /* absolute */
  int64_t num_values;
  int32_t has_dict_page_offset;
  int32_t codec;
  int32_t type;                  /* ColumnMetaData.type */
  int32_t reserved;
} pqg_chunk_meta;

/* Parse a whole parquet file held in host memory: PAR1 magic at both ends,
 * footer length, thrift FileMetaData, schema → leaf columns with maxD/maxR. */
int pqg_file_open(const uint8_t* file, int64_t len, pqg_file** out);
/* The same from the file's first head_len bytes and its LAST tail_len bytes
 * (file_len in all): a range reader's footer fetch.  PQG_ERR_INVALID_ARG when
 * the tail is shorter than the footer + 8 bytes (read the i32 footer length
 * in the last 8 bytes, then fetch footer + 8). */
int pqg_file_open_tail(const uint8_t* head, int64_t head_len, const uint8_t* tail, int64_t tail_len, int64_t file_len,
                       pqg_file** out);
void pqg_file_close(pqg_file* f);
int pqg_file_num_columns(const pqg_file* f);
int pqg_file_num_row_groups(const pqg_file* f);
int64_t pqg_file_num_rows(const pqg_file* f);
/* PQG_ERR_METADATA when the column's dotted path does not fit pqg_column_info.path */
int pqg_file_column(const pqg_file* f, int col, pqg_column_info* out);
int pqg_file_chunk(const pqg_file* f, int row_group, int col, pqg_chunk_meta* out);
int64_t pqg_file_row_group_rows(const pqg_file* f, int row_group);

/* The schema tree below the root, depth first (makeSchema / readGroupSchema
 * schema.go:789-894, 996-1025): what NextRow's row assembly walks
 * (Column.getData schema.go:171-264).  Replaces the Column tree the reference
 * builds for FileReader. */
typedef struct pqg_schema_node {
  char name[128];
  int32_t repetition;    /* 0 REQUIRED, 1 OPTIONAL, 2 REPEATED */
  int32_t num_children;  /* 0 for a leaf */
  int32_t leaf;          /* column index of a leaf (pqg_file_column), -1 for a group */
  int32_t max_def, max_rep;
  int32_t reserved;
} pqg_schema_node;
int pqg_file_num_schema_nodes(const pqg_file* f);
/* PQG_ERR_METADATA when the node's name does not fit pqg_schema_node.name (a
 * truncated name would be a different map key than the reference's) */
int pqg_file_schema_node(const pqg_file* f, int i, pqg_schema_node* out);

/* ======================= oracle (TEST INFRASTRUCTURE) ===================== */
/* Implemented only by oracle/liboracle.so.  Host pointers everywhere. */
int pqo_decode_chunk(const pqg_chunk_job* job, pqg_chunk_result* res,
                     pqg_page_info* pages, int page_cap, int* n_pages);
void pqo_free_result(pqg_chunk_result* res);
int pqo_unpack8_32(const uint8_t* data, int width, int32_t* out8);
int pqo_unpack8_64(const uint8_t* data, int width, int64_t* out8);
/* hybrid RLE/bit-pack: decode `count` values of `width` bits (levelDecoder.next) */
int pqo_hybrid_decode(const uint8_t* buf, int64_t len, int width, int64_t count, int32_t* out);
int pqo_snappy_decode(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap, int64_t* out_len);
int pqo_delta_decode64(const uint8_t* buf, int64_t len, int64_t count, int64_t* out);
int pqo_delta_decode32(const uint8_t* buf, int64_t len, int64_t count, int32_t* out);
/* Reference column-store contents (triage of Q1/Q2): decode the chunks of one
 * column over `n_row_groups` consecutive row groups the way readRowGroup fills
 * ColumnStore.values (readPageData chunk_reader.go:380-402), with the quirks in
 * `quirks` reproduced (Q2 requires Q1, as in the reference).  Per row group:
 * `entries` store slots, `nil_flags` one byte per entry; fixed width:
 * `values` entries x value_width bytes (a nil slot is zeros); byte arrays
 * (value_width 0): `values` the entries' bytes back to back (`chars` of them)
 * and `offsets[entries + 1]` (a nil entry is empty).  Q2 follows Go 1.13's
 * slice growth (runtime growslice + malloc size classes) for []interface{}:
 * outside /root/reference, stated in the oracle, so parity for it is unpinned. */
typedef struct pqo_store_rg {
  int32_t status;
  int32_t value_width;
  int64_t entries;
  uint8_t* values;
  uint8_t* nil_flags;
  int64_t* offsets;
  int64_t chars;
} pqo_store_rg;
int pqo_decode_column_store(const pqg_chunk_job* jobs, int n_row_groups, int quirks, pqo_store_rg* out);
void pqo_free_store(pqo_store_rg* out, int n_row_groups);
/* CPU-baseline helper: decode data pages [page_lo, page_hi) of a chunk (its
 * dictionary page always), for a thread pool over pages; *out_bytes = output
 * bytes of those pages.  Returns the number of data pages, or a status < 0. */
int64_t pqo_decode_page_range(const pqg_chunk_job* job, int page_lo, int page_hi, int64_t* out_bytes);
/* K8 restatements (host pointers): the ColumnStore.get / getData cursor walks */
int pqo_assemble(pqg_assemble_args* args);
int pqo_assemble_list(pqg_list_args* args);
/* packedArray layout of levels (host pointers): see pqg_pack_levels */
int pqo_pack_levels(const uint8_t* levels, int64_t n, int max_level, uint8_t* packed);
/* test hook of the Q2 emulation: Go 1.13 malloc size-class rounding */
int64_t pqo_go_roundupsize(int64_t size);

#ifdef __cplusplus
}
#endif
#endif /* PQGPU_H */
