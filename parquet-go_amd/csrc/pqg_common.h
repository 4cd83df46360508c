// pqg_common.h — device/host shared records of the gfx950 decode pipeline.
//
// Layout in HBM (one ctx, one batch of chunk jobs):
//   JobDev[n_jobs]             per column chunk: inputs, arena regions, results
//   PageDev[page_cap_total]    page table; job j owns [page_base, page_base+page_cap)
//   level arena  (u8)          def/rep levels, job j at slot_base (num_slots each)
//   value arena  (bytes)       dense values[:nn], job j at value_base
//   scratch arena (bytes)      decompressed (snappy) page blocks, job j at scratch_base
//   offsets arena (i64)        variable-length value offsets
#pragma once
#include <stdint.h>

#ifndef __HIPCC__
#ifndef __host__
#define __host__
#define __device__
#define __forceinline__ inline
#endif
#endif

namespace pqg {

enum : int32_t {
  kOK = 0,
  kEOF = -1,
  kTHRIFT = -2,
  kPAGE_HEADER = -3,
  kSIZE = -4,
  kSNAPPY = -5,
  kRLE = -6,
  kDICT_INDEX = -7,
  kBIT_WIDTH = -8,
  kDELTA = -9,
  kUNSUPPORTED = -10,
  kDICT_PAGE = -11,
  kBYTE_ARRAY = -12,
  kLEVELS = -13,
  kFIXED_LEN = -14,  // DELTA_BYTE_ARRAY on FLBA: a value of another length than type_length
  kGZIP = -15,       // gzip: invalid header, DEFLATE data or checksum
  kCAPACITY = -20,
  kCOMPLEX = -30,   // internal: header needs the serial walk (deep thrift nesting)
};

// Header fields of one page (thrift PageHeader subset, parquet.go:5794-5803).
struct PageHdr {
  int32_t type, usize, csize;
  int32_t num_values, encoding, def_enc, rep_enc;   // DataPageHeader / Dict / V2
  int32_t v2_def_len, v2_rep_len;
  int32_t has_dph, has_dict, has_v2;
  int32_t hlen;  // header bytes
};

struct PageDev {
  int64_t header_offset;   // relative to job data
  int64_t payload_offset;  // header_offset + hlen
  int64_t slot_offset;     // Σ num_values of preceding data pages (job-relative)
  int64_t value_offset;    // Σ not_null of preceding data pages (job-relative)
  int64_t scratch_offset;  // decompressed block (job-relative), -1 = not compressed
  // resolved streams (absolute device pointers, filled by the level stage)
  const uint8_t* block;    // values block (V1: the whole page body)
  int64_t block_len;
  const uint8_t* rep;  int64_t rep_n;
  const uint8_t* def;  int64_t def_n;
  const uint8_t* val;  int64_t val_n;
  int32_t page_type, encoding, num_values, csize, usize;
  int32_t def_len, rep_len, def_enc, rep_enc;
  int32_t job;
  int32_t read_status;     // error of the reference's read phase (readPages)
  int32_t decode_status;   // error of readValues (readPageData)
  int32_t not_null;
  int32_t flags;
  int32_t dict_width;      // RLE_DICTIONARY: index bit width byte
  int32_t hs_rep, hs_def, hs_val;  // hybrid streams of the page (HStream index, -1: none)
  int32_t vmode;           // values stage of the page: 1 4-byte dictionary, 3 DELTA_BINARY_PACKED, 0 other fixed width, 2 variable, -1 none
  int64_t run_off, blk_off;  // the page's run-table / block-index region (job-relative, k_page_list)
  // variable-length values (BYTE_ARRAY, FLBA of length 0): chars of the page
  // and their offset in the chunk's chars (exclusive scan over the pages)
  int64_t chars;
  int64_t char_offset;
  // DELTA_LENGTH_BYTE_ARRAY / DELTA_BYTE_ARRAY: where the value bytes (the
  // suffixes) start in the values section, after the DBP length stream(s)
  int64_t cstart;
  // K2 snappy split (pqg_snappy.hip, k_snap_plan): bytes of the block's
  // length varint, 64 KiB output sub-blocks and their SnapSub entries, 4 KiB
  // compressed segments, and the serial-fallback flag (non-zero: k_snappy
  // decodes the page as one block)
  int32_t sn_hdr, sn_nsub, sn_sub_base, sn_nseg, sn_seg_base, sn_fallback;
  int64_t gz_len;          // K2g (pqg_inflate.hip), bare blocks: decoded bytes
};
constexpr int32_t kPageBareBlock = 1 << 4;  // PageDev.flags: a pqg_block_decompress block (no page around it)
constexpr int32_t kPageInflateRedo = 1 << 6;  // PageDev.flags: a GZIP page for k_inflate's 32 KiB ring (k_inflate_s left it)
constexpr int32_t kCodecSnappy = 1, kCodecGzip = 2;

// K2 snappy sub-block: the output [j * kSnapSub, (j + 1) * kSnapSub) of one
// compressed block, decoded by one wave from a chain tag at or before its
// start (found by k_snap_link from the segment exits of k_snap_seg).
constexpr int kSnapSub = 65536;   // golang/snappy maxBlockSize (snappy.go:72)
constexpr int kSnapSeg = 4096;    // compressed bytes per segment of the tag-chain search
struct SnapSub {
  int32_t page;  // PageDev index
  int32_t j;     // sub-block of the page
  int32_t pos;   // block offset of a chain tag whose output starts at `out` (-1: not found)
  int32_t out;   // output offset of that tag (<= j * kSnapSub)
};

// One RLE/bit-packed hybrid stream (hybrid_decoder.go): a page's rep or def
// levels, its dictionary indices or its RLE booleans.  k_page_setup registers
// it, k_hybrid_walk turns it into a run table, the expanders read the table.
struct HStream {
  const uint8_t* p;  // first byte of the stream
  int64_t n;         // stream bytes (reads at or past n are EOF)
  int64_t run_base;  // first RunEnt of the stream's run table
  int64_t blk_base;  // first BlockDesc of the stream
  int32_t page;      // PageDev index
  int32_t kind;      // 0 rep, 1 def, 2 dictionary indices, 3 RLE booleans
  int32_t w;         // bit width (1..32)
  int32_t count;     // values wanted (levels: NumValues; values: an upper bound of notNull)
  // walker results
  int32_t n_runs;
  int32_t produced;  // values available before the end of the stream / an error
  int32_t status;    // error met after `produced` values (kOK: none before `count`)
  int32_t n_blocks;  // BlockDescs written
};

// A block of a stream's values for the expanders: at most kHBlock values and
// kHBlockRuns runs, with the byte range of the bit-packed payload they use.
struct BlockDesc {
  uint32_t v0;      // first value index
  uint32_t r0;      // first run (index into the stream's run table)
  uint32_t lo;      // first payload byte used (stream offset)
  uint16_t nbytes;  // payload bytes used from lo (0: RLE only)
  uint16_t nr;      // runs in the block
};

// Run table entry: start = first value index of the run (bit 31: bit-packed);
// src = RLE value, or the byte offset of a bit-packed run's payload.
struct RunEnt {
  uint32_t start;
  uint32_t src;
};
constexpr uint32_t kRunBP = 0x80000000u;
constexpr int kHBlock = 512;      // values per expander block
constexpr int kHBlockRuns = 64;   // runs per expander block (one per lane)
constexpr int kHBlockBytes = 1008;  // payload bytes per block: 64 16-byte granules, aligned anywhere

// One 4-byte dictionary data page, as the values kernel needs it (k_dict_plan).
struct VRec {
  uint8_t* out;            // values[:nn] of the page
  const uint8_t* p;        // index stream (after the bit-width byte)
  const RunEnt* runs;      // the stream's run table
  const BlockDesc* blks;   // the stream's block index
  const uint8_t* dict;     // dictionary entries (null: none)
  int32_t n;               // stream bytes
  int32_t w;               // index bit width (0: every key is 0)
  int32_t nn;              // notNull
  int32_t count;           // keys to expand: min(nn, the stream's produced)
  int32_t n_blocks;
  int32_t dcount;          // dictionary entries
  int32_t job;             // -1: nothing to decode
  int32_t pidx;            // PageDev index
  int32_t serr;            // stream error met before nn keys (kOK: none)
  int32_t produced;        // keys before that error
};

struct JobDev {
  // ---- inputs
  const uint8_t* data;
  int64_t data_len, tcs, data_page_offset;
  int32_t type, type_length, max_def, max_rep, codec, has_dict_off;
  int32_t value_width;     // bytes per value, 0 = variable
  int32_t page_cap;
  int64_t page_base;
  int64_t slot_cap, slot_base;        // level arenas (bytes == slots)
  int64_t value_cap, value_base;      // value arena (bytes)
  int64_t scratch_cap, scratch_base;  // scratch arena (bytes)
  int64_t offs_cap, offs_base;        // offsets arena (entries)
  // ---- results (device written)
  int32_t num_pages;       // pages found by the walk (may exceed page_cap)
  int32_t dict_page;       // page index of the dictionary page, -1 if none
  int32_t scan_status;     // first read-phase error found by the walk
  int32_t status;          // final chunk status
  int32_t error_page;
  int32_t n_out_pages;     // pages reported (truncated at first read error)
  int64_t num_slots, num_values, values_bytes;
  int64_t need_scratch;    // Σ usize of compressed blocks
  const uint8_t* dict_data;  // dictionary entries (fixed width) or chars (var)
  int64_t dict_count, dict_len;
  const int64_t* dict_offs;  // variable-length dictionary: record start of each entry (count+1)
  int32_t flags;             // bit0 INT96 nil entry (Q8), bit1 variable-length dictionary to walk
  int32_t no_prewalk;        // host: the chunk is known not to be taken by the K1 prewalk / stride walk
  int64_t doffs_cap, doffs_base;  // dictionary-offsets arena region (entries)
  int64_t need_doffs;             // entries the dictionary needs (count+1)
  // ---- K1 speculative page scan (see k_page_cands / k_page_chain)
  int64_t tile_base;       // first scan tile of this job (global tile index)
  int32_t n_tiles;         // ceil(min(tcs, data_len) / kScanTile)
  int32_t scan_fallback;   // 1: the serial walk (k_scan_pages) decodes this job's page list;
                           // 2: walked before the candidate scan (a few big pages)
  int32_t n_cands;         // header candidates found in the job's bytes
  int32_t n_ok;            // candidates whose read phase succeeds
  int32_t brk;             // first ok-rank whose successor is not the next ok candidate
  int32_t first_dict;      // first ok-rank of a dictionary page
  // ---- K3 hybrid run tables (pqg_levels.hip)
  int64_t run_cap, run_base;   // RunEnt arena region
  int64_t blk_cap, blk_base;   // block-index arena region
  int64_t run_used, blk_used;  // run-table / block-index entries the pages need (k_page_list)
  // ---- values-stage work items of the job (k_part_plan): parts [item_base, item_base + n_items)
  int64_t item_base;
  int32_t n_items, pad2;
};

// ---------------------------------------------------------------------------
// Big pages (parquet-go's own writer puts a whole column chunk in ONE data
// page, chunk_writer.go:237-246, with each level / index stream one
// bit-packed run, hybrid_encoder.go:59-73).  The values stages work on PARTS:
// a page of at most kSplitMin values is one part; a bigger one is cut into
// parts of about kPart values, each decoded by its own wave / workgroup.
//   PLAIN (fixed width or byte arrays): values [p kPart, (p + 1) kPart)
//   hybrid value streams (dictionary indices, RLE booleans): the blocks of the
//     stream's block index whose first value lies in [p kPart, (p + 1) kPart)
// Long runs inside the serial walks are handed to parallel kernels: level
// runs of more than kLongLev values (k_level_long) and value-stream bit-packed
// runs of more than kLongWalk values (k_walk_long).
// ---------------------------------------------------------------------------
constexpr int kSplitMin = 65536;
constexpr int kPart = 4096;
constexpr int kLongLev = 32768;
constexpr int kLevPiece = 16384;
constexpr int kLongWalk = 16384;
// counters (ints after the counters base, zeroed by k_page_list)
constexpr int kCtrItems = 48;     // values-stage parts of the batch
constexpr int kCtrLongLev = 49;   // long level runs
constexpr int kCtrLevPieces = 50; // pieces of the long level runs
constexpr int kCtrLongWalk = 51;  // long bit-packed runs of value streams
constexpr int kCtrPartsCap = 52;  // the parts table's capacity (k_nn_scan): consumers read min(items, this)

struct PartRec {
  int32_t pidx;    // PageDev index
  int32_t p, np;   // part p of np
  uint32_t v0;     // first value (page-relative); the part ends at the next part's v0, or the page's count
  int32_t b0;      // hybrid parts: first block (stream-relative); the part's blocks end at the next part's b0
  int32_t vmode;   // the page's values stage (PageDev.vmode)
  int64_t chars;   // byte arrays: chars of the part (k_str_count / k_char_scan)
  int64_t cstart;  // byte arrays: chunk char offset of the part's first value (k_char_scan)
  int64_t prel;    // byte arrays: page-relative char offset of the part's first value (k_char_scan)
};

// A level run of more than kLongLev values, expanded by k_level_long in
// pieces of kLevPiece values.
struct LongLev {
  uint8_t* out;       // level bytes of the run's first value
  const uint8_t* p;   // bit-packed: the run's payload (byte of its first value's bit 0); null for RLE
  const uint8_t* end; // stream end (bytes at or past it read as zero: the short-read padding, Q5)
  uint32_t count;     // values
  uint32_t value;     // RLE value
  int32_t w;          // bit width (1..8)
  int32_t maxl;       // def levels: maxD (notNull counted into the page); rep levels: 0x100
  int32_t pidx;       // PageDev index
  int32_t pad;
};
struct LevPiece {
  int32_t run;        // LongLev index
  uint32_t v0, v1;    // values of the run
};

// A bit-packed run of a value stream longer than kLongWalk values: its block
// descriptors (K values each) are written by k_walk_long.
struct LongWalk {
  int64_t blk;        // BlockDesc index (absolute) of the run's first block
  uint32_t v0;        // first value of the run (stream-relative)
  uint32_t take;      // values of the run that are used
  uint32_t run;       // its run-table index (stream-relative)
  uint32_t src;       // stream offset of its payload
  int32_t w, K;       // bit width, values per block
};

// k_hybrid_walk block size: its LDS layout (pqg_levels.hip) and its launch
// (pqg_runtime.hip) share this one definition.
#ifndef PQG_WALK_THREADS
#define PQG_WALK_THREADS 64
#endif
constexpr int kWalkThreads = PQG_WALK_THREADS;
#ifndef PQG_PW_THREADS
#define PQG_PW_THREADS 256
#endif
constexpr int kPwThreads = PQG_PW_THREADS;  // k_str_plain block size (PLAIN byte-array length walk)

// Work queues: kQShards heads kQStride ints apart (see queue_pull, pqg_device.h).
constexpr int kQShards = 8;
constexpr int kQStride = 32;
constexpr int kQueueInts = kQShards * kQStride;
// ints after the counters base (ctr[0] = page-list total): one flag per values
// stage (PageDev.vmode 0..3), set by k_page_levels when a page of that stage
// exists, so an empty stage's kernel exits at once instead of walking the list
constexpr int kModePresentOff = 1024 + 9 * kQueueInts;
// the serial snappy pass (k_snappy after the split decode) pulls its own queue
constexpr int kQueueSnapSerial = 10;
// DELTA_LENGTH_BYTE_ARRAY / DELTA_BYTE_ARRAY lengths (k_str_delta) and values (k_str_dba)
constexpr int kQueueStrDelta = 11;
constexpr int kQueueStrDba = 12;
constexpr int kQueueLevLong = 13;  // pieces of the long level runs (k_level_long)
constexpr int kQueueInflate = 14;  // GZIP pages (k_inflate)
constexpr int kQueueLevGen = 15;  // k_page_levels when k_page_levels_w1 takes the w = 1 jobs' pages
constexpr int kQueueDictBig = 16; // k_dict4_big: run-table pages of dictionaries past 4096 entries
constexpr int kQueueInflateRedo = 17;  // k_inflate (32 KiB ring) over the pages k_inflate_s left
// queue regions zeroed per launch: 0-8, the stage flags (9), 10-17
constexpr int kQueueSlots = 18;
constexpr int kPresentBigDict = 8;  // stage flag (kModePresentOff + 8): a page for k_dict4_big

// Scan tiles of the speculative page-header search.
constexpr int kScanTile = 16384;
constexpr int kPrewalkPages = 4;  // K1: chunks of <= this many big pages are walked, not scanned
constexpr int kCandPerTile = 64;

// A page-header candidate: a position whose bytes parse as a PageHeader
// (parsed by one lane, classified as if it were the chunk's first dictionary
// page when it is one).  The chain kernel keeps the ones reachable from
// position 0 by next-page links.
struct Cand {
  int64_t pos, next, payload;
  int64_t comp;            // scratch bytes of its decompressed block (16-rounded), 0 if none
  int32_t type, encoding, num_values, csize, usize;
  int32_t def_len, rep_len, def_enc, rep_enc;
  int32_t status;          // read-phase status, kCOMPLEX: re-parse serially
};

}  // namespace pqg
