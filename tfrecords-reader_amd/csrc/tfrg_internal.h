// tfrg_internal.h — device-side views shared by the kernels (tfrg_kernels.hip) and the C-ABI
// orchestration (tfrg_capi.cpp). Not part of the public ABI (include/tfrg.h is).
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

namespace tfrg {

// Device key table (the "schema"): distinct key byte strings, each with up to one slot per kind.
// A slot is one (key, kind) column of the columnar result.
struct DevSchema {
  uint32_t n_keys;
  uint32_t n_slots;
  uint32_t ht_mask;            // open-addressing table size - 1
  const uint32_t* ht;          // [ht_mask+1] key_id + 1, 0 = empty
  const uint32_t* key_hash;    // [n_keys] FNV-1a of the key bytes
  const uint32_t* key_off;     // [n_keys+1] into key_blob
  const uint8_t* key_blob;
  const int32_t* key_slot;     // [n_keys*4]: [0] flags (bit0 invalid UTF-8), [1..3] slot per kind or -1
  const uint8_t* slot_kind;    // [n_slots]
  const uint32_t* key_w;       // [n_keys][2]: first / last 4 key bytes (see key_hash_words)
  const uint32_t* krec;        // [n_keys][8] packed key record, see KeyRec
  const uint32_t* tpl;         // [n_tpl][kLtWords] record-shape templates in window form (below)
  const uint32_t* tpl_img;     // their lane image (kLiHdr ...), tpl_img_words words
  uint32_t tpl_img_words;
  uint32_t n_tpl;
  uint32_t tpl_w;              // their window words W (16, 32 or 64)
  // [n_slots] speculative placement of single values (null = off): 0, or (rank + 1) << 2 | kind for
  // a slot that is an inline single value in every learned template, as are all slots of its kind
  // before it. The lane kernel then writes such a value straight to its column at n * rank + r (the
  // row split r stays implicit for the first 64 slots); k_down_gather skips the slot when every
  // record was regular (irr == 0) and the slot's column base is n * rank, i.e. when that placement
  // is the final one (tfrg_info.placed_slots), and writes all its row splits otherwise.
  const uint32_t* spec;
};

// Record-shape template: the payload of a canonical record whose every byte except list contents is
// fixed (keys, tags, lengths, entry order; for packed int64 lists the continuation bits, i.e. the
// varint boundaries). A record equal to it under the mask has exactly the template's dict (slots,
// ranks, counts, list locations), which k_tpl_lane (tfrg_tpl.hip) writes without a walk. Learned on
// the host (tfrg_learn_templates) and stored in WINDOW form: the last 4 W bytes of the framed record,
// [end - 4 W, end), as W little-endian words, so that the length field, its masked CRC, the payload
// and the stored data CRC (word W - 1) sit at template-constant positions for every record of the
// shape. Per window word: Bm = fixed bytes & mask, Mm = mask (0 outside the record, for the data
// CRC and for variable payload bits), Cm = the variable payload bits (the CRC's input). Payload
// byte p of a length-L record is window byte y = p + 4 W - 4 - L, at distance d = 4 W - 5 - y from
// the payload end; d < 32 for words W - 9 .. W - 2.
// Layout (u32): [kLtL] L, [kLtNe] entries, [kLtCrcw] bit j: word W - 9 + j has variable payload
// bits, [kLtChain] first word < W - 9 with variable payload bits (W: none), [kLtK] CRC-32C of the
// payload with every variable bit 0, [kLtAbsent] slots (< kLeanMaxSlots) absent from the shape,
// [kLtEnt + 4 e] entries {slot | mode << 8 | spec << 12 | len << 16, rank, count word, pos}; mode 0:
// list location (pos = payload offset, len), 1: inline int64 varint of len bytes at window byte pos,
// 2: inline float at window byte pos, 3: inline bytes element of len bytes, pos = payload offset -
// 4 - L (the element's batch offset is end + pos); [kLtWin, +W) Bm, [+W, +2W) Mm, [+2W, +3W) Cm;
// [kLtSlot + 3 k] the same entries by SLOT k (< kLeanMaxSlots), so that k_tpl_lane stores slot k's
// columns once for the lanes of every template: {mode | len << 8 | rank << 16 (0: absent), pos,
// count word (0: absent)}.
constexpr uint32_t kTplMaxL = 240, kTplMaxEntries = 16;  // (tfrg.h TFRG_TPL_MAX_PAYLOAD / _ENTRIES)
constexpr uint32_t kLtMaxW = 64;
constexpr uint32_t kLeanMaxSlots = 16;  // k_tpl_lane runs for schemas of at most this many slots
constexpr uint32_t kLtL = 0, kLtNe = 1, kLtCrcw = 2, kLtChain = 3, kLtK = 4, kLtAbsent = 5, kLtEnt = 8,
                   kLtWin = kLtEnt + 4 * kTplMaxEntries, kLtSlot = kLtWin + 3 * kLtMaxW,
                   kLtWords = kLtSlot + 3 * kLeanMaxSlots;
constexpr uint32_t kLeanTabOff = 51200;  // crc_tab words: T_d, d < 32, 256 entries each (slice-by-32)

// Lane image of the templates (k_tpl_lane): each lane matches the template its record's payload
// length selects, so the template words are read per lane from LDS, where the workgroup copies this
// image. Built on the host from the window-form templates (tfrg_learn_templates) and stored after
// them in the template buffer (DevSchema::tpl_img). u32 words:
//   header [0, kLiHdr): [0] templates, [1] W, [2] words per template (kLiTw), [3] union over the
//     templates of kLtCrcw, [4] the smallest kLtChain;
//   [kLiSlotQ + k] slot k (< kLeanMaxSlots): qlo | qhi << 8 | kLiQValue (some template holds an
//     inline int64 / float there, in window words qlo .. qhi + 1) | kLiQSingle (no template has more
//     than one value there);
//   [kLiLut, + kLiLutWords) bytes: for payload length L <= kTplMaxL the first template of that
//     length (0xff: none);
//   [kLiTpl + t kLiTw(W)] template t: [0] L, [1] K, [2] the next template of the same length
//     (0xff: none), [4, 4 + W) Bm, [4 + W, 4 + 2 W) Mm, [4 + 2 W, 4 + 3 W) Cm, then per slot k 4 words
//     {mode | len << 8 | rank << 16 (0: absent), pos, count word (0: absent), 0}
//     (tfrg_internal.h "Record-shape template" for the fields).
constexpr uint32_t kTplMaxLane = 32;  // templates kept for the lane kernel (the most frequent shapes; TFRG_TPL_MAX)
constexpr uint32_t kLiHdr = 8, kLiSlotQ = kLiHdr, kLiLut = kLiSlotQ + kLeanMaxSlots,
                   kLiLutWords = (kTplMaxL + 1 + 3) / 4, kLiTpl = (kLiLut + kLiLutWords + 3) & ~3u;
constexpr uint32_t kLiQValue = 1u << 16, kLiQSingle = 1u << 17;
__host__ __device__ constexpr uint32_t kLiTw(uint32_t W) { return 4 + 3 * W + 4 * kLeanMaxSlots; }
// LDS words the lane image may take: a workgroup's 64 KiB less k_tpl_lane's static 32 KiB of CRC
// tables and 512 B for its other static words (tfrg_tpl.hip asserts it). With W = 64 this keeps 30
// templates, not kTplMaxLane (learn_shapes drops the least frequent ones).
constexpr uint32_t kLiMaxWords = (65536u - 32768u - 512u) / 4u;

// Column targets of one slot for k_tpl_lane, computed on the host per decode.
struct LeanTgt {
  uint16_t* ord;   // order column of the slot
  uint32_t* cnt;   // count column
  uint2* loc;      // loc column
  uint32_t* rs;    // row-split column (speculative placement)
  void* v1;        // speculative placement: value column at n * (rank - 1) (int64 / float bits / bytes offset)
  uint32_t* v2;    // speculative placement of bytes: the length column at n * (rank - 1)
  uint32_t lim;    // speculative placement: records r < lim are stored (capacity)
  uint32_t kind;   // speculative placement kind (0: the slot is not placed speculatively)
  uint32_t pad[2];
};
struct LeanArgs {
  uint32_t n_tpl;
  uint32_t lane_max;
  uint32_t* tsum;  // tile sums, slot k's at k * tile_stride (nullptr: an optimistic decode, none stored)
  uint32_t n_slots;
  uint32_t tile_stride;
  uint32_t img_words;  // the templates' lane image (DevSchema::tpl_img), copied into LDS
  uint32_t gpw;    // (launch_tpl_lane) 64-record groups per wave: 1 or 2 (part of a tile: small batches,
                   // twice the waves, tile sums added atomically) or a multiple of 4 (whole tiles)
  uint32_t bsplit; // workgroups from this one on take 2 groups per wave, from group gsplit on (the
  uint32_t gsplit; // batch's tail in small pieces: the last workgroups dispatched finish together)
  const uint8_t* finish;  // optimistic decode: DevSchema::slot_kind, and the last workgroup finishes
                          // the decode (tpl_quiet_finish); nullptr: the passes after this kernel do
  uint32_t implicit;      // optimistic decode, TFRG_IMPLICIT_* columns not stored for template hits
                          // (constant: every record of a confirmed decode is one)
  LeanTgt tg[kLeanMaxSlots];
};

// Packed per-key record (8 x u32) staged into LDS by the lane kernels' fast path.
enum KeyRec : uint32_t { kKrHash = 0, kKrLen, kKrW0, kKrW1, kKrSlot1, kKrSlot2, kKrSlot3, kKrFlags, kKrWords };
constexpr uint32_t kLdsMaxKeys = 256;     // key tables up to this size are staged into LDS
constexpr uint32_t kLdsMaxHt = 1024;      // hash-table entries staged into LDS

// Key hash over (length, first 4 bytes, last 4 bytes), all little-endian and zero padded:
// w0 = bytes [0, min(n,4)), w1 = n > 4 ? bytes [n-4, n) : 0. For n <= 8 the triple (n, w0, w1)
// IS the key, so a table hit needs no byte compare. Every input bit is folded into 24-bit
// operands so that the device multiplies are full-rate v_mul_u32_u24 (v_mul_lo_u32 is quarter
// rate, and the lane kernel is VALU-bound).
__host__ __device__ inline uint32_t key_hash_words(uint32_t n, uint32_t w0, uint32_t w1) {
  const uint32_t a = (w0 ^ (w0 >> 11) ^ (n << 17)) & 0xffffffu;
  const uint32_t b = (w1 ^ (w1 >> 13) ^ (n << 7)) & 0xffffffu;
#if defined(__HIP_DEVICE_COMPILE__)
  // = the host's products mod 2^32 (both operands < 2^24); spelled out because the backend picks
  // the quarter-rate v_mul_lo_u32 for these once the masks are reassociated
  uint32_t p0, p1;
  asm("v_mul_u32_u24 %0, %1, %2" : "=v"(p0) : "v"(a), "v"(0x9E3779u));
  asm("v_mul_u32_u24 %0, %1, %2" : "=v"(p1) : "v"(b), "v"(0x85EBCBu));
  uint32_t h = p0 ^ p1;
#else
  uint32_t h = a * 0x9E3779u;
  h ^= b * 0x85EBCBu;
#endif
  return h ^ (h >> 15);
}

// Record offsets of a batch (tfrg_decode_device: u64 pairs; tfrg_decode_device32: u32 pairs, or u32
// ends alone for back-to-back records, record r > 0 starting where record r - 1 ends)
enum OffMode : uint32_t { kOffU64 = 0, kOffU32 = 1, kOffEnds = 2 };

struct DevBatch {
  const uint8_t* bytes;        // records (framed or bare payloads); readable to round_up(nbytes,16)
  uint64_t nbytes;
  const uint64_t* start;       // [n] absolute offsets into bytes (kOffU64)
  const uint64_t* end;         // [n]
  const uint32_t* start32;     // [n] (kOffU32)
  const uint32_t* end32;       // [n] (kOffU32, kOffEnds)
  uint32_t first;              // kOffEnds: start of record 0
  uint32_t omode;              // OffMode
  uint32_t n;
  uint32_t flags;
};

#if defined(__HIPCC__)
__device__ __forceinline__ uint64_t rec_end(const DevBatch& B, uint32_t r) {
  return B.omode == kOffU64 ? B.end[r] : (uint64_t)B.end32[r];
}
__device__ __forceinline__ uint64_t rec_start(const DevBatch& B, uint32_t r) {
  if (B.omode == kOffU64) return B.start[r];
  if (B.omode == kOffU32) return B.start32[r];
  return r ? (uint64_t)B.end32[r - 1] : (uint64_t)B.first;
}
#endif

// Info counters (device, zero at the start of every decode: the previous decode's k_lane_count
// zeroes the slot the next one uses, DevOut::info_next)
enum InfoIdx : uint32_t {
  kInfoErrors = 0,       // records with a decode error (reference exception / UB status)
  kInfoFirstError = 1,   // ~(lowest record index with an error): atomicMax of ~r, init 0
  kInfoMissRecords = 2,  // records with a schema miss
  kInfoMissEntries = 3,  // miss entries appended (may exceed capacity)
  kInfoBig = 4,          // records routed to the wave-per-record kernels
  kInfoScanTimeout = 5,  // reserved (always 0: the scan has no inter-workgroup waits)
  kInfoHuge = 6,         // wave records too large for the LDS stage (listed from the end of big_list)
  kInfoSlow = 7,         // lane records left to the exact (slow) walker
  kInfoSpineDone = 8,    // spine workgroups finished (the last one computes the column bases)
  kInfoNeed = 9,         // lane records with an out-of-line list (k_tail_gather; listed in slow_list)
  kInfoSpineTicket = 10, // k_spine workgroup tickets (chunk order of the look-back)
  kInfoOverflow = 11,    // a kind's value total exceeds its column capacity (overlapping ranges)
  kInfoBytesTicket = 12, // k_bytes_scan tile tickets
  kInfoBytesBig = 13,    // k_bytes_scan: long elements listed for the wave copy
  kInfoCrcCtr = 14,      // [14..15] u64: streaming-CRC list entries << kCrcIdxShift | flat 1 KiB rounds
  kInfoDefer = 16,       // k_lane_count: 64-record rows of deferred packed-int64 bodies reserved (k_body_count)
  kInfoResid = 17,       // k_tpl_lane: 64-record groups listed for k_lane_count (records no template took)
  kInfoPlacedLo = 18,    // [18..19] k_down_gather: the (first 64) slots whose speculative placement is final
  kInfoPlacedHi = 19,
  kInfoTplDone = 20,     // [20..21] u64, optimistic decodes: k_tpl_lane workgroups finished | groups
                         // they listed << 32 (one atomic: the last workgroup knows the total)
  kInfoBigRecs = 22,     // records above lane_max (tfrg_info.n_big; kInfoBig + kInfoHuge count the
                         // ones listed for the wave gathers: those with out-of-line lists)
  kInfoWalkMiss = 23,    // records above lane_max walked beside the CRC (k_tail_count) that the
                         // canonical walker did not take or that have an out-of-line list: re-run
  kInfoCount = 24        // (even: the two slots' u64 words stay 8-byte aligned)
};
static_assert(kInfoCount % 2 == 0 && kInfoCrcCtr % 2 == 0 && kInfoTplDone % 2 == 0,
              "u64 info words stay 8-byte aligned in both slots");

// Deferred packed int64 bodies of records walked from HBM (k_lane_count -> k_body_count): a wave
// reserves one block of 64 rows, row = one record, kDeferK entries (record, slot, absolute body
// offset, length) and a count byte per row
constexpr uint32_t kDeferK = 32;
// status of a record whose deferred body did not count canonically (k_body_count): k_tail_count's
// exact walker withdraws its columns and re-walks it (never left in the status column)
constexpr int32_t kStatusRedo = 0x7fff0001;

// verdict byte of a record the lane kernel left to the exact walker (k_tail_count role 1 writes its
// final verdict, payload CRC included); role 2 (payload CRCs of large records) never lists such
// records (a record k_body_count sends back is on both lists: role 2 ORs its bit in atomically)
constexpr uint32_t kVerdictPending = 0x80u;

// streaming payload CRC of the large records (k_tail_count role 2)
constexpr int kCrcIdxShift = 40;
constexpr uint64_t kCrcRoundMask = (1ull << kCrcIdxShift) - 1ull;
constexpr uint32_t kCrcListMin = 64;  // shorter payloads of large records: the lane kernel's serial CRC

// count column: bit 31 set = the slot's single value is stored inline in the loc word
constexpr uint32_t kCountInline = 0x80000000u;

struct DevOut {
  int32_t* status;       // [n]
  int64_t* aux;          // [n] error detail
  uint8_t* verdict;      // [n] tfrg_verdict bits
  uint16_t* order;       // [n_slots][n]  0 = absent, else 1 + rank in the record's key order
  uint32_t* count;       // [n_slots][n]
  uint2* loc;            // [n_slots][n]  (payload-relative offset, length) of the list message
  uint32_t* rs;          // [n_slots][n+1] row splits (exclusive prefix of count)
  uint64_t* slot_base;   // [n_slots] element base of each slot inside its kind's value array
  uint32_t* totals;      // [n_slots]
  uint64_t* kind_totals; // [4]
  int64_t* i64;          // int64 values
  uint32_t* f32;         // float values (raw bits)
  uint32_t* b_off;       // bytes_list element views: absolute offset into bytes
  uint32_t* b_len;
  uint64_t cap_i64, cap_f32, cap_b;
  uint32_t* big_list;    // records for the wave-per-record kernels
  uint32_t* miss;        // [miss_cap][4] (record, kind, key abs offset, key length)
  uint32_t miss_cap;
  uint32_t* info;        // [kInfoCount]
  uint32_t* info_next;   // [kInfoCount] the next decode's info words (k_lane_count workgroup 0 zeroes them)
  uint32_t* tsum;        // [n_slots][tile_stride] per-tile value counts, then their exclusive prefixes
  uint32_t tile_stride;  // >= n_tiles, multiple of 4
  uint64_t* spine_lb;    // [n_slots][n_chunks] k_spine look-back words: flag << 32 | chunk total / inclusive
                         // prefix (flag 1 / 2; zeroed per decode with tsum)
  uint32_t n_chunks;     // ceil(n_tiles / 2^kSpineChunkShift)
  uint32_t* slow_list;   // [n] lane records for the exact walker; reused by k_down_gather for the
                         // records k_tail_gather decodes (the slow list is consumed by then)
  uint32_t* crc_rec;     // [n] streaming-CRC list: record
  uint64_t* crc_base;    // [n] its first flat round (ascending with the list index)
  uint64_t* crc_part;    // [n] rounds done << 32 | XOR of the slices, of a record split over waves
  uint32_t* irr;         // [n_slots] records not placed speculatively per slot (DevSchema::spec; after
                         // the scan words in their buffer, zero between decodes: k_tail_gather clears)
  uint4* dq;             // [dq_blocks][64][kDeferK] deferred bodies (nullptr: no deferral this decode)
  uint8_t* dq_cnt;       // [dq_blocks][64] entries used per row (0 for records not accepted)
  uint32_t dq_blocks;
  uint64_t* lmask;       // [groups] k_tpl_lane: per 64-record group, the records it did not take (null: not run)
  uint32_t* rlist;       // [groups] k_tpl_lane: the groups with such records (null: k_lane_count takes all)
};

// Row-split scan tiles: 256 consecutive records (one lane-kernel workgroup iteration)
constexpr uint32_t kTileShift = 8;
constexpr uint32_t kTileRecs = 1u << kTileShift;
// k_spine chunks: 2^12 tiles (1 M records) per workgroup
constexpr uint32_t kSpineChunkShift = 12;

// flags (mirrors include/tfrg.h)
constexpr uint32_t kFlagPayloadOnly = 1u;
constexpr uint32_t kFlagSpecVarint = 2u;
constexpr uint32_t kFlagNoCrc = 4u;
constexpr uint32_t kFlagStrictCrc = 8u;
constexpr uint32_t kFlagMaterializeBytes = 16u;


// TFRG_FLAG_MATERIALIZE_BYTES (tfrg_bytes.hip): bytes_list elements gathered into one column
struct DevBytes {
  const uint8_t* in;             // batch bytes
  uint64_t in_readable;          // round_up(nbytes, 16)
  const uint32_t* b_off;         // element views (absolute offset, length)
  const uint32_t* b_len;
  const uint64_t* kind_totals;   // [1] = element count (k_spine)
  uint64_t* offsets;             // [nb + 1] exclusive prefix of the lengths
  uint64_t offsets_cap;          // elements the offsets buffer holds (cap_b)
  uint8_t* data;                 // the byte column
  uint64_t data_cap;
  uint64_t* lb;                  // look-back words (zeroed per decode)
  uint32_t* ticket;              // scan tile tickets (zeroed per decode)
  uint32_t* big_count;           // elements longer than the short-copy bound (zeroed per decode)
  uint32_t* big_list;            // [cap_b]
  uint32_t* overflow;            // info[kInfoOverflow]
};
hipError_t launch_materialize(const DevBytes& d, int num_cus, hipStream_t st);
uint64_t materialize_lb_words(uint64_t cap_b);

// launchers (tfrg_kernels.hip)
struct LaunchCfg {
  int num_cus;
  bool lean;               // k_tpl_lane first (window-form templates, framed records with CRCs)
  bool tpl_full;           // the templates took their whole learning sample (the later passes are
                           // then usually empty: launched with small grids)
  const uint32_t* spec_h;  // host copy of DevSchema::spec (k_tpl_lane's placement targets)
  int lane_grid;           // cap: workgroups for one record per lane
  int wave_grid;
  uint32_t lane_max;       // records above this size go to the wave kernels
  uint32_t wave_stage;     // wave records spanning <= this many bytes are staged in LDS (<= kWStage)
  bool body_count;         // deferred packed bodies possible (DevOut::dq): launch k_body_count
  uint32_t poison[4];      // debug hook (env TFRG_DEBUG_POISON_LOC): records whose list locations are
                           // overwritten after the count passes (0xffffffff: none)
  bool optimistic;         // allow an optimistic decode (launch_all: k_tpl_lane alone)
  bool ran_optimistic;     // (out) this decode was launched optimistically: it is complete only once
                           // the host has read kInfoResid as 0 (else it is re-run in full)
  bool ord_const;          // every learned shape has every slot at the same key position
  bool len_const;          // every bytes slot one element of one length in every learned shape
  bool ran_quiet_big;      // (out) optimistic without shapes: k_tail_count's last workgroup ends it
  bool walk_beside;        // optimistic without shapes: records above lane_max walked beside the CRC
                           // (k_tail_count's first workgroups) instead of before it (k_lane_count)
  uint32_t walk_blocks;    // cap on those workgroups (0: automatic)
  uint32_t implicit;       // (out) TFRG_IMPLICIT_* columns the decode did not store
};

// Kernel stages, in launch order (profiling events bracket each one).
enum Stage : int { kStageTplLane = 0, kStageLaneCount, kStageBodyCount, kStageTailCount, kStageSpine,
                   kStageDownGather, kStageTailGather, kStageMaterialize, kNumStages };
extern const char* const kStageNames[kNumStages];

// ev: optional kNumStages + 1 events recorded on `stream` before each stage and after the last.
hipError_t launch_tpl_lane(const DevBatch& b, const DevOut& o, const LeanArgs& a, const uint32_t* img, uint32_t w,
                           const uint32_t* d_tab, int num_cus, hipStream_t st);
hipError_t launch_fill_placed_rows(uint32_t* rs, const uint32_t* info, uint32_t n_slots, uint32_t n, hipStream_t st);
hipError_t launch_stream_read(const void* d, uint64_t nbytes, uint32_t* sink, hipStream_t st, int variant);
hipError_t launch_decode(const DevBatch& b, const DevSchema& sc, const DevOut& o, LaunchCfg& cfg,
                         const uint32_t* d_crc_tables, const uint32_t* d_wave_consts, hipStream_t stream,
                         hipEvent_t* ev);

}  // namespace tfrg
