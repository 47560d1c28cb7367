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
  const uint32_t* tpl;         // [n_tpl][kTplWords] record-shape templates (below), learned on the host
  uint32_t n_tpl;
  // [n_slots] speculative placement of single values (null = off): 0, or (rank + 1) << 2 | kind for
  // a slot that is an inline single value in every learned template, as are all slots of its kind
  // before it. The lane kernel then writes such a value straight to its column at n * rank + r and
  // the row split r; k_down_gather skips the slot when every record was regular (irr == 0) and the
  // slot's column base is n * rank, i.e. when that placement is the final one.
  const uint32_t* spec;
};

// Record-shape template: the payload of a canonical record whose every byte except list contents is
// fixed (keys, tags, lengths, entry order; for packed int64 lists the continuation bits, i.e. the
// varint boundaries). A record equal to it under the mask has exactly the template's dict (slots,
// ranks, counts, list locations): the lane kernel then skips the canonical walk and reads only the
// inline values. Layout (u32 words): [0] payload length L, [1] entries, [2] ceil(L/4), [3] 0,
// [4, 4+64) bytes, [68, 68+64) mask, [132, 132+4*16) entries {slot | mode << 24, rank, count word,
// a | b << 16}; mode 0: loc (a, b) = (list offset, list length), 1: inline int64 varint at a of b
// bytes, 2: inline float at a, 3: inline bytes element at a of b bytes.
// [196] K = U(0, (bytes & mask) with its first 4 bytes inverted) over the L bytes, [197] the masked
// CRC-32C of the 8 length bytes of L, [198] v0 = the first payload byte with a variable bit
// (0xffffffff: no CRC shortcut, L < 4). A matching record M = (bytes & mask) ^ V, V = M & ~mask, so
// its CRC-32C is ~(K ^ U(0, V[v0, L))) (U linear, crc32c.h): only the bytes from v0 on are read.
constexpr uint32_t kTplMaxL = 256, kTplMaxEntries = 16, kTplMax = 4;
constexpr uint32_t kTplBytes = 4, kTplMask = 68, kTplEnt = 132, kTplCrcK = 196, kTplLenCrc = 197, kTplV0 = 198,
                   kTplWords = 200;

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

struct DevBatch {
  const uint8_t* bytes;        // records (framed or bare payloads); readable to round_up(nbytes,16)
  uint64_t nbytes;
  const uint64_t* start;       // [n] absolute offsets into bytes
  const uint64_t* end;         // [n]
  uint32_t n;
  uint32_t flags;
};

// Info counters (device, zeroed per decode)
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
  kInfoNeed = 9,         // lane records with an out-of-line list (k_list_gather; listed in slow_list)
  kInfoSpineTicket = 10, // k_spine workgroup tickets (chunk order of the look-back)
  kInfoOverflow = 11,    // a kind's value total exceeds its column capacity (overlapping ranges)
  kInfoBytesTicket = 12, // k_bytes_scan tile tickets
  kInfoBytesBig = 13,    // k_bytes_scan: long elements listed for the wave copy
  kInfoCrcCtr = 14,      // [14..15] u64: streaming-CRC list entries << kCrcIdxShift | flat 1 KiB rounds
  kInfoDefer = 16,       // k_lane_count: 64-record rows of deferred packed-int64 bodies reserved (k_body_count)
  kInfoCount = 20
};

// Deferred packed int64 bodies of records walked from HBM (k_lane_count -> k_body_count): a wave
// reserves one block of 64 rows, row = one record, kDeferK entries (record, slot, absolute body
// offset, length) and a count byte per row
constexpr uint32_t kDeferK = 32;
// status of a record whose deferred body did not count canonically (k_body_count): k_tail_count's
// exact walker withdraws its columns and re-walks it (never left in the status column)
constexpr int32_t kStatusRedo = 0x7fff0001;

// verdict byte of a record the lane kernel left to the exact walker (k_tail_count role 1 writes its
// final verdict, payload CRC included); role 2 (payload CRCs of large records) skips such records,
// so the two roles of one launch never write the same verdict byte
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
  uint32_t* tsum;        // [n_slots][tile_stride] per-tile value counts, then their exclusive prefixes
  uint32_t tile_stride;  // >= n_tiles, multiple of 4
  uint64_t* spine_lb;    // [n_slots][n_chunks] k_spine look-back words: flag << 32 | chunk total / inclusive
                         // prefix (flag 1 / 2; zeroed per decode with tsum)
  uint32_t n_chunks;     // ceil(n_tiles / 2^kSpineChunkShift)
  uint32_t* slow_list;   // [n] lane records for the exact walker; reused by k_down_gather for the
                         // records k_list_gather decodes (the slow list is consumed by then)
  uint32_t* crc_rec;     // [n] streaming-CRC list: record
  uint64_t* crc_base;    // [n] its first flat round (ascending with the list index)
  uint64_t* crc_part;    // [n] rounds done << 32 | XOR of the slices, of a record split over waves
  uint32_t* irr;         // [n_slots] records not placed speculatively per slot (DevSchema::spec; after
                         // the scan words in their buffer, zero between decodes: k_tail_gather clears)
  uint4* dq;             // [dq_blocks][64][kDeferK] deferred bodies (nullptr: no deferral this decode)
  uint8_t* dq_cnt;       // [dq_blocks][64] entries used per row (0 for records not accepted)
  uint32_t dq_blocks;
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
  int lane_grid;           // cap: workgroups for one record per lane
  int wave_grid;
  uint32_t lane_max;       // records above this size go to the wave kernels
  uint32_t wave_stage;     // wave records spanning <= this many bytes are staged in LDS (<= kWStage)
  bool stage_count;        // the batch may hold staged records above lane_max: launch k_stage_count
  bool body_count;         // deferred packed bodies possible (DevOut::dq): launch k_body_count
};

// Kernel stages, in launch order (profiling events bracket each one).
enum Stage : int { kStageLaneCount = 0, kStageStageCount, kStageBodyCount, kStageTailCount, kStageSpine,
                   kStageDownGather, kStageTailGather, kStageMaterialize, kNumStages };
extern const char* const kStageNames[kNumStages];

// ev: optional kNumStages + 1 events recorded on `stream` before each stage and after the last.
hipError_t launch_stream_read(const void* d, uint64_t nbytes, uint32_t* sink, hipStream_t st, int variant);
hipError_t launch_decode(const DevBatch& b, const DevSchema& sc, const DevOut& o, const LaunchCfg& cfg,
                         const uint32_t* d_crc_tables, const uint32_t* d_wave_consts, hipStream_t stream,
                         hipEvent_t* ev);

}  // namespace tfrg
