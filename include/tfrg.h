/* tfrg.h — C-ABI of libtfrg, the MI355X TFRecord -> tf.train.Example -> Feature decode path.
 *
 * Plain pointers and sizes only (no torch / HIP types): the Python host mirror binds it with
 * ctypes (which releases the GIL), see INTEGRATION.md for the binding stubs. Every entry point
 * cites the reference interface (kmkolasinski/tfrecords-reader v1.1.0) whose work it replaces.
 *
 * Return convention: int functions return 0 on success and a negative TFRG_E_* code on a runtime
 * failure (HIP error, bad argument, allocation). Per-record DATA errors are never return codes:
 * they are the per-record int32 status column (include/tfrg_status.h), mirroring the exception the
 * reference would raise for that record.
 */
#ifndef TFRG_H
#define TFRG_H
#include <stdint.h>
#include "tfrg_status.h"

#ifdef __cplusplus
extern "C" {
#endif

#define TFRG_ABI_VERSION 1

/* runtime error codes (return values) */
#define TFRG_E_ARG (-1)
#define TFRG_E_HIP (-2)
#define TFRG_E_NOMEM (-3)
#define TFRG_E_IO (-4)
#define TFRG_E_LIMIT (-5)

/* decode flags */
#define TFRG_FLAG_PAYLOAD_ONLY 1u /* ranges are bare Example payloads (decode(raw) semantics)   */
#define TFRG_FLAG_SPEC_VARINT 2u  /* protobuf-spec int64 varints instead of the reference's
                                     int-width shift (decoder.pyx:44)               */
#define TFRG_FLAG_NO_CRC 4u       /* skip the CRC-32C verdicts                                   */
#define TFRG_FLAG_STRICT_CRC 8u   /* a record whose length field or either masked CRC-32C does not
                                     match fails with TFRG_ERR_CRC (no values) instead of only
                                     clearing its verdict bits; overrides TFRG_FLAG_NO_CRC      */
#define TFRG_FLAG_MATERIALIZE_BYTES 16u /* also gather every bytes_list element's payload into a
                                     contiguous device byte column (tfrg_columns.bytes_data) with
                                     u64 offsets (bytes_offsets); default: (offset, len) views  */

int tfrg_abi_version(void);
/* Per-record status (tfrg_status.h) -> the reference's exception: its Python type name ("Exception",
 * "UnicodeDecodeError", "AttributeError", "OSError", ...) and message text, literal for the
 * decoder.pyx:49-297 exceptions ("Unsupported wire type: <aux>" for TFRG_ERR_WIRE_TYPE). The
 * message pointer is thread-local storage, valid until the next call on the thread. */
const char* tfrg_status_exception(int status);
const char* tfrg_status_message(int status, int64_t aux);
/* message of the last runtime failure on this thread */
const char* tfrg_last_error(void);

/* ---------------------------------------------------------------------------------------------
 * Host framing index (replaces cython/indexer.pyx:212-252 create_tfrecord_pointers_index).
 * Pointers are (start, end, example_size) u64 triples, end = start + 16 + size; bit-exact with the
 * reference, including its acceptance of a last record that runs past EOF.
 * ------------------------------------------------------------------------------------------- */
/* over an in-memory file image; writes up to cap triples, returns the record count */
int64_t tfrg_index_buffer(const uint8_t* file, uint64_t size, uint64_t* out_triples, int64_t cap);
/* mmap + index; *out_triples is malloc'd (free with tfrg_free) */
int tfrg_index_file(const char* path, uint64_t** out_triples, int64_t* n);
/* .idx cache file, indexer.pyx:260-328: native size_t n, then n x {u64 start, end, size} */
int tfrg_idx_save(const char* idx_path, const uint64_t* triples, int64_t n);
int tfrg_idx_load(const char* idx_path, uint64_t** out_triples, int64_t* n);
void tfrg_free(void* p);
/* Host staging of a selection (reader.py:212-247 load_records): copies the n byte ranges
 * [starts[i], ends[i]) of src back to back into dst (NULL: only sizes them); returns the total. */
uint64_t tfrg_gather_ranges(const uint8_t* src, const uint64_t* starts, const uint64_t* ends, int64_t n,
                            uint8_t* dst);
/* Key discovery before a device decode (no reference counterpart: the keys and kinds that
 * decoder.pyx:130-199 would meet). Parses the Example -> Features -> map entries of the n records
 * [start[i], end[i]) of bytes (framed, or bare payloads with TFRG_FLAG_PAYLOAD_ONLY) and writes up
 * to cap distinct (key offset, key length, kind) u64 triples: absolute key offsets into bytes, kind =
 * the field number of the entry's Feature (1 bytes_list, 2 float_list, 3 int64_list). Only canonical
 * records seed (Example = features fields, each map entry = key then value, each Feature = one list
 * field); any other record is left to the device decode's schema-miss pass, which follows the
 * reference's semantics. Returns the triple count. Seeding the key table with them spares a first
 * decode the exact walker's schema-miss pass. */
int64_t tfrg_scan_keys(const uint8_t* bytes, uint64_t nbytes, const uint64_t* start, const uint64_t* end, int64_t n,
                       uint32_t flags, uint64_t* out_triples, int64_t cap);

/* Compressed TFRecord files (TensorFlow TFRecordOptions "ZLIB" / "GZIP": the whole framed stream
 * deflated; claimed by the reference's README.md:14, not implemented there). tfrg_compression_of
 * classifies a file image: an image whose length chain tiles it exactly is uncompressed, else a
 * gzip / zlib header selects that format. tfrg_inflate decodes either (concatenated gzip members
 * included) into a malloc'd buffer (free with tfrg_free); the framing index is then built over it. */
#define TFRG_COMPRESSION_NONE 0
#define TFRG_COMPRESSION_ZLIB 1
#define TFRG_COMPRESSION_GZIP 2
int tfrg_compression_of(const uint8_t* image, uint64_t size);
int tfrg_inflate(const uint8_t* in, uint64_t size, uint8_t** out, uint64_t* out_len);

/* CRC-32C (Castagnoli) and the TFRecord mask (absent from the reference) */
uint32_t tfrg_crc32c(const uint8_t* p, uint64_t n);
uint32_t tfrg_masked_crc32c(const uint8_t* p, uint64_t n);
/* TFRecord writer framing: n payloads (concatenated, offsets[n+1]) -> framed bytes with spec CRCs
 * (crc != 0) or the zero CRCs the reference's test writers use (tests/utils.py:31-36).
 * Returns the framed size; writes only if out_cap suffices. */
int64_t tfrg_frame_records(const uint8_t* payloads, const uint64_t* offsets, int64_t n, int crc,
                           uint8_t* out, int64_t out_cap);

/* ---------------------------------------------------------------------------------------------
 * Device decode (replaces cython/decoder.pyx:107 example_from_bytes per record, batched).
 * One context per (device, host thread); calls on one context are serialised by the caller.
 * ------------------------------------------------------------------------------------------- */
typedef struct tfrg_ctx tfrg_ctx;

int tfrg_ctx_create(int device, tfrg_ctx** out);
int tfrg_ctx_destroy(tfrg_ctx* ctx);
/* records larger than lane_max bytes take the wavefront-per-record kernels (default 2048) */
int tfrg_ctx_set_lane_max(tfrg_ctx* ctx, uint32_t lane_max);
/* An upper bound on (end - start) of the records of the following tfrg_decode_device calls (0 =
 * unknown, the default). With a bound <= lane_max the batch has no large records and their count
 * kernel is not launched (a few microseconds per decode); a wrong bound still decodes correctly
 * (such records take the lane kernel's slower path). tfrg_decode_host derives it per call. */
int tfrg_ctx_set_record_bound(tfrg_ctx* ctx, uint64_t max_record_bytes);
/* Value-capacity hints: the int64 / float / bytes_list values the following decodes are expected to
 * produce at most (0 = unknown, the default: the worst case one int64 per input byte, one float per
 * 4 bytes, one bytes element per 2 -- about 13 x the batch's bytes of device memory). A decode whose
 * values exceed a hint is re-run with the worst case inside tfrg_result_info before it returns (the
 * results are always complete); tfrg_ctx_device_bytes counts those re-runs. */
int tfrg_ctx_set_value_caps(tfrg_ctx* ctx, uint64_t int64_values, uint64_t float_values, uint64_t bytes_values);
/* device memory held by the context (bytes) and the decodes re-run so far: a value-capacity hint was
 * too small, or an optimistic decode left records (tfrg_result_info) */
int tfrg_ctx_device_bytes(tfrg_ctx* ctx, uint64_t* bytes, uint64_t* hint_reruns);
/* wavefront records spanning <= nbytes are staged in LDS (clamped to the kernel's 12 KiB stage;
 * 0 routes every wavefront record to the streaming kernels). A tuning/testing knob. */
int tfrg_ctx_set_wave_stage(tfrg_ctx* ctx, uint32_t nbytes);

/* Record-shape templates (no reference counterpart: a fast path under decoder.pyx:107-300). Up to
 * TFRG_TPL_MAX shapes of canonical records (payload <= TFRG_TPL_MAX_PAYLOAD bytes, at most
 * TFRG_TPL_MAX_ENTRIES feature entries) -- every byte fixed except list contents, incl. the
 * continuation bits of packed int64 lists -- are learned from up to TFRG_TPL_SAMPLE host records
 * spread over the batch, the most frequent shapes first (a shape seen once in a sample of >= 256 is
 * not kept; with payloads over 112 bytes the lane image holds at most 30, the LDS beside the CRC
 * tables). A framed record equal to a template under its mask, with matching length field and CRCs,
 * gets the template's dict without a walk (its values are still read from the record; k_tpl_lane,
 * schemas of <= TFRG_TPL_MAX_SLOTS slots, CRC verdicts on); any other record takes the canonical walk.
 * Learned automatically from the first tfrg_decode_host batch after each tfrg_set_schema; device-only
 * callers pass a host sample here. Returns the number of templates (0..TFRG_TPL_MAX). With no shape
 * kept, the slots that are one inline value in every sampled record (host decode) are still learned
 * for speculative placement (the optimistic decode of large single-value records).
 * tfrg_ctx_set_templates(ctx, 0) disables the match (env TFRG_TEMPLATES=0); the speculative
 * placement of slots that are one inline value in every learned shape stays on. */
#define TFRG_TPL_MAX 32
#define TFRG_TPL_MAX_PAYLOAD 240
#define TFRG_TPL_MAX_ENTRIES 16
#define TFRG_TPL_MAX_SLOTS 16
#define TFRG_TPL_SAMPLE 4096
int tfrg_learn_templates(tfrg_ctx* ctx, const uint8_t* h_bytes, uint64_t nbytes, const uint64_t* h_start,
                         const uint64_t* h_end, uint32_t n, uint32_t flags);
int tfrg_template_count(tfrg_ctx* ctx);
/* The learned templates in their window form (u32 words, layout in csrc/tfrg_internal.h): up to cap
 * words into out, the window size W (words) into *window_words; returns the template count. For
 * checking a template against records on the host. */
int tfrg_template_words(tfrg_ctx* ctx, uint32_t* out, uint64_t cap, uint32_t* window_words);
/* Host only (no device): the templates tfrg_learn_templates would learn for the given key table
 * (as tfrg_set_schema) from the given records, in window form into out; returns their count. */
int tfrg_learn_templates_host(uint32_t n_keys, const uint8_t* key_blob, const uint64_t* key_offsets,
                              const uint32_t* key_flags, uint32_t n_slots, const uint32_t* slot_key,
                              const uint8_t* slot_kind, const uint8_t* h_bytes, uint64_t nbytes,
                              const uint64_t* h_start, const uint64_t* h_end, uint32_t n, uint32_t flags,
                              uint32_t* out, uint64_t cap, uint32_t* window_words);
int tfrg_ctx_set_templates(tfrg_ctx* ctx, int on);

/* Per-kernel timing: with profiling on, every decode records HIP events on its stream around
 * each kernel stage; tfrg_profile_last waits for the last decode and writes up to cap stage
 * durations (ms) and names, returning the stage count. */
int tfrg_ctx_set_profiling(tfrg_ctx* ctx, int on);
int tfrg_profile_last(tfrg_ctx* ctx, float* ms, const char** names, int cap);

/* Key table ("schema"): n_keys distinct key byte strings (key_blob[key_offsets[i]..[i+1]]),
 * key_flags bit0 = the bytes are not valid UTF-8 (decoder.pyx:164 would raise); n_slots columns,
 * slot s = (slot_key[s], slot_kind[s]) with kind 1 bytes_list, 2 float_list, 3 int64_list.
 * Records whose keys are not all in the table finish with status TFRG_ST_SCHEMA_MISS and list the
 * missing (key, kind) pairs (tfrg_result_misses): intern them and decode again. */
int tfrg_set_schema(tfrg_ctx* ctx, uint32_t n_keys, const uint8_t* key_blob, const uint64_t* key_offsets,
                    const uint32_t* key_flags, uint32_t n_slots, const uint32_t* slot_key,
                    const uint8_t* slot_kind);

/* ---------------------------------------------------------------------------------------------
 * Host decode of ONE payload (replaces cython/decoder.pyx:107 example_from_bytes for single
 * records: the "cython" decoder type, and the one-record calls decode(raw) / example_from_bytes /
 * ds[i] of the "hip" type, far below the device's launch latency). The reference's exact
 * semantics (error precedence, dict rules, varint compat mode unless TFRG_FLAG_SPEC_VARINT) on the
 * calling thread; no device, no schema. One context per host thread.
 * ------------------------------------------------------------------------------------------- */
typedef struct tfrg_host_ctx tfrg_host_ctx;
typedef struct tfrg_host_record {
  int32_t status;            /* tfrg_status of the record (0 = ok), as the device's status column */
  uint32_t n_entries;        /* dict entries (status 0), in the reference's dict order */
  int64_t aux;               /* error detail, as the device's aux column */
  const uint32_t* key_off;   /* entry e's key: payload bytes [key_off[e], key_off[e] + key_len[e]) */
  const uint32_t* key_len;
  const uint8_t* kind;       /* tfrg_kind of entry e */
  const uint32_t* val_off;   /* entry e's values: [val_off[e], val_off[e] + val_cnt[e]) of its kind's array */
  const uint32_t* val_cnt;
  const int64_t* i64;
  const uint32_t* f32;       /* raw bits */
  const uint32_t* b_off;     /* bytes elements: payload-relative (offset, length) */
  const uint32_t* b_len;
} tfrg_host_record;
int tfrg_host_ctx_create(tfrg_host_ctx** out);
int tfrg_host_ctx_destroy(tfrg_host_ctx* ctx);
/* Decodes payload[0, len) into *out (arrays owned by ctx, valid until its next call). Returns 0 or a
 * TFRG_E_* code; data errors are out->status. */
int tfrg_host_decode(tfrg_host_ctx* ctx, const uint8_t* payload, uint64_t len, uint32_t flags, tfrg_host_record* out);

/* Asynchronous decode of n records [start[i], end[i]) of a device buffer (framed TFRecords unless
 * TFRG_FLAG_PAYLOAD_ONLY). d_bytes must stay readable up to round_up(nbytes, 16) and nbytes must be
 * < 2^32 (split larger batches). d_start/d_end are device arrays. stream: hipStream_t or NULL for
 * the context's own stream. Results stay valid until the next decode on this context. */
int tfrg_decode_device(tfrg_ctx* ctx, const uint8_t* d_bytes, uint64_t nbytes, const uint64_t* d_start,
                       const uint64_t* d_end, uint32_t n, uint32_t flags, void* stream);
/* Same with 32-bit offsets (a batch is < 4 GiB, so offsets relative to d_bytes fit; the index's
 * (tfrecord_start, tfrecord_end) of indexer.pyx:212-252 rebased per batch). d_start32 == NULL: the
 * records lie back to back -- record 0 starts at first_start and record i > 0 where record i - 1
 * ends, as the framing index of a file image or a gathered selection always gives them -- and
 * only their u32 ends are read (4 bytes per record instead of 16). Results are those of
 * tfrg_decode_device on the same ranges. */
int tfrg_decode_device32(tfrg_ctx* ctx, const uint8_t* d_bytes, uint64_t nbytes, const uint32_t* d_start32,
                         const uint32_t* d_end32, uint32_t first_start, uint32_t n, uint32_t flags, void* stream);
/* Same from host memory: stages bytes/start/end into context-owned HBM (H2D on the stream). */
int tfrg_decode_host(tfrg_ctx* ctx, const uint8_t* h_bytes, uint64_t nbytes, const uint64_t* h_start,
                     const uint64_t* h_end, uint32_t n, uint32_t flags, void* stream);

typedef struct tfrg_info {
  uint32_t n_records;
  uint32_t n_slots;
  uint32_t n_errors;        /* records whose status is a decode error           */
  uint32_t first_error;     /* lowest such record index, 0xffffffff if none      */
  uint32_t n_miss_records;  /* records with TFRG_ST_SCHEMA_MISS                   */
  uint32_t n_miss_entries;  /* missing (key, kind) entries reported (may exceed the list capacity) */
  uint32_t n_big;           /* records decoded by the wavefront-per-record kernels */
  uint32_t scan_timeout;    /* must be 0                                          */
  uint64_t kind_totals[4];  /* values per kind: [1] bytes elements, [2] floats, [3] int64s */
  uint64_t nbytes;
  uint64_t bytes_data_len;  /* TFRG_FLAG_MATERIALIZE_BYTES: bytes in the byte column, else 0   */
  uint32_t tpl_groups_missed; /* 64-record groups with a record no record-shape template took */
  /* TFRG_IMPLICIT_* bits: columns an optimistic decode (tfrg_result_info) did not store because every
   * record of the batch took a record shape: STATUS -- every status 0 (aux unused) and every verdict
   * TFRG_V_LEN_MATCH | TFRG_V_LEN_CRC | TFRG_V_DATA_CRC; ORDER -- every slot's order word is the
   * same for every record (its key position in the shapes); BYTES_LEN -- every bytes_list slot holds
   * one element per record whose length is the same in every shape (the bytes_len column is that
   * constant; not with TFRG_FLAG_MATERIALIZE_BYTES). tfrg_result_fetch fills them into the
   * caller's buffers on the host (no copy), tfrg_result_device into the device columns (once per
   * decode, on the decode's stream, before it returns the view). */
  uint32_t implicit_cols;
  /* bit k: slot k (< 64) holds exactly one value per record, at row r of its column (final
   * speculative placement). Its row splits are the identity 0..n: the decode does not store them;
   * tfrg_result_fetch writes them into the caller's buffer, and tfrg_result_device into the device
   * columns (one small kernel on the decode's stream, before it returns the view). */
  uint64_t placed_slots;
} tfrg_info;

/* Waits for the last decode and returns its summary. Optimistic decodes: when the context's record
 * shapes took their whole learning sample, every slot is a single value and no record can exceed
 * lane_max (tfrg_ctx_set_record_bound), a decode is launched as the template pass alone plus one
 * bookkeeping kernel; this call confirms that every record took a shape, or re-runs the same decode
 * with every pass before it returns (its inputs must still be in place: the decode is not complete
 * before this call, tfrg_result_fetch or tfrg_result_device). Env TFRG_OPTIMISTIC=0 at context
 * creation turns it off. */
int tfrg_result_info(tfrg_ctx* ctx, tfrg_info* info);

/* Columnar result. Per record: status/aux/verdict. Per slot s (row-major [n_slots][n]):
 * order (0 absent, else 1 + the key's position in the record's dict), row_splits [n_slots][n+1]
 * (element offsets inside the slot's column), slot_base [n_slots] (column start inside its kind's
 * value array). Values: int64, float bits, bytes views (absolute offset into the input buffer,
 * length). miss: [min(n_miss_entries, cap)][4] = (record, kind, key offset, key length). */
typedef struct tfrg_columns {
  int32_t* status;
  int64_t* aux;
  uint8_t* verdict;
  uint16_t* order;
  uint32_t* row_splits;
  uint64_t* slot_base;
  int64_t* i64;
  uint32_t* f32;
  uint32_t* bytes_off;
  uint32_t* bytes_len;
  uint32_t* miss;
  /* TFRG_FLAG_MATERIALIZE_BYTES only: element e of the bytes values is
   * bytes_data[bytes_offsets[e] .. bytes_offsets[e + 1]) (kind_totals[1] + 1 offsets) */
  uint8_t* bytes_data;
  uint64_t* bytes_offsets;
} tfrg_columns;

/* device pointers of the last result (valid until the next decode / destroy). Asynchronous: the
 * columns are complete once the decode's stream reaches this call (it enqueues the identity row
 * splits of the placed slots there, once per decode). After an optimistic decode (tfrg_result_info)
 * it first synchronizes the decode's stream to confirm it, re-running it in full if needed. */
int tfrg_result_device(tfrg_ctx* ctx, tfrg_columns* cols);
/* copy the last result into caller host buffers sized from tfrg_info; NULL members are skipped */
int tfrg_result_fetch(tfrg_ctx* ctx, const tfrg_columns* host);

/* ---------------------------------------------------------------------------------------------
 * Double-buffered host -> HBM decode stream (replaces reader.py:212-247's per-record ThreadPool
 * read+decode for whole-dataset reads). Two slots, each with a pinned staging buffer of batch_bytes,
 * a device input buffer and its own decode context + stream. tfrg_stream_submit hands a batch (pieces:
 * file byte ranges or host memory, whole files or record-aligned runs of them) to the slot's worker
 * thread, which reads / copies it into the slot's pinned buffer (copy_threads threads), indexes every piece with the native framing walk,
 * enqueues the H2D copies and tfrg_decode_device on the slot's stream, and returns at once; so the
 * next batch stages while this one decodes. tfrg_stream_wait blocks until the slot's batch is
 * enqueued and gives its record count (and records per piece); results are then read from
 * tfrg_stream_ctx(slot) with tfrg_result_info / _fetch / _device and stay valid until the next
 * submit to that slot. A slot is submitted again only after tfrg_stream_wait claimed its last batch
 * (else TFRG_E_ARG). The pieces' memory must stay valid until tfrg_stream_wait returns. Set the
 * key table on both contexts (tfrg_set_schema) while their slots are idle.
 * ------------------------------------------------------------------------------------------- */
typedef struct tfrg_stream tfrg_stream;
int tfrg_stream_create(int device, uint64_t batch_bytes, int copy_threads, tfrg_stream** out);
int tfrg_stream_destroy(tfrg_stream* s);
tfrg_ctx* tfrg_stream_ctx(tfrg_stream* s, int slot);
/* piece i: bytes [offsets[i], offsets[i] + sizes[i]) of file paths[i] (read with pread), or, where
 * paths is NULL or paths[i] is NULL, sizes[i] bytes of host memory at pieces[i] (e.g. the
 * decompressed stream of a ZLIB / GZIP file) */
int tfrg_stream_submit(tfrg_stream* s, int slot, const uint8_t* const* pieces, const char* const* paths,
                       const uint64_t* offsets, const uint64_t* sizes, int n_pieces, uint32_t flags);
/* stage_ms (NULL or 4 doubles): the batch's phases in ms, for the end-to-end report: file read /
 * copy into pinned memory, framing index, H2D + decode (synchronised), D2H of the columns */
int tfrg_stream_wait(tfrg_stream* s, int slot, uint64_t* n_records, uint64_t* nbytes, uint64_t* piece_records,
                     int cap, double* stage_ms);
/* the slot's decode summary and its result columns, already copied into pinned host memory by the
 * slot's worker (NULL members: aux when no record failed, bytes_off when bytes are materialised);
 * valid until the next submit to the slot. A summary with n_miss_records != 0 needs the key table
 * extended and the batch decoded again (tfrg_decode_host on the slot's context). */
int tfrg_stream_result(tfrg_stream* s, int slot, tfrg_info* info, tfrg_columns* host);
/* the slot's pinned copy of its batch (bytes_list views index into it) and its record ranges */
const uint8_t* tfrg_stream_host_buffer(tfrg_stream* s, int slot);
int tfrg_stream_host_ranges(tfrg_stream* s, int slot, const uint64_t** starts, const uint64_t** ends);

/* Measurement helper (achievable HBM read bandwidth next to the 8 TB/s spec): one
 * streaming read of d_bytes[0, nbytes) (16 B nontemporal loads, nbytes a multiple of 16) on
 * `stream`, XOR-folded into the u32 at d_sink so the loads are live. variant 0..3 picks the loads in
 * flight per lane and the grid (4/16 blocks per CU, 8/8, 8/16, 16/4). Not part of the decode path. */
int tfrg_stream_read(const void* d_bytes, uint64_t nbytes, uint32_t* d_sink, void* stream, int variant);

/* Devices visible to libtfrg (hipGetDeviceCount); the multi-device host paths spread files over them. */
int tfrg_device_count(void);

#ifdef __cplusplus
}
#endif
#endif
