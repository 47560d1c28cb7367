// tfrg_capi.cpp — device context of libtfrg: key table upload, HBM arena, decode orchestration and
// result transfer (include/tfrg.h). The kernels live in tfrg_kernels.hip.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <numeric>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/tfrg.h"
#include "crc32c.h"
#include "tfrg_internal.h"

namespace tfrg {
void set_error(const std::string& s);

#define HIP_TRY(expr)                                                              \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) {                                                        \
      set_error(std::string(#expr) + ": " + hipGetErrorString(e_));               \
      return TFRG_E_HIP;                                                           \
    }                                                                              \
  } while (0)

// grow-only device buffer
struct DBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap && p) return hipSuccess;
    if (p) {
      hipError_t e = hipFree(p);
      if (e != hipSuccess) return e;
      p = nullptr;
      cap = 0;
    }
    size_t want = bytes < 256 ? 256 : bytes;
    want = (want + 4095) & ~(size_t)4095;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const {
    return reinterpret_cast<T*>(p);
  }
};

constexpr uint32_t kMissCap = 1u << 16;

// CRC-32C byte tables, built once (thread-safe: contexts of several host threads learn templates)
const CrcTables& crc_tables() {
  static const CrcTables T = [] {
    CrcTables t;
    crc_make_tables(&t);
    return t;
  }();
  return T;
}

}  // namespace tfrg

using namespace tfrg;

// record offsets of one decode call (DevBatch: u64 pairs, u32 pairs, or u32 ends of back-to-back records)
struct Offsets {
  const uint64_t* s64 = nullptr;
  const uint64_t* e64 = nullptr;
  const uint32_t* s32 = nullptr;
  const uint32_t* e32 = nullptr;
  uint32_t first = 0;
  uint32_t mode = kOffU64;
};

struct tfrg_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t last_stream = nullptr;
  uint32_t lane_max = 2048;
  uint32_t wave_stage = 0xffffffffu;  // clamped to the kernel's stage size
  uint64_t record_bound = 0;  // tfrg_ctx_set_record_bound: no record above this (0 = unknown)
  uint64_t call_bound = 0;    // tfrg_decode_host: the bound of its own ranges (one call)
  int num_cus = 256;
  // constants
  DBuf crc_tab, consts;
  // schema
  DBuf ht, key_hash, key_off, key_blob, key_slot, slot_kind, key_w, krec;
  uint32_t n_keys = 0, n_slots = 0, ht_mask = 0;
  // host staging for tfrg_decode_host
  DBuf in_bytes, in_start, in_end;
  // arena
  DBuf status, aux, verdict, order, count, loc, rs, slot_base, totals, kind_totals;
  DBuf ident;            // 0, 1, 2, ... (ident_n words): the fetched row splits of placed slots
  size_t ident_n = 0;
  DBuf i64, f32, b_off, b_len, big_list, slow_list, miss, info, tsum, crc_rec, crc_base, crc_part;
  DBuf dq, dq_cnt;  // deferred packed-int64 bodies (k_body_count)
  DBuf lmask, rlist;  // k_tpl_lane's per-group miss masks and listed groups
  DBuf bdata, boff64, blb, bbig;  // TFRG_FLAG_MATERIALIZE_BYTES
  bool materialized = false;
  bool tsum_dirty = true;  // the scan words must be cleared before the next decode
  // info words: two slots, decode k using slot k % 2; k_lane_count zeroes the other one for the
  // next decode (no per-call memset). info_clean: the next slot is known to be zero.
  uint32_t info_slot = 0;
  bool info_clean = false;
  // last batch
  uint32_t n = 0;
  uint64_t cap_hint = 0;  // tfrg_decode_host: total bytes of the given ranges (>= nbytes when they overlap)
  hipEvent_t order_ev = nullptr;  // orders a decode on a new stream after the previous one
  uint64_t nbytes = 0;
  uint64_t cap_i64 = 0, cap_f32 = 0, cap_b = 0;
  bool have_result = false;
  bool rs_complete = false;  // the placed slots' identity rows are written into the device columns
  // record-shape templates (tfrg_learn_templates): host key table, device templates
  std::unordered_map<std::string, uint32_t> key_id;
  std::vector<int32_t> key_slot_h;  // [4 * key]: flags, slot per kind
  DBuf tpl;
  uint32_t n_tpl = 0;
  uint32_t tpl_w = 0;  // window words of the templates (16 / 32 / 64)
  size_t tpl_img_off = 0;  // the lane image follows the window-form templates in tpl
  uint32_t tpl_img_words = 0;
  std::vector<uint32_t> tpl_h;  // host copy of the template words
  bool tpl_learned = false;
  bool tpl_full = false;  // the templates took every record of their learning sample
  bool tpl_on = true;
  // speculative single-value placement (DevSchema::spec), derived from the templates
  std::vector<uint8_t> slot_kind_h;
  DBuf spec;
  std::vector<uint32_t> spec_h;  // host copy (k_tpl_lane's placement targets)
  bool have_spec = false;
  bool spec_on = true;
  // optional per-stage HIP events (tfrg_ctx_set_profiling)
  bool profiling = false;
  bool have_events = false;
  hipEvent_t ev[kNumStages + 1] = {};
  // value-capacity hints (tfrg_ctx_set_value_caps; 0: the worst case) and the last decode's
  // arguments, for the transparent worst-case re-run when a hint proved too small
  uint64_t hint_i64 = 0, hint_f32 = 0, hint_b = 0;
  bool hinted = false;  // the last decode ran with a hint below its worst case
  bool no_hints = false;  // (the re-run: the worst case)
  uint64_t hint_reruns = 0;  // decodes re-run: a hint was too small, or an optimistic decode incomplete
  // optimistic decodes (launch_all): a batch of C1-shaped records whose templates took the learning
  // sample is launched as k_tpl_lane alone (its last workgroup finishes it); the decode is complete once tfrg_result_info
  // (or tfrg_result_device) has read that no record was left, else it is re-run with every pass
  bool optimistic_on = true;  // (env TFRG_OPTIMISTIC=0: off, for A/B measurements)
  bool walk_beside = true;    // (env TFRG_WALK_BESIDE=0: large records walked before the CRC, A/B)
  uint32_t walk_blocks = 0;   // (env TFRG_WALK_BLOCKS: cap on its walking workgroups; 0 = automatic)
  bool no_quiet = false;      // (the re-run)
  bool opt_pending = false;   // the last decode ran optimistically and is not confirmed yet
  bool ord_const = false;     // (Learned::ord_const) of the learned shapes
  bool len_const = false;     // (Learned::len_const)
  std::vector<uint32_t> const_len;  // per slot: the bytes element length of every learned shape
  uint32_t last_implicit = 0; // TFRG_IMPLICIT_* columns the last decode did not store
  uint32_t* info_pin = nullptr;  // pinned host copy of the info words + kind totals (confirmation)
  bool cols_complete = false; // tfrg_result_device filled them into the device columns
  bool mat_pending = false;   // an optimistic decode's byte materialization waits for its confirmation
  struct LastCall {
    const uint8_t* d_bytes;
    uint64_t nbytes;
    uint64_t cap_in;
    uint64_t bound;
    uint32_t n, flags;
    hipStream_t st;
  } last{};
  Offsets last_off{};
  // debug hook: records whose list locations are poisoned after the count passes (tests)
  uint32_t poison[4] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
};

extern "C" {

int tfrg_ctx_create(int device, tfrg_ctx** out) {
  *out = nullptr;
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) {
    set_error("bad device index");
    return TFRG_E_ARG;
  }
  HIP_TRY(hipSetDevice(device));
  tfrg_ctx* c = new tfrg_ctx();
  c->device = device;
  if (const char* e = getenv("TFRG_TEMPLATES")) c->tpl_on = atoi(e) != 0;  // (A/B measurements)
  if (const char* e = getenv("TFRG_SPEC")) c->spec_on = atoi(e) != 0;
  if (const char* e = getenv("TFRG_OPTIMISTIC")) c->optimistic_on = atoi(e) != 0;
  if (const char* e = getenv("TFRG_WALK_BESIDE")) c->walk_beside = atoi(e) != 0;
  if (const char* e = getenv("TFRG_WALK_BLOCKS")) c->walk_blocks = (uint32_t)atoi(e);
  if (const char* e = getenv("TFRG_DEBUG_POISON_LOC")) {  // "r0,r1,..." (at most 4)
    char* q = const_cast<char*>(e);
    for (int i = 0; i < 4 && *q; ++i) {
      c->poison[i] = (uint32_t)strtoul(q, &q, 10);
      while (*q == ',' || *q == ' ') ++q;
    }
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->num_cus = prop.multiProcessorCount;
  if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    set_error("hipStreamCreate failed");
    return TFRG_E_HIP;
  }
  if (hipHostMalloc(reinterpret_cast<void**>(&c->info_pin), (kInfoCount + 8) * 4) != hipSuccess) {
    (void)hipStreamDestroy(c->own_stream);
    delete c;
    set_error("hipHostMalloc failed");
    return TFRG_E_NOMEM;
  }
  // CRC tables: [4][256] slice-by-4 + [4][256] multiply-by-x^8192 (streaming CRC), then
  // [8][256] slice-by-8 (lane kernel), then [16][256] slice-by-16 (streaming CRC), ..., then at
  // kLeanTabOff [32][256] slice-by-32 (k_tpl_lane's position tables); consts: 64 lane shifts
  // x^(128 l), 16 un-shifts x^(-8z) and 32 round shifts x^(8192 * 2^k)
  std::vector<uint32_t> tab(kLeanTabOff + 32 * 256), cst(128);
  CrcTables T;
  crc_make_tables(&T);
  memcpy(tab.data(), T.t, 4096);
  uint32_t M[4][256];
  crc_make_mul_tables(gf_xpow8(1024), M);
  memcpy(tab.data() + 1024, M, 4096);
  memcpy(tab.data() + 2048, T.t, 8192);
  memcpy(tab.data() + 4096, T.t, 16384);  // slice-by-16 (streaming CRC)
  // the slice-by-16 tables in the streaming CRC's bank-conflict-free layout (tfrg_kernels.hip
  // chunk_rot): row e of 64 dwords, column c < 47 holding table (c + 1) & 15
  for (int e = 0; e < 256; ++e)
    for (int col = 0; col < 47; ++col) tab[8192 + e * 64 + col] = T.t[(col + 1) & 15][e];
  // multiply-by-x^16384 and x^32768 tables (the streaming CRC's split Horner sum over 4 rounds)
  crc_make_mul_tables(gf_xpow8(2048), M);
  memcpy(tab.data() + 24576, M, 4096);
  crc_make_mul_tables(gf_xpow8(4096), M);
  memcpy(tab.data() + 25600, M, 4096);
  // multiply by x^(8192 * 2^k), k < 24: a slice of a record split over waves shifted to its place
  for (int k = 0; k < 24; ++k) {
    crc_make_mul_tables(gf_xpow8(1024ull << k), M);
    memcpy(tab.data() + 26624 + k * 1024, M, 4096);
  }
  for (int l = 0; l < 64; ++l) cst[l] = gf_xpow8(16ull * l);
  for (int z = 0; z < 16; ++z) cst[64 + z] = gf_xpow8_inv((uint64_t)z);
  for (int k = 0; k < 32; ++k) cst[96 + k] = gf_xpow8(1024ull << k);  // x^(8192 * 2^k): round shifts
  // T_d[v] = U(0, v followed by d zero bytes), d < 32
  for (int v = 0; v < 256; ++v) {
    uint32_t x = T.t[0][v];
    for (int d = 0; d < 32; ++d) {
      tab[kLeanTabOff + d * 256 + v] = x;
      x = (x >> 8) ^ T.t[0][x & 0xff];
    }
  }
  if (c->crc_tab.ensure(tab.size() * 4) != hipSuccess || c->consts.ensure(cst.size() * 4) != hipSuccess ||
      hipMemcpy(c->crc_tab.p, tab.data(), tab.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(c->consts.p, cst.data(), cst.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
    set_error("constant upload failed");
    tfrg_ctx_destroy(c);
    return TFRG_E_HIP;
  }
  *out = c;
  return 0;
}

int tfrg_ctx_destroy(tfrg_ctx* c) {
  if (!c) return 0;
  (void)hipSetDevice(c->device);
  if (c->last_stream) (void)hipStreamSynchronize(c->last_stream);
  DBuf* all[] = {&c->crc_tab, &c->consts, &c->ht, &c->key_hash, &c->key_off, &c->key_blob, &c->key_slot,
                 &c->slot_kind, &c->key_w, &c->krec, &c->in_bytes, &c->in_start, &c->in_end, &c->status, &c->aux, &c->verdict,
                 &c->order, &c->count, &c->loc, &c->rs, &c->ident, &c->slot_base, &c->totals, &c->kind_totals, &c->i64,
                 &c->f32, &c->b_off, &c->b_len, &c->big_list, &c->slow_list, &c->miss, &c->info, &c->tsum,
                 &c->bdata, &c->boff64, &c->blb, &c->bbig, &c->crc_rec, &c->crc_base, &c->crc_part, &c->tpl, &c->spec,
                 &c->dq, &c->dq_cnt, &c->lmask, &c->rlist};
  for (DBuf* b : all) b->release();
  if (c->order_ev) (void)hipEventDestroy(c->order_ev);
  if (c->have_events)
    for (auto& e : c->ev) (void)hipEventDestroy(e);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  if (c->info_pin) (void)hipHostFree(c->info_pin);
  delete c;
  return 0;
}

int tfrg_ctx_set_lane_max(tfrg_ctx* c, uint32_t lane_max) {
  if (!c) return TFRG_E_ARG;
  c->lane_max = lane_max;
  return 0;
}

int tfrg_ctx_set_record_bound(tfrg_ctx* c, uint64_t max_record_bytes) {
  if (!c) return TFRG_E_ARG;
  c->record_bound = max_record_bytes;
  return 0;
}

int tfrg_ctx_set_value_caps(tfrg_ctx* c, uint64_t int64_values, uint64_t float_values, uint64_t bytes_values) {
  if (!c) return TFRG_E_ARG;
  c->hint_i64 = int64_values;
  c->hint_f32 = float_values;
  c->hint_b = bytes_values;
  return 0;
}

int tfrg_ctx_device_bytes(tfrg_ctx* c, uint64_t* bytes, uint64_t* reruns) {
  if (!c) return TFRG_E_ARG;
  const DBuf* all[] = {&c->crc_tab, &c->consts, &c->ht, &c->key_hash, &c->key_off, &c->key_blob, &c->key_slot,
                       &c->slot_kind, &c->key_w, &c->krec, &c->in_bytes, &c->in_start, &c->in_end, &c->status,
                       &c->aux, &c->verdict, &c->order, &c->count, &c->loc, &c->rs, &c->ident, &c->slot_base,
                       &c->totals, &c->kind_totals, &c->i64, &c->f32, &c->b_off, &c->b_len, &c->big_list,
                       &c->slow_list, &c->miss, &c->info, &c->tsum, &c->bdata, &c->boff64, &c->blb, &c->bbig,
                       &c->crc_rec, &c->crc_base, &c->crc_part, &c->tpl, &c->spec, &c->dq, &c->dq_cnt, &c->lmask,
                       &c->rlist};
  uint64_t t = 0;
  for (const DBuf* b : all) t += b->cap;
  if (bytes) *bytes = t;
  if (reruns) *reruns = c->hint_reruns;
  return 0;
}

int tfrg_ctx_set_wave_stage(tfrg_ctx* c, uint32_t nbytes) {
  if (!c) return TFRG_E_ARG;
  c->wave_stage = nbytes;
  return 0;
}

int tfrg_ctx_set_profiling(tfrg_ctx* c, int on) {
  if (!c) return TFRG_E_ARG;
  c->profiling = on != 0;
  return 0;
}

int tfrg_profile_last(tfrg_ctx* c, float* ms, const char** names, int cap) {
  if (!c || !c->have_events || !c->have_result) return TFRG_E_ARG;
  HIP_TRY(hipEventSynchronize(c->ev[kNumStages]));
  const int k = cap < kNumStages ? cap : (int)kNumStages;
  for (int i = 0; i < k; ++i) {
    float t = 0.f;
    HIP_TRY(hipEventElapsedTime(&t, c->ev[i], c->ev[i + 1]));
    if (ms) ms[i] = t;
    if (names) names[i] = kStageNames[i];
  }
  return k;
}

static void key_words(const uint8_t* p, uint64_t n, uint32_t* w0, uint32_t* w1) {
  uint32_t a = 0, b = 0;
  for (uint64_t i = 0; i < (n < 4 ? n : 4); ++i) a |= (uint32_t)p[i] << (8 * i);
  if (n > 4)
    for (uint64_t i = 0; i < 4; ++i) b |= (uint32_t)p[n - 4 + i] << (8 * i);
  *w0 = a;
  *w1 = b;
}

int tfrg_set_schema(tfrg_ctx* c, uint32_t n_keys, const uint8_t* key_blob, const uint64_t* key_offsets,
                    const uint32_t* key_flags, uint32_t n_slots, const uint32_t* slot_key, const uint8_t* slot_kind) {
  if (!c) return TFRG_E_ARG;
  HIP_TRY(hipSetDevice(c->device));
  if (c->last_stream) HIP_TRY(hipStreamSynchronize(c->last_stream));
  // a failure below may leave buffers reallocated: no schema and no result until this succeeds
  c->have_result = false;
  c->n_keys = c->n_slots = 0;
  c->ht_mask = 0;
  uint32_t hsz = 16;
  while (hsz < 2 * n_keys + 2) hsz <<= 1;
  std::vector<uint32_t> ht(hsz, 0), hash(n_keys ? n_keys : 1), off(n_keys + 1), kw(2ull * (n_keys ? n_keys : 1));
  std::vector<int32_t> ks(4ull * (n_keys ? n_keys : 1), -1);
  const uint64_t blob_len = n_keys ? key_offsets[n_keys] : 0;
  for (uint32_t k = 0; k < n_keys; ++k) {
    if (key_offsets[k + 1] < key_offsets[k] || key_offsets[k + 1] > 0xffffffffull) {
      set_error("bad key offsets");
      return TFRG_E_ARG;
    }
    off[k] = (uint32_t)key_offsets[k];
    const uint64_t kl = key_offsets[k + 1] - key_offsets[k];
    key_words(key_blob + key_offsets[k], kl, &kw[2ull * k], &kw[2ull * k + 1]);
    hash[k] = key_hash_words((uint32_t)kl, kw[2ull * k], kw[2ull * k + 1]);
    ks[4ull * k] = (int32_t)(key_flags ? (key_flags[k] & 1u) : 0u);
    uint32_t j = hash[k] & (hsz - 1);
    while (ht[j]) j = (j + 1) & (hsz - 1);
    ht[j] = k + 1;
  }
  off[n_keys] = (uint32_t)blob_len;
  for (uint32_t s = 0; s < n_slots; ++s) {
    if (slot_key[s] >= n_keys || slot_kind[s] < 1 || slot_kind[s] > 3) {
      set_error("bad slot");
      return TFRG_E_ARG;
    }
    ks[4ull * slot_key[s] + slot_kind[s]] = (int32_t)s;
  }
  if (c->ht.ensure(hsz * 4) || c->key_hash.ensure(hash.size() * 4) || c->key_off.ensure(off.size() * 4) ||
      c->key_blob.ensure(blob_len + 16) || c->key_slot.ensure(ks.size() * 4) || c->slot_kind.ensure(n_slots + 16) ||
      c->key_w.ensure(kw.size() * 4)) {
    set_error("schema allocation failed");
    return TFRG_E_NOMEM;
  }
  HIP_TRY(hipMemcpy(c->ht.p, ht.data(), hsz * 4, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(c->key_hash.p, hash.data(), hash.size() * 4, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(c->key_off.p, off.data(), off.size() * 4, hipMemcpyHostToDevice));
  if (blob_len) HIP_TRY(hipMemcpy(c->key_blob.p, key_blob, blob_len, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(c->key_slot.p, ks.data(), ks.size() * 4, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(c->key_w.p, kw.data(), kw.size() * 4, hipMemcpyHostToDevice));
  std::vector<uint32_t> kr((size_t)kKrWords * (n_keys ? n_keys : 1), 0);
  for (uint32_t k = 0; k < n_keys; ++k) {
    uint32_t* r = &kr[(size_t)kKrWords * k];
    r[kKrHash] = hash[k];
    r[kKrLen] = (uint32_t)(key_offsets[k + 1] - key_offsets[k]);
    r[kKrW0] = kw[2ull * k];
    r[kKrW1] = kw[2ull * k + 1];
    for (int kind = 1; kind <= 3; ++kind) r[kKrSlot1 + kind - 1] = (uint32_t)ks[4ull * k + kind];
    r[kKrFlags] = (uint32_t)ks[4ull * k];
  }
  if (c->krec.ensure(kr.size() * 4)) {
    set_error("schema allocation failed");
    return TFRG_E_NOMEM;
  }
  HIP_TRY(hipMemcpy(c->krec.p, kr.data(), kr.size() * 4, hipMemcpyHostToDevice));
  if (n_slots) HIP_TRY(hipMemcpy(c->slot_kind.p, slot_kind, n_slots, hipMemcpyHostToDevice));
  c->n_keys = n_keys;
  c->n_slots = n_slots;
  c->ht_mask = hsz - 1;
  c->key_id.clear();
  for (uint32_t k = 0; k < n_keys; ++k)
    c->key_id.emplace(std::string((const char*)key_blob + key_offsets[k], key_offsets[k + 1] - key_offsets[k]), k);
  c->key_slot_h = ks;
  c->slot_kind_h.assign(slot_kind, slot_kind + n_slots);
  c->n_tpl = 0;  // slots may have moved: learn again from the next host batch
  c->tpl_learned = false;
  c->have_spec = false;
  return 0;
}

static DevSchema schema_view(const tfrg_ctx* c) {
  DevSchema s;
  s.n_keys = c->n_keys;
  s.n_slots = c->n_slots;
  s.ht_mask = c->ht_mask;
  s.ht = c->ht.as<uint32_t>();
  s.key_hash = c->key_hash.as<uint32_t>();
  s.key_off = c->key_off.as<uint32_t>();
  s.key_blob = c->key_blob.as<uint8_t>();
  s.key_slot = c->key_slot.as<int32_t>();
  s.slot_kind = c->slot_kind.as<uint8_t>();
  s.key_w = c->key_w.as<uint32_t>();
  s.krec = c->krec.as<uint32_t>();
  s.tpl = c->tpl.as<uint32_t>();
  s.tpl_img = s.tpl + c->tpl_img_off;
  s.tpl_img_words = c->tpl_img_words;
  s.n_tpl = c->tpl_on ? c->n_tpl : 0u;
  s.tpl_w = c->tpl_w;
  // speculative placement is a property of the learned shapes' schema (a slot that is one inline
  // value in every shape), not of the template match: it stays on with the templates off, where
  // k_lane_count places those values itself
  // (and without any shape: learn_single_slots)
  s.spec = c->spec_on && c->have_spec ? c->spec.as<uint32_t>() : nullptr;
  return s;
}

// ---- record-shape templates (tfrg_internal.h): learned from host records --------------------------
namespace {

// k_lane_count's hdr2 (tfrg_kernels.hip): 1-byte tag of wire type 2, 1..3-byte length, body in end
bool tpl_hdr2(const uint8_t* p, uint32_t L, uint32_t pos, uint32_t end, uint32_t& fn, uint32_t& off, uint32_t& len) {
  if (pos >= L || (p[pos] & 0x87u) != 0x02u) return false;
  fn = (p[pos] >> 3) & 0xfu;
  uint32_t q = pos + 1, l = 0;
  for (uint32_t nb = 0;; ++nb) {
    if (nb == 3 || q >= L) return false;
    const uint32_t b = p[q++];
    l |= (b & 0x7fu) << (7 * nb);
    if (!(b & 0x80u)) break;
  }
  off = q;
  len = l;
  return off <= end && l <= end - off;
}

struct Tpl {
  uint32_t L = 0;
  std::vector<uint8_t> bytes, mask;
  std::vector<uint32_t> ent;  // 4 words per entry
  std::string key() const {  // identity: length, masked bytes, mask
    std::string k((const char*)&L, 4);
    for (uint32_t i = 0; i < L; ++i) k.push_back((char)(bytes[i] & mask[i]));
    k.append((const char*)mask.data(), mask.size());
    return k;
  }
};

// The dict fast_walk (tfrg_kernels.hip) builds for this payload, as a template; false where
// fast_walk would bail (or the shape does not fit a template).
// the host key table the templates are derived against (tfrg_set_schema's, or a test's)
struct TplSchema {
  const std::unordered_map<std::string, uint32_t>& key_id;
  const std::vector<int32_t>& key_slot;  // [4 * key]: flags, slot per kind
  const std::vector<uint8_t>& slot_kind;
};

bool tpl_derive(const TplSchema* c, const uint8_t* p, uint32_t L, Tpl& t) {
  if (L < 2 || L > kTplMaxL) return false;
  t.L = L;
  t.bytes.assign(p, p + L);
  t.mask.assign(L, 0xffu);
  t.ent.clear();
  uint32_t fn, fo, fl;
  if (!tpl_hdr2(p, L, 0, L, fn, fo, fl) || fn != 1u || fo + fl != L) return false;
  std::vector<uint32_t> seen;
  uint32_t rank = 0;
  for (uint32_t q = fo; q < L;) {
    uint32_t en, eo, el, kn, ko, kl, vn, vo, vl, kind, lo, ll;
    if (!tpl_hdr2(p, L, q, L, en, eo, el) || en != 1u) return false;
    const uint32_t ee = eo + el;
    q = ee;
    if (!tpl_hdr2(p, L, eo, ee, kn, ko, kl) || kn != 1u) return false;
    if (!tpl_hdr2(p, L, ko + kl, ee, vn, vo, vl) || vn != 2u || vo + vl != ee) return false;
    if (!tpl_hdr2(p, L, vo, ee, kind, lo, ll) || lo + ll != ee || kind < 1u || kind > 3u) return false;
    if (kl > 256u) return false;
    const auto it = c->key_id.find(std::string((const char*)p + ko, kl));
    if (it == c->key_id.end()) return false;
    const uint32_t kid = it->second;
    if (c->key_slot[4ull * kid] & 1) return false;  // invalid UTF-8 key: the exact path
    const int32_t slot = c->key_slot[4ull * kid + kind];
    if (slot < 0 || std::find(seen.begin(), seen.end(), kid) != seen.end()) return false;
    seen.push_back(kid);
    uint32_t cnt = 0, nch = 0, c0o = 0, c0l = 0;
    const uint32_t le = lo + ll;
    for (uint32_t g = lo; g < le;) {
      uint32_t cf, co, cl;
      if (!tpl_hdr2(p, L, g, le, cf, co, cl) || cf != 1u) return false;
      g = co + cl;
      if (kind == TFRG_KIND_BYTES) {
        ++cnt;
        std::fill(t.mask.begin() + co, t.mask.begin() + co + cl, 0);
      } else if (kind == TFRG_KIND_FLOAT) {
        if (cl & 3u) return false;
        cnt += cl >> 2;
        std::fill(t.mask.begin() + co, t.mask.begin() + co + cl, 0);
      } else {  // packed varints: terminated, none longer than 10 bytes; their boundaries are fixed
        uint32_t run = 0;
        for (uint32_t i = co; i < co + cl; ++i) {
          t.mask[i] = 0x80u;
          if (p[i] & 0x80u) {
            if (++run >= 10u) return false;
          } else {
            run = 0;
            ++cnt;
          }
        }
        if (cl && (p[co + cl - 1] & 0x80u)) return false;
      }
      if (nch == 0) {
        c0o = co;
        c0l = cl;
      }
      ++nch;
    }
    if (rank >= 65534u || t.ent.size() / 4 >= kTplMaxEntries) return false;
    ++rank;
    uint32_t mode = 0, cw = cnt, a = lo, b = ll;
    if (cnt == 1u && nch == 1u) {
      if (kind == TFRG_KIND_BYTES) {
        mode = 3;
      } else if (kind == TFRG_KIND_FLOAT) {
        mode = 2;
      } else if (c0l <= 4u) {
        mode = 1;
      }
      if (mode) {
        cw = 1u | kCountInline;
        a = c0o;
        b = c0l;
      }
    }
    t.ent.insert(t.ent.end(), {(uint32_t)slot | (mode << 24), rank, cw, a | (b << 16)});
  }
  return !t.ent.empty();
}

// Record shapes of a host sample -> window-form templates (tfrg_internal.h) + the speculative
// placement words. Returns the template count (0: none).
struct Learned {
  std::vector<uint32_t> w, spec, img;  // window-form templates, spec words, lane image
  uint32_t W = 0;
  bool have_spec = false;
  bool full = false;  // every sampled record took a kept template
  bool ord_const = false;  // every slot (< kLeanMaxSlots) at one key position in every kept template
  // every bytes slot one element (mode 3) of one length in every kept template: an optimistic decode
  // leaves the bytes_len column implicit (TFRG_IMPLICIT_BYTES_LEN); const_len[k] that length
  bool len_const = false;
  std::vector<uint32_t> const_len;
};
uint32_t learn_shapes(const TplSchema* c, uint32_t S, const uint8_t* h_bytes, uint64_t nbytes, const uint64_t* h_start,
                      const uint64_t* h_end, uint32_t n, uint32_t flags, Learned& out) {
  std::map<std::string, std::pair<uint32_t, Tpl>> seen;  // shape -> (records, template)
  Tpl t;
  // up to 4,096 records spread over the whole batch (not its first ones: ids that grow with the
  // record index give the first records shapes the rest of a file does not have)
  const uint32_t lim = n < 4096u ? n : 4096u;
  for (uint32_t j = 0; j < lim; ++j) {
    const uint32_t i = (uint32_t)((uint64_t)j * n / lim);
    uint64_t a = h_start[i], e = h_end[i];
    if (e > nbytes || e < a) continue;
    if (!(flags & TFRG_FLAG_PAYLOAD_ONLY)) {  // framed: a length field matching the range
      if (e - a < 16) continue;
      uint64_t len = 0;
      memcpy(&len, h_bytes + a, 8);
      if (len != e - a - 16) continue;
      a += 12;
      e -= 4;
    }
    if (!tpl_derive(c, h_bytes + a, (uint32_t)(e - a > 0xffffffffull ? 0 : e - a), t)) continue;
    auto& slot = seen[t.key()];
    if (!slot.first) slot.second = t;
    ++slot.first;
  }
  std::vector<std::pair<uint32_t, const Tpl*>> order;
  // shapes seen at least twice in a large sample (a one-off shape would only cost the kernel a
  // template and could turn a speculatively placed slot irregular), the most frequent first
  const uint32_t min_count = lim >= 256u ? 2u : 1u;
  for (auto& kv : seen)
    if (kv.second.first >= min_count) order.push_back({kv.second.first, &kv.second.second});
  std::stable_sort(order.begin(), order.end(), [](const auto& x, const auto& y) { return x.first > y.first; });
  uint32_t nt = (uint32_t)std::min<size_t>(order.size(), kTplMaxLane);
  if (!nt) return 0;
  // the window the longest kept shape needs, and as many templates as fit LDS beside the CRC tables
  // at that window (the least frequent dropped first; a smaller maximum length may shrink W again)
  auto window_of = [&](uint32_t m) {
    uint32_t mx = 0;
    for (uint32_t k = 0; k < m; ++k) mx = std::max(mx, order[k].second->L);
    return mx + 16 <= 64 ? 16u : (mx + 16 <= 128 ? 32u : 64u);
  };
  while (nt > 1 && kLiTpl + (uint64_t)nt * kLiTw(window_of(nt)) > kLiMaxWords) --nt;
  uint64_t kept = 0;
  for (uint32_t k = 0; k < nt; ++k) kept += order[k].first;
  out.full = kept == lim;
  // speculative placement (DevSchema::spec): slots that are an inline single value in every kept
  // template, taken per kind in slot order up to the first slot of that kind that is not one (its
  // column base n * rank then holds whenever every record is regular)
  std::vector<uint32_t> seen_inline(S, 0), spec(S ? S : 1, 0);
  for (uint32_t k = 0; k < nt; ++k) {
    const Tpl& x = *order[k].second;
    for (size_t e = 0; e < x.ent.size(); e += 4) {
      const uint32_t slot = x.ent[e] & 0xffffffu, mode = x.ent[e] >> 24;
      if (mode && slot < S) ++seen_inline[slot];
    }
  }
  bool have_spec = false;
  uint32_t rank[4] = {0, 0, 0, 0};
  bool open[4] = {true, true, true, true};
  for (uint32_t k = 0; k < S; ++k) {
    const uint32_t kd = c->slot_kind[k] & 3u;
    if (!open[kd]) continue;
    if (seen_inline[k] == nt) {
      spec[k] = ((++rank[kd]) << 2) | kd;
      have_spec = true;
    } else {
      open[kd] = false;
    }
  }
  // window form (tfrg_internal.h): the last 4 W bytes of every kept shape's framed record
  const uint32_t W = window_of(nt);
  const CrcTables& CT = crc_tables();
  std::vector<uint32_t> w((size_t)nt * kLtWords, 0);
  for (uint32_t k = 0; k < nt; ++k) {
    const Tpl& x = *order[k].second;
    const uint32_t L = x.L;
    uint32_t* d = &w[(size_t)k * kLtWords];
    std::vector<uint8_t> Bm(4 * W, 0), Mm(4 * W, 0), Cm(4 * W, 0);
    const uint32_t off = 4 * W - (L + 16);  // window byte of the record start
    const uint64_t L64 = L;
    const uint32_t lcrc = tfrg_masked_crc32c(reinterpret_cast<const uint8_t*>(&L64), 8);
    for (int i = 0; i < 8; ++i) {
      Bm[off + i] = (uint8_t)(L64 >> (8 * i));
      Mm[off + i] = 0xffu;
    }
    for (int i = 0; i < 4; ++i) {
      Bm[off + 8 + i] = (uint8_t)(lcrc >> (8 * i));
      Mm[off + 8 + i] = 0xffu;
    }
    std::vector<uint8_t> fixed(L);
    for (uint32_t p = 0; p < L; ++p) {
      fixed[p] = x.bytes[p] & x.mask[p];
      Bm[off + 12 + p] = fixed[p];
      Mm[off + 12 + p] = x.mask[p];
      Cm[off + 12 + p] = (uint8_t)~x.mask[p];
    }
    auto word = [&](const std::vector<uint8_t>& v, uint32_t i) {
      return (uint32_t)v[4 * i] | ((uint32_t)v[4 * i + 1] << 8) | ((uint32_t)v[4 * i + 2] << 16) |
             ((uint32_t)v[4 * i + 3] << 24);
    };
    uint32_t crcw = 0, chain = W;
    for (uint32_t i = 0; i < W; ++i) {
      d[kLtWin + i] = word(Bm, i);
      d[kLtWin + W + i] = word(Mm, i);
      d[kLtWin + 2 * W + i] = word(Cm, i);
      if (!word(Cm, i)) continue;
      if (i + 9 < W) chain = std::min(chain, i);
      else crcw |= 1u << (i - (W - 9));
    }
    if (chain < W) crcw |= 1u;  // the chain's state joins word W - 9
    d[kLtL] = L;
    d[kLtNe] = (uint32_t)(x.ent.size() / 4);
    d[kLtCrcw] = crcw;
    d[kLtChain] = chain;
    d[kLtK] = ~crc_update_bytes(CT, 0xffffffffu, fixed.data(), L);  // CRC-32C with every variable bit 0
    uint32_t present = 0;
    for (size_t e = 0; e < x.ent.size(); e += 4) {
      const uint32_t slot = x.ent[e] & 0xffffffu, mode = x.ent[e] >> 24;
      const uint32_t a = x.ent[e + 3] & 0xffffu, b = x.ent[e + 3] >> 16;
      uint32_t pos = a;  // mode 0: list location
      if (mode == 1 || mode == 2) pos = off + 12 + a;                  // window byte of the value
      else if (mode == 3) pos = (uint32_t)((int64_t)a - 4 - (int64_t)L);  // element = end + pos
      const uint32_t sp = slot < S && spec[slot] ? 1u : 0u;
      uint32_t* q = d + kLtEnt + e;  // (e steps by 4 words)
      q[0] = (slot & 0xffu) | (mode << 8) | (sp << 12) | (b << 16);
      q[1] = x.ent[e + 1];
      q[2] = x.ent[e + 2];
      q[3] = pos;
      if (slot < 32) present |= 1u << slot;
      if (slot < kLeanMaxSlots) {  // the slot table (ranks < 2^16: tpl_derive caps them)
        uint32_t* z = d + kLtSlot + 3 * slot;
        z[0] = mode | (b << 8) | (x.ent[e + 1] << 16);
        z[1] = pos;
        z[2] = x.ent[e + 2];
      }
    }
    d[kLtAbsent] = ~present & (S >= kLeanMaxSlots ? 0xffffu : ((1u << S) - 1u));
  }
  // the lane image (tfrg_internal.h kLi*): per-lane template words, the length table, per-slot ranges
  const uint32_t tw = kLiTw(W);
  std::vector<uint32_t> img(kLiTpl + (size_t)nt * tw, 0);
  img[0] = nt;
  img[1] = W;
  img[2] = tw;
  img[4] = W;
  std::vector<uint8_t> lut(kTplMaxL + 1, 0xffu);
  for (uint32_t k = 0; k < nt; ++k) {
    const uint32_t* d = &w[(size_t)k * kLtWords];
    uint32_t* q = &img[kLiTpl + (size_t)k * tw];
    const uint32_t L = d[kLtL];
    q[0] = L;
    q[1] = d[kLtK];
    q[2] = 0xffu;
    for (uint32_t i = 0; i < 3 * W; ++i) q[4 + i] = d[kLtWin + (i / W) * W + i % W];
    for (uint32_t s2 = 0; s2 < kLeanMaxSlots; ++s2) {
      const uint32_t* z = d + kLtSlot + 3 * s2;
      uint32_t* y = q + 4 + 3 * W + 4 * s2;
      y[0] = z[0];
      y[1] = z[1];
      y[2] = z[2];
      const uint32_t mode = z[0] & 0xffu, rk = z[0] >> 16;
      uint32_t& sq = img[kLiSlotQ + s2];
      if (rk && (mode == 1u || mode == 2u)) {  // an inline value in window words [pos / 4, pos / 4 + 1]
        const uint32_t qw = z[1] >> 2;
        const uint32_t lo = (sq & kLiQValue) ? std::min(sq & 0xffu, qw) : qw;
        const uint32_t hi = (sq & kLiQValue) ? std::max((sq >> 8) & 0xffu, qw) : qw;
        sq = (sq & kLiQSingle) | kLiQValue | lo | (hi << 8);
      }
      if (k == 0) sq |= kLiQSingle;
      if ((z[2] & ~kCountInline) > 1u) sq &= ~kLiQSingle;
    }
    img[3] |= d[kLtCrcw];
    img[4] = std::min(img[4], d[kLtChain]);
    // the length chain: templates of one length in order of frequency
    if (lut[L] == 0xffu) {
      lut[L] = (uint8_t)k;
    } else {
      uint32_t p = lut[L];
      while (img[kLiTpl + (size_t)p * tw + 2] != 0xffu) p = img[kLiTpl + (size_t)p * tw + 2];
      img[kLiTpl + (size_t)p * tw + 2] = k;
    }
  }
  memcpy(&img[kLiLut], lut.data(), lut.size());
  // every slot present at the same key position (order word) in every kept shape: an optimistic
  // decode leaves the order column implicit (TFRG_IMPLICIT_ORDER)
  out.ord_const = S > 0 && S <= kLeanMaxSlots;
  for (uint32_t s2 = 0; out.ord_const && s2 < S; ++s2) {
    const uint32_t r0 = w[kLtSlot + 3 * s2] >> 16;
    out.ord_const = r0 != 0;
    for (uint32_t k = 1; out.ord_const && k < nt; ++k) out.ord_const = (w[(size_t)k * kLtWords + kLtSlot + 3 * s2] >> 16) == r0;
  }
  out.len_const = S > 0 && S <= kLeanMaxSlots;
  out.const_len.assign(S, 0u);
  for (uint32_t s2 = 0; out.len_const && s2 < S; ++s2) {
    if ((c->slot_kind[s2] & 3u) != TFRG_KIND_BYTES) continue;
    const uint32_t z0 = w[kLtSlot + 3 * s2];
    out.len_const = (z0 & 0xffu) == 3u && (z0 >> 16) != 0;
    for (uint32_t k = 1; out.len_const && k < nt; ++k) {
      const uint32_t zk = w[(size_t)k * kLtWords + kLtSlot + 3 * s2];
      out.len_const = (zk & 0xffu) == 3u && (zk >> 16) != 0 && ((zk >> 8) & 0xffu) == ((z0 >> 8) & 0xffu);
    }
    out.const_len[s2] = (z0 >> 8) & 0xffu;
  }
  out.w = std::move(w);
  out.spec = std::move(spec);
  out.img = std::move(img);
  out.W = W;
  out.have_spec = have_spec;
  return nt;
}

// Speculative placement without record shapes (records too large or too varied for a template,
// C2's flowers): a slot whose list is one inline value -- one bytes element, one float, one int64
// varint of <= 4 bytes (k_lane_count's inline rule) -- in every record of the sample that decodes,
// by the host decoder (the reference's semantics). Ranks per kind in slot order up to the first slot
// of that kind that is not one (as learn_shapes). Returns whether any slot was placed.
bool learn_single_slots(const TplSchema* c, uint32_t S, const uint8_t* h_bytes, uint64_t nbytes,
                        const uint64_t* h_start, const uint64_t* h_end, uint32_t n, uint32_t flags,
                        std::vector<uint32_t>& spec) {
  spec.assign(S ? S : 1, 0u);
  if (!S || !n) return false;
  tfrg_host_ctx* hc = nullptr;
  if (tfrg_host_ctx_create(&hc)) return false;
  std::vector<uint32_t> single(S, 0u);
  uint32_t m = 0;
  const uint32_t lim = n < 4096u ? n : 4096u;
  for (uint32_t j = 0; j < lim; ++j) {
    const uint32_t i = (uint32_t)((uint64_t)j * n / lim);
    uint64_t a = h_start[i], e = h_end[i];
    if (e > nbytes || e < a) continue;
    if (!(flags & TFRG_FLAG_PAYLOAD_ONLY)) {
      if (e - a < 16) continue;
      a += 12;
      e -= 4;
    }
    tfrg_host_record rec;
    if (tfrg_host_decode(hc, h_bytes + a, e - a, flags, &rec) || rec.status != TFRG_OK) continue;
    ++m;
    for (uint32_t k = 0; k < rec.n_entries; ++k) {
      const auto it = c->key_id.find(std::string((const char*)h_bytes + a + rec.key_off[k], rec.key_len[k]));
      if (it == c->key_id.end()) continue;
      const uint32_t kind = rec.kind[k];
      if (kind < 1 || kind > 3) continue;
      const int32_t slot = c->key_slot[4ull * it->second + kind];
      if (slot < 0 || (uint32_t)slot >= S || rec.val_cnt[k] != 1) continue;
      if (kind == TFRG_KIND_INT64) {
        const int64_t v = rec.i64[rec.val_off[k]];
        if (v < 0 || v >= (int64_t)1 << 28) continue;  // (more than 4 varint bytes: not inline)
      }
      ++single[slot];
    }
  }
  tfrg_host_ctx_destroy(hc);
  if (!m) return false;
  bool any = false;
  uint32_t rank[4] = {0, 0, 0, 0};
  bool open[4] = {true, true, true, true};
  for (uint32_t k = 0; k < S; ++k) {
    const uint32_t kd = c->slot_kind[k] & 3u;
    if (!open[kd]) continue;
    if (single[k] == m) {
      spec[k] = ((++rank[kd]) << 2) | kd;
      any = true;
    } else {
      open[kd] = false;
    }
  }
  return any;
}

}  // namespace

extern "C" int tfrg_learn_templates(tfrg_ctx* c, const uint8_t* h_bytes, uint64_t nbytes, const uint64_t* h_start,
                                    const uint64_t* h_end, uint32_t n, uint32_t flags) {
  if (!c || (n && (!h_bytes || !h_start || !h_end))) return TFRG_E_ARG;
  c->tpl_learned = true;
  c->n_tpl = 0;
  c->have_spec = false;
  if (!c->n_keys) return 0;
  const TplSchema sch{c->key_id, c->key_slot_h, c->slot_kind_h};
  Learned L;
  const uint32_t nt = learn_shapes(&sch, c->n_slots, h_bytes, nbytes, h_start, h_end, n, flags, L);
  if (!nt) {  // no record shape: the speculative placement of single-value slots alone
    std::vector<uint32_t> spec;
    if (!learn_single_slots(&sch, c->n_slots, h_bytes, nbytes, h_start, h_end, n, flags, spec)) return 0;
    HIP_TRY(hipSetDevice(c->device));
    if (c->last_stream) HIP_TRY(hipStreamSynchronize(c->last_stream));
    if (c->spec.ensure((size_t)c->n_slots * 4)) {
      set_error("template allocation failed");
      return TFRG_E_NOMEM;
    }
    HIP_TRY(hipMemcpy(c->spec.p, spec.data(), (size_t)c->n_slots * 4, hipMemcpyHostToDevice));
    c->spec_h = spec;
    c->have_spec = true;
    return 0;
  }
  const uint32_t S = c->n_slots;
  const std::vector<uint32_t>& w = L.w;
  const bool have_spec = L.have_spec;
  const std::vector<uint32_t>& spec = L.spec;
  const uint32_t W = L.W;
  HIP_TRY(hipSetDevice(c->device));
  if (c->last_stream) HIP_TRY(hipStreamSynchronize(c->last_stream));
  if (c->tpl.ensure((w.size() + L.img.size()) * 4) || (have_spec && c->spec.ensure((size_t)S * 4))) {
    set_error("template allocation failed");
    return TFRG_E_NOMEM;
  }
  HIP_TRY(hipMemcpy(c->tpl.p, w.data(), w.size() * 4, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(c->tpl.as<uint32_t>() + w.size(), L.img.data(), L.img.size() * 4, hipMemcpyHostToDevice));
  c->tpl_img_off = w.size();
  c->tpl_img_words = (uint32_t)L.img.size();
  if (have_spec) HIP_TRY(hipMemcpy(c->spec.p, spec.data(), (size_t)S * 4, hipMemcpyHostToDevice));
  c->n_tpl = nt;
  c->tpl_w = W;
  c->tpl_h = w;
  c->spec_h = spec;
  c->have_spec = have_spec;
  c->tpl_full = L.full;
  c->ord_const = L.ord_const;
  c->len_const = L.len_const;
  c->const_len = L.const_len;
  return (int)nt;
}

extern "C" int tfrg_learn_templates_host(uint32_t n_keys, const uint8_t* key_blob, const uint64_t* key_offsets,
                                         const uint32_t* key_flags, uint32_t n_slots, const uint32_t* slot_key,
                                         const uint8_t* slot_kind, const uint8_t* h_bytes, uint64_t nbytes,
                                         const uint64_t* h_start, const uint64_t* h_end, uint32_t n, uint32_t flags,
                                         uint32_t* out, uint64_t cap, uint32_t* window_words) {
  if (n && (!h_bytes || !h_start || !h_end)) return TFRG_E_ARG;
  std::unordered_map<std::string, uint32_t> key_id;
  std::vector<int32_t> ks(4ull * (n_keys ? n_keys : 1), -1);
  for (uint32_t k = 0; k < n_keys; ++k) {
    key_id.emplace(std::string((const char*)key_blob + key_offsets[k], key_offsets[k + 1] - key_offsets[k]), k);
    ks[4ull * k] = (int32_t)(key_flags ? (key_flags[k] & 1u) : 0u);
  }
  for (uint32_t s2 = 0; s2 < n_slots; ++s2) {
    if (slot_key[s2] >= n_keys || slot_kind[s2] < 1 || slot_kind[s2] > 3) return TFRG_E_ARG;
    ks[4ull * slot_key[s2] + slot_kind[s2]] = (int32_t)s2;
  }
  std::vector<uint8_t> sk(slot_kind, slot_kind + n_slots);
  const TplSchema sch{key_id, ks, sk};
  Learned L;
  const uint32_t nt = learn_shapes(&sch, n_slots, h_bytes, nbytes, h_start, h_end, n, flags, L);
  if (window_words) *window_words = L.W;
  if (out && nt) memcpy(out, L.w.data(), std::min<uint64_t>(L.w.size(), cap) * 4);
  return (int)nt;
}

extern "C" int tfrg_template_count(tfrg_ctx* c) { return c ? (int)c->n_tpl : TFRG_E_ARG; }

extern "C" int tfrg_template_words(tfrg_ctx* c, uint32_t* out, uint64_t cap, uint32_t* window_words) {
  if (!c) return TFRG_E_ARG;
  if (window_words) *window_words = c->tpl_w;
  const uint64_t nw = (uint64_t)c->n_tpl * kLtWords;
  if (out) memcpy(out, c->tpl_h.data(), (nw < cap ? nw : cap) * 4);
  return (int)c->n_tpl;
}

extern "C" int tfrg_ctx_set_templates(tfrg_ctx* c, int on) {
  if (!c) return TFRG_E_ARG;
  c->tpl_on = on != 0;
  return 0;
}

static int decode_device_any(tfrg_ctx* c, const uint8_t* d_bytes, uint64_t nbytes, const Offsets& off, uint32_t n,
                             uint32_t flags, void* stream);

int tfrg_decode_device(tfrg_ctx* c, const uint8_t* d_bytes, uint64_t nbytes, const uint64_t* d_start,
                       const uint64_t* d_end, uint32_t n, uint32_t flags, void* stream) {
  Offsets off;
  off.s64 = d_start;
  off.e64 = d_end;
  return decode_device_any(c, d_bytes, nbytes, off, n, flags, stream);
}

int tfrg_decode_device32(tfrg_ctx* c, const uint8_t* d_bytes, uint64_t nbytes, const uint32_t* d_start32,
                         const uint32_t* d_end32, uint32_t first_start, uint32_t n, uint32_t flags, void* stream) {
  if (n && !d_end32) return TFRG_E_ARG;
  Offsets off;
  off.s32 = d_start32;
  off.e32 = d_end32;
  off.first = first_start;
  off.mode = d_start32 ? kOffU32 : kOffEnds;
  return decode_device_any(c, d_bytes, nbytes, off, n, flags, stream);
}

// TFRG_FLAG_MATERIALIZE_BYTES: the bytes views of the decode just enqueued on `st` gathered into one
// contiguous column. Reads the decode's kind totals and b_off / b_len, so it runs only once they are
// final: after a full decode at once, after an optimistic one once finish_decode has confirmed it.
static hipError_t launch_materialize_last(tfrg_ctx* c, const uint8_t* d_bytes, uint64_t nbytes, uint64_t cap_in,
                                          uint64_t cap_b, hipStream_t st) {
  uint32_t* const info = c->info.as<uint32_t>() + c->info_slot * kInfoCount;
  DevBytes d;
  d.in = d_bytes;
  d.in_readable = (nbytes + 15) & ~15ull;
  d.b_off = c->b_off.as<uint32_t>();
  d.b_len = c->b_len.as<uint32_t>();
  d.kind_totals = c->kind_totals.as<uint64_t>();
  d.offsets = c->boff64.as<uint64_t>();
  d.offsets_cap = cap_b;
  d.data = c->bdata.as<uint8_t>();
  d.data_cap = cap_in + 16;
  d.lb = c->blb.as<uint64_t>();
  d.ticket = info + kInfoBytesTicket;
  d.big_count = info + kInfoBytesBig;
  d.big_list = c->bbig.as<uint32_t>();
  d.overflow = info + kInfoOverflow;
  return launch_materialize(d, c->num_cus, st);
}

static int decode_device_any(tfrg_ctx* c, const uint8_t* d_bytes, uint64_t nbytes, const Offsets& off, uint32_t n,
                             uint32_t flags, void* stream) {
  if (!c) return TFRG_E_ARG;
  if (nbytes >= (1ull << 32)) {
    set_error("batch larger than 4 GiB: split it");
    return TFRG_E_LIMIT;
  }
  if (c->n_keys == 0) {  // an empty table still needs valid (non-null) pointers
    uint64_t z = 0;
    int st = tfrg_set_schema(c, 0, nullptr, &z, nullptr, 0, nullptr, nullptr);
    if (st) return st;
  }
  HIP_TRY(hipSetDevice(c->device));
  c->have_result = false;  // set again once this decode is enqueued
  hipStream_t st = stream ? (hipStream_t)stream : c->own_stream;
  if (flags & TFRG_FLAG_STRICT_CRC) flags &= ~TFRG_FLAG_NO_CRC;  // strict mode needs the verdicts
  // a decode on another stream than the previous one must not overtake it (shared arena)
  if (c->last_stream && c->last_stream != st) {
    if (!c->order_ev) HIP_TRY(hipEventCreateWithFlags(&c->order_ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(c->order_ev, c->last_stream));
    HIP_TRY(hipStreamWaitEvent(st, c->order_ev, 0));
  }
  const uint32_t S = c->n_slots;
  const uint64_t nn = n ? n : 1;
  const uint64_t ngroups = (nn + 63) / 64;  // k_tpl_lane's 64-record groups
  const uint32_t n_tiles = (n + kTileRecs - 1) / kTileRecs;
  const uint32_t tile_stride = (n_tiles + 3u) & ~3u;
  const uint32_t n_chunks = (n_tiles + (1u << kSpineChunkShift) - 1u) >> kSpineChunkShift;
  // tile sums + look-back words + per-slot irregular-record counts (DevOut::irr)
  const uint64_t tsum_words = (uint64_t)S * tile_stride + 2ull * S * n_chunks + S;
  // value capacities: bounds for disjoint ranges (one int64 per byte, one float per 4, one bytes
  // element per 2); tfrg_decode_host passes the total of its ranges, which covers overlaps. A batch
  // of overlapping device ranges that exceeds them is reported by tfrg_result_info (TFRG_E_LIMIT).
  const uint64_t cap_in = c->cap_hint > nbytes ? c->cap_hint : nbytes;
  c->cap_hint = 0;
  uint64_t cap_i64 = cap_in + 16, cap_f32 = cap_in / 4 + 16, cap_b = cap_in / 2 + 16;
  // value-capacity hints (tfrg_ctx_set_value_caps) below the worst case: a decode that overflows one
  // is re-run with the worst case by tfrg_result_info (decode_rerun), before any result is read
  c->hinted = false;
  auto hint = [&](uint64_t h, uint64_t& cap) {
    if (h && h + 16 < cap) {
      cap = h + 16;
      c->hinted = true;
    }
  };
  if (!c->no_hints) {
    hint(c->hint_i64, cap_i64);
    hint(c->hint_f32, cap_f32);
    hint(c->hint_b, cap_b);
  }
  // growing an arena buffer frees the old one: wait for work that may still read it
  bool grow = c->status.cap < nn * 4 || c->aux.cap < nn * 8 || c->verdict.cap < nn ||
              c->order.cap < S * nn * 2 || c->count.cap < S * nn * 4 || c->loc.cap < S * nn * 8 ||
              c->rs.cap < S * (nn + 1) * 4 || c->i64.cap < cap_i64 * 8 || c->f32.cap < cap_f32 * 4 ||
              c->b_off.cap < cap_b * 4 || c->b_len.cap < cap_b * 4 || c->big_list.cap < nn * 4 ||
              c->slow_list.cap < nn * 4 || c->tsum.cap < tsum_words * 4 + 16 || c->crc_rec.cap < nn * 4 ||
              c->crc_base.cap < nn * 8 || c->crc_part.cap < nn * 8 || c->lmask.cap < ngroups * 8 ||
              c->rlist.cap < ngroups * 4;
  if (grow && c->last_stream) HIP_TRY(hipStreamSynchronize(c->last_stream));
  const size_t tsum_cap0 = c->tsum.cap;
  if (c->status.ensure(nn * 4) || c->aux.ensure(nn * 8) || c->verdict.ensure(nn) || c->order.ensure(S * nn * 2) ||
      c->count.ensure(S * nn * 4) || c->loc.ensure(S * nn * 8) || c->rs.ensure(S * (nn + 1) * 4) ||
      c->slot_base.ensure((S + 1) * 8) || c->totals.ensure((S + 1) * 4) || c->kind_totals.ensure(32) ||
      c->i64.ensure(cap_i64 * 8) || c->f32.ensure(cap_f32 * 4) || c->b_off.ensure(cap_b * 4) ||
      c->b_len.ensure(cap_b * 4) || c->big_list.ensure(nn * 4) || c->slow_list.ensure(nn * 4) ||
      c->miss.ensure(kMissCap * 16ull) || c->info.ensure(2 * kInfoCount * 4) ||
      c->tsum.ensure(tsum_words * 4 + 16) || c->crc_rec.ensure(nn * 4) || c->crc_base.ensure(nn * 8) ||
      c->crc_part.ensure(nn * 8) || c->lmask.ensure(ngroups * 8) || c->rlist.ensure(ngroups * 4)) {
    set_error("device allocation failed");
    return TFRG_E_NOMEM;
  }
  // per-call counters (Guideline 16: every polled word zero per call): this decode's info slot was
  // zeroed by the previous decode's k_lane_count, else (a fresh context, an empty batch or a failed
  // launch before) here
  const uint32_t islot = c->info_slot ^ 1u;
  uint32_t* const info_cur = c->info.as<uint32_t>() + islot * kInfoCount;
  if (!c->info_clean) HIP_TRY(hipMemsetAsync(info_cur, 0, kInfoCount * 4, st));
  c->info_clean = false;
  c->info_slot = islot;
  // the row-split scan words are zero between decodes (k_down_gather clears what it used): only a
  // fresh buffer, or one a failed launch may have left dirty, is cleared here
  if (c->tsum.cap != tsum_cap0 || c->tsum_dirty) {
    HIP_TRY(hipMemsetAsync(c->tsum.p, 0, c->tsum.cap, st));
    // (no stale kStatusRedo: a decode whose launches failed may have left one)
    HIP_TRY(hipMemsetAsync(c->status.p, 0, c->status.cap, st));
    c->tsum_dirty = false;
  }
  if (S && n == 0) HIP_TRY(hipMemsetAsync(c->rs.p, 0, S * 4, st));
  const bool mat = (flags & TFRG_FLAG_MATERIALIZE_BYTES) != 0;
  const uint64_t lb_words = materialize_lb_words(cap_b);
  if (mat) {
    const bool g2 = c->bdata.cap < cap_in + 16 || c->boff64.cap < (cap_b + 1) * 8 || c->blb.cap < lb_words * 8 ||
                    c->bbig.cap < cap_b * 4;
    if (g2 && c->last_stream) HIP_TRY(hipStreamSynchronize(c->last_stream));
    if (c->bdata.ensure(cap_in + 16) || c->boff64.ensure((cap_b + 1) * 8) || c->blb.ensure(lb_words * 8) ||
        c->bbig.ensure(cap_b * 4)) {
      set_error("device allocation failed (materialized bytes)");
      return TFRG_E_NOMEM;
    }
    HIP_TRY(hipMemsetAsync(c->blb.p, 0, lb_words * 8, st));
    if (!n) HIP_TRY(hipMemsetAsync(c->boff64.p, 0, 8, st));
  }
  if (!S || !n) HIP_TRY(hipMemsetAsync(c->kind_totals.p, 0, 32, st));

  DevBatch b;
  b.bytes = d_bytes;
  b.nbytes = nbytes;
  b.start = off.s64;
  b.end = off.e64;
  b.start32 = off.s32;
  b.end32 = off.e32;
  b.first = off.first;
  b.omode = off.mode;
  b.n = n;
  b.flags = flags;
  DevOut o;
  o.status = c->status.as<int32_t>();
  o.aux = c->aux.as<int64_t>();
  o.verdict = c->verdict.as<uint8_t>();
  o.order = c->order.as<uint16_t>();
  o.count = c->count.as<uint32_t>();
  o.loc = c->loc.as<uint2>();
  o.rs = c->rs.as<uint32_t>();
  o.slot_base = c->slot_base.as<uint64_t>();
  o.totals = c->totals.as<uint32_t>();
  o.kind_totals = c->kind_totals.as<uint64_t>();
  o.i64 = c->i64.as<int64_t>();
  o.f32 = c->f32.as<uint32_t>();
  o.b_off = c->b_off.as<uint32_t>();
  o.b_len = c->b_len.as<uint32_t>();
  o.cap_i64 = cap_i64;
  o.cap_f32 = cap_f32;
  o.cap_b = cap_b;
  o.big_list = c->big_list.as<uint32_t>();
  o.miss = c->miss.as<uint32_t>();
  o.miss_cap = kMissCap;
  o.info = info_cur;
  o.info_next = c->info.as<uint32_t>() + (islot ^ 1u) * kInfoCount;
  o.tsum = c->tsum.as<uint32_t>();
  o.tile_stride = tile_stride;
  o.spine_lb = reinterpret_cast<uint64_t*>(o.tsum + (size_t)S * tile_stride);  // 16-byte aligned
  o.n_chunks = n_chunks;
  o.irr = o.tsum + (size_t)S * tile_stride + 2ull * S * n_chunks;
  o.slow_list = c->slow_list.as<uint32_t>();
  o.crc_rec = c->crc_rec.as<uint32_t>();
  o.crc_base = c->crc_base.as<uint64_t>();
  o.crc_part = c->crc_part.as<uint64_t>();
  o.lmask = c->lmask.as<uint64_t>();
  o.rlist = c->rlist.as<uint32_t>();
  LaunchCfg cfg;
  cfg.num_cus = c->num_cus;
  cfg.lean = c->tpl_on && c->n_tpl;
  cfg.tpl_full = cfg.lean && c->tpl_full;
  cfg.spec_h = c->spec_h.empty() ? nullptr : c->spec_h.data();
  const uint64_t lane_blocks = (n + 255) / 256;
  const uint64_t lane_cap = (uint64_t)c->num_cus * 8;
  cfg.lane_grid = (int)(lane_blocks < 1 ? 1 : (lane_blocks < lane_cap ? lane_blocks : lane_cap));
  const uint64_t wave_cap = (uint64_t)c->num_cus * 4;
  const uint64_t wave_blocks = (n + 3) / 4;
  cfg.wave_grid = (int)(wave_blocks < 1 ? 1 : (wave_blocks < wave_cap ? wave_blocks : wave_cap));
  cfg.lane_max = c->lane_max;
  cfg.wave_stage = c->wave_stage;
  memcpy(cfg.poison, c->poison, sizeof(cfg.poison));
  // (the poison hook needs the gathers it tests)
  cfg.optimistic = c->optimistic_on && !c->no_quiet && c->poison[0] == 0xffffffffu;
  cfg.walk_beside = c->walk_beside;
  cfg.walk_blocks = c->walk_blocks;
  cfg.ran_optimistic = false;
  cfg.ran_quiet_big = false;
  cfg.ord_const = c->ord_const;
  cfg.len_const = c->len_const && !mat;  // (the byte gather reads the lengths)
  cfg.implicit = 0;
  const uint64_t bound = c->call_bound ? c->call_bound : c->record_bound;
  c->call_bound = 0;
  c->last = tfrg_ctx::LastCall{d_bytes, nbytes, cap_in, bound, n, flags, st};
  c->last_off = off;
  // deferred packed bodies when records above lane_max may be walked from HBM: one 64-row block
  // (2,048 entries of 16 bytes) per 256 KiB of input, at least 16
  o.dq = nullptr;
  o.dq_cnt = nullptr;
  o.dq_blocks = 0;
  cfg.body_count = false;
  if (n && (bound == 0 || bound > c->lane_max)) {
    uint64_t blocks = nbytes >> 18;
    blocks = blocks < 16 ? 16 : (blocks > (1u << 16) ? (1u << 16) : blocks);
    const size_t qb = (size_t)blocks * 64u * kDeferK * 16u, cb = (size_t)blocks * 64u;
    if ((c->dq.cap < qb || c->dq_cnt.cap < cb) && c->last_stream) HIP_TRY(hipStreamSynchronize(c->last_stream));
    if (c->dq.ensure(qb) || c->dq_cnt.ensure(cb)) {
      set_error("device allocation failed (deferred bodies)");
      return TFRG_E_NOMEM;
    }
    o.dq = c->dq.as<uint4>();
    o.dq_cnt = c->dq_cnt.as<uint8_t>();
    o.dq_blocks = (uint32_t)blocks;
    cfg.body_count = true;
  }
  if (n) {
    hipEvent_t* ev = nullptr;
    if (c->profiling) {
      if (!c->have_events) {
        for (auto& e : c->ev) HIP_TRY(hipEventCreate(&e));
        c->have_events = true;
      }
      ev = c->ev;
    }
    hipError_t e = launch_decode(b, schema_view(c), o, cfg, c->crc_tab.as<uint32_t>(), c->consts.as<uint32_t>(), st, ev);
    // (an optimistic decode that leaves records writes no kind totals and is re-run in full: its
    // byte views are gathered only once finish_decode has confirmed it)
    if (e == hipSuccess && mat && S && !cfg.ran_optimistic) {
      e = launch_materialize_last(c, d_bytes, nbytes, cap_in, cap_b, st);
    } else if (e == hipSuccess && mat && !S) {
      e = hipMemsetAsync(c->boff64.p, 0, 8, st);  // no slots: no elements
    }
    if (ev && e == hipSuccess) e = hipEventRecord(ev[kNumStages], st);
    if (e != hipSuccess) {
      c->tsum_dirty = true;
      set_error(std::string("kernel launch: ") + hipGetErrorString(e));
      return TFRG_E_HIP;
    }
  }
  c->info_clean = n != 0;  // (k_lane_count ran: the other slot is zero)
  c->n = n;
  c->nbytes = nbytes;
  c->cap_i64 = cap_i64;
  c->cap_f32 = cap_f32;
  c->cap_b = cap_b;
  c->last_stream = st;
  c->materialized = mat;
  c->have_result = true;
  c->rs_complete = false;
  c->opt_pending = n != 0 && cfg.ran_optimistic;
  // (an optimistic decode without shapes leaves the lane kernel's tile sums in the scan words: the
  // next decode clears them; one with shapes writes none)
  if (n != 0 && cfg.ran_quiet_big) c->tsum_dirty = true;
  c->mat_pending = c->opt_pending && mat && S;
  c->last_implicit = n != 0 ? cfg.implicit : 0u;
  c->cols_complete = false;
  return 0;
}

int tfrg_decode_host(tfrg_ctx* c, const uint8_t* h_bytes, uint64_t nbytes, const uint64_t* h_start,
                     const uint64_t* h_end, uint32_t n, uint32_t flags, void* stream) {
  if (!c) return TFRG_E_ARG;
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = stream ? (hipStream_t)stream : c->own_stream;
  const uint64_t pad = ((nbytes + 15) & ~15ull) + 16;
  if (c->last_stream) HIP_TRY(hipStreamSynchronize(c->last_stream));
  if (c->in_bytes.ensure(pad) || c->in_start.ensure((uint64_t)(n ? n : 1) * 8) ||
      c->in_end.ensure((uint64_t)(n ? n : 1) * 8)) {
    set_error("staging allocation failed");
    return TFRG_E_NOMEM;
  }
  if (nbytes) HIP_TRY(hipMemcpyAsync(c->in_bytes.p, h_bytes, nbytes, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemsetAsync(c->in_bytes.as<uint8_t>() + nbytes, 0, pad - nbytes, st));
  if (n) {
    HIP_TRY(hipMemcpyAsync(c->in_start.p, h_start, (size_t)n * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(c->in_end.p, h_end, (size_t)n * 8, hipMemcpyHostToDevice, st));
  }
  uint64_t total = 0, widest = 0;  // bytes of all ranges (clamped to the buffer): repeated ranges count again
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t a = h_start[i], b = h_end[i] < nbytes ? h_end[i] : nbytes;
    if (b > a) total += b - a;
    if (h_end[i] > a && h_end[i] - a > widest) widest = h_end[i] - a;
  }
  if (!c->tpl_learned && c->n_keys && c->tpl_on) {  // record shapes of the first host batch of a schema
    const int t = tfrg_learn_templates(c, h_bytes, nbytes, h_start, h_end, n, flags);
    if (t < 0) return t;
  }
  c->cap_hint = total;
  c->call_bound = widest ? widest : 1;
  return tfrg_decode_device(c, c->in_bytes.as<uint8_t>(), nbytes, c->in_start.as<uint64_t>(),
                            c->in_end.as<uint64_t>(), n, flags, st);
}

// The last decode's info words and kind totals (synchronizes its stream). The same decode is re-run
// -- its inputs are still the caller's: it has not been reported complete -- when it ran
// optimistically and a record took no template (kInfoResid: again with every pass), or when a
// value-capacity hint was too small for it (again with the worst-case capacities).
static int finish_decode(tfrg_ctx* c, uint32_t* h, uint64_t* kt) {
  bool widened = false;
  // (into pinned memory, allocated with the context: two DMA copies instead of staged pageable ones)
  for (;;) {
    HIP_TRY(hipMemcpyAsync(c->info_pin, c->info.as<uint32_t>() + c->info_slot * kInfoCount, kInfoCount * 4,
                           hipMemcpyDeviceToHost, c->last_stream));
    HIP_TRY(hipMemcpyAsync(c->info_pin + kInfoCount, c->kind_totals.p, 32, hipMemcpyDeviceToHost, c->last_stream));
    HIP_TRY(hipStreamSynchronize(c->last_stream));
    memcpy(h, c->info_pin, kInfoCount * 4);
    memcpy(kt, c->info_pin + kInfoCount, 32);
    const bool full = c->opt_pending && h[kInfoResid] != 0;  // (records no template took)
    const bool widen = h[kInfoOverflow] && c->hinted && !widened;
    if (!full && !widen) {
      if (!c->mat_pending) break;
      // a confirmed optimistic decode: its byte views now, then its info words again (the gather
      // reports an overflow there)
      c->mat_pending = false;
      const tfrg_ctx::LastCall& L = c->last;
      HIP_TRY(launch_materialize_last(c, L.d_bytes, L.nbytes, L.cap_in, c->cap_b, c->last_stream));
      continue;
    }
    const tfrg_ctx::LastCall L = c->last;
    c->no_quiet = true;
    c->no_hints = widen;
    c->cap_hint = L.cap_in;
    c->call_bound = L.bound;
    c->tsum_dirty = true;  // (the optimistic pass skipped the tile sums; clear every scan word)
    const int rc = decode_device_any(c, L.d_bytes, L.nbytes, c->last_off, L.n, L.flags, L.st);
    c->no_quiet = false;
    c->no_hints = false;
    if (rc) return rc;
    widened |= widen;
    ++c->hint_reruns;
  }
  c->opt_pending = false;
  c->hinted = false;  // (confirmed: the capacities held, or the worst-case re-run replaced it)
  return 0;
}

int tfrg_result_info(tfrg_ctx* c, tfrg_info* info) {
  if (!c || !c->have_result) return TFRG_E_ARG;
  HIP_TRY(hipSetDevice(c->device));
  uint32_t h[kInfoCount] = {0};
  uint64_t kt[4] = {0, 0, 0, 0};
  const int rc = finish_decode(c, h, kt);
  if (rc) return rc;
  uint64_t blen = 0;
  if (c->materialized && !h[kInfoOverflow]) {  // the byte column's length: offsets[nb]
    const uint64_t nb = c->n ? kt[TFRG_KIND_BYTES] : 0;
    HIP_TRY(hipMemcpy(&blen, c->boff64.as<uint64_t>() + nb, 8, hipMemcpyDeviceToHost));
  }
  memset(info, 0, sizeof(*info));
  info->n_records = c->n;
  info->n_slots = c->n_slots;
  info->n_errors = h[kInfoErrors];
  info->first_error = ~h[kInfoFirstError];  // (stored inverted by atomicMax; 0 = no error -> 0xffffffff)
  info->n_miss_records = h[kInfoMissRecords];
  info->n_miss_entries = h[kInfoMissEntries];
  info->n_big = h[kInfoBigRecs];
  info->scan_timeout = h[kInfoScanTimeout];
  for (int k = 0; k < 4; ++k) info->kind_totals[k] = kt[k];
  info->nbytes = c->nbytes;
  info->bytes_data_len = blen;
  info->tpl_groups_missed = h[kInfoResid];
  info->placed_slots = ((uint64_t)h[kInfoPlacedHi] << 32) | h[kInfoPlacedLo];
  info->implicit_cols = c->last_implicit;
  if (h[kInfoOverflow]) {
    set_error("value columns overflowed their capacity (overlapping ranges in a device batch): decode "
              "the ranges from host memory (tfrg_decode_host) or split the batch");
    return TFRG_E_LIMIT;
  }
  return 0;
}

// (TFRG_IMPLICIT_BYTES_LEN) per bytes slot of an optimistic decode: its first row in the bytes
// columns and its constant length. Every slot is placed, so slot k's rows are n * (its rank among
// the bytes slots), as tpl_quiet_finish sets the column bases.
static std::vector<std::pair<uint64_t, uint32_t>> implicit_len_runs(const tfrg_ctx* c) {
  std::vector<std::pair<uint64_t, uint32_t>> out;
  uint64_t base = 0;
  for (uint32_t k = 0; k < c->n_slots; ++k) {
    if ((c->slot_kind_h[k] & 3u) != TFRG_KIND_BYTES) continue;
    out.push_back({base, k < c->const_len.size() ? c->const_len[k] : 0u});
    base += c->n;
  }
  return out;
}

int tfrg_result_device(tfrg_ctx* c, tfrg_columns* d) {
  if (!c || !c->have_result) return TFRG_E_ARG;
  // an optimistic decode, or one whose value capacities were hinted below the worst case: confirmed
  // (or re-run in full / at the worst case) before the view, as tfrg_result_info does
  if (c->opt_pending || c->hinted) {
    HIP_TRY(hipSetDevice(c->device));
    uint32_t h[kInfoCount];
    uint64_t kt[4];
    const int rc = finish_decode(c, h, kt);
    if (rc) return rc;
    if (h[kInfoOverflow]) {
      set_error("value columns overflowed their capacity (overlapping ranges in a device batch): decode "
                "the ranges from host memory (tfrg_decode_host) or split the batch");
      return TFRG_E_LIMIT;
    }
  }
  if (!c->rs_complete && c->n_slots && c->n) {
    // a self-consistent view: the identity rows of the finally placed slots, which the decode does
    // not store, are written by one small kernel on the decode's stream (placed mask read on the
    // device), once per decode
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(launch_fill_placed_rows(c->rs.as<uint32_t>(), c->info.as<uint32_t>() + c->info_slot * kInfoCount,
                                    c->n_slots, c->n, c->last_stream));
  }
  c->rs_complete = true;
  if (c->last_implicit && !c->cols_complete) {  // the constant columns of an optimistic decode
    HIP_TRY(hipSetDevice(c->device));
    const size_t n = c->n;
    if (c->last_implicit & TFRG_IMPLICIT_STATUS) {
      HIP_TRY(hipMemsetAsync(c->status.p, 0, n * 4, c->last_stream));
      HIP_TRY(hipMemsetAsync(c->aux.p, 0, n * 8, c->last_stream));
      HIP_TRY(hipMemsetAsync(c->verdict.p, (int)(TFRG_V_LEN_MATCH | TFRG_V_LEN_CRC | TFRG_V_DATA_CRC), n, c->last_stream));
    }
    if (c->last_implicit & TFRG_IMPLICIT_ORDER)
      for (uint32_t k = 0; k < c->n_slots; ++k)
        HIP_TRY(hipMemsetD16Async(reinterpret_cast<hipDeviceptr_t>(c->order.as<uint16_t>() + (size_t)k * n),
                                  (unsigned short)(c->tpl_h[kLtSlot + 3 * k] >> 16), n, c->last_stream));
    if (c->last_implicit & TFRG_IMPLICIT_BYTES_LEN)
      for (const auto& [base, len] : implicit_len_runs(c))
        HIP_TRY(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(c->b_len.as<uint32_t>() + base), (int)len, n,
                                  c->last_stream));
  }
  c->cols_complete = true;
  d->status = c->status.as<int32_t>();
  d->aux = c->aux.as<int64_t>();
  d->verdict = c->verdict.as<uint8_t>();
  d->order = c->order.as<uint16_t>();
  d->row_splits = c->rs.as<uint32_t>();
  d->slot_base = c->slot_base.as<uint64_t>();
  d->i64 = c->i64.as<int64_t>();
  d->f32 = c->f32.as<uint32_t>();
  d->bytes_off = c->b_off.as<uint32_t>();
  d->bytes_len = c->b_len.as<uint32_t>();
  d->miss = c->miss.as<uint32_t>();
  d->bytes_data = c->materialized ? c->bdata.as<uint8_t>() : nullptr;
  d->bytes_offsets = c->materialized ? c->boff64.as<uint64_t>() : nullptr;
  return 0;
}

int tfrg_result_fetch(tfrg_ctx* c, const tfrg_columns* h) {
  tfrg_info info;
  int rc = tfrg_result_info(c, &info);
  if (rc) return rc;
  const hipStream_t st = c->last_stream;
  const size_t n = c->n, S = c->n_slots;
  auto cp = [&](void* dst, const void* src, size_t bytes) -> hipError_t {
    if (!dst || !bytes) return hipSuccess;
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st);
  };
  // (an optimistic decode's constant columns are written here, not copied: tfrg_info.implicit_cols)
  if (info.implicit_cols & TFRG_IMPLICIT_STATUS) {
    if (h->status) memset(h->status, 0, n * 4);
    if (h->aux) memset(h->aux, 0, n * 8);
    if (h->verdict) memset(h->verdict, TFRG_V_LEN_MATCH | TFRG_V_LEN_CRC | TFRG_V_DATA_CRC, n);
  } else {
    HIP_TRY(cp(h->status, c->status.p, n * 4));
    HIP_TRY(cp(h->aux, c->aux.p, n * 8));
    HIP_TRY(cp(h->verdict, c->verdict.p, n));
  }
  if ((info.implicit_cols & TFRG_IMPLICIT_ORDER) && h->order) {
    for (size_t k = 0; k < S; ++k) std::fill_n(h->order + k * n, n, (uint16_t)(c->tpl_h[kLtSlot + 3 * k] >> 16));
  } else {
    HIP_TRY(cp(h->order, c->order.p, S * n * 2));
  }
  // row splits: a placed slot's are the identity, never stored by the decode; they copy from a
  // device identity row (filled once per size), as fast as the stored rows and as asynchronous
  if (h->row_splits) {
    if (S && (info.placed_slots & (S >= 64 ? ~0ull : (1ull << S) - 1ull)) && c->ident_n < n + 1) {
      const size_t m = std::max<size_t>(n + 1, 2 * c->ident_n);
      std::vector<uint32_t> v(m);
      std::iota(v.begin(), v.end(), 0u);
      c->ident_n = 0;
      HIP_TRY(c->ident.ensure(m * 4));
      HIP_TRY(hipMemcpy(c->ident.p, v.data(), m * 4, hipMemcpyHostToDevice));
      c->ident_n = m;
    }
    for (size_t k = 0; k < S; ++k) {
      const bool pk = k < 64 && ((info.placed_slots >> k) & 1ull);
      HIP_TRY(cp(h->row_splits + k * (n + 1), pk ? c->ident.as<uint32_t>() : c->rs.as<uint32_t>() + k * (n + 1),
                 (n + 1) * 4));
    }
  }
  HIP_TRY(cp(h->slot_base, c->slot_base.p, S * 8));
  // (clamped to the capacities: a result that overflowed them fails in tfrg_result_info above)
  auto cl = [](uint64_t v, uint64_t cap) { return v < cap ? v : cap; };
  HIP_TRY(cp(h->i64, c->i64.p, cl(info.kind_totals[TFRG_KIND_INT64], c->cap_i64) * 8));
  HIP_TRY(cp(h->f32, c->f32.p, cl(info.kind_totals[TFRG_KIND_FLOAT], c->cap_f32) * 4));
  HIP_TRY(cp(h->bytes_off, c->b_off.p, cl(info.kind_totals[TFRG_KIND_BYTES], c->cap_b) * 4));
  if ((info.implicit_cols & TFRG_IMPLICIT_BYTES_LEN) && h->bytes_len) {
    for (const auto& [base, len] : implicit_len_runs(c)) std::fill_n(h->bytes_len + base, n, len);
  } else {
    HIP_TRY(cp(h->bytes_len, c->b_len.p, cl(info.kind_totals[TFRG_KIND_BYTES], c->cap_b) * 4));
  }
  if (c->materialized) {
    HIP_TRY(cp(h->bytes_data, c->bdata.p, info.bytes_data_len));
    HIP_TRY(cp(h->bytes_offsets, c->boff64.p, (info.kind_totals[TFRG_KIND_BYTES] + 1) * 8));
  }
  const size_t nm = info.n_miss_entries < kMissCap ? info.n_miss_entries : kMissCap;
  HIP_TRY(cp(h->miss, c->miss.p, nm * 16));
  HIP_TRY(hipStreamSynchronize(st));
  return 0;
}

}  // extern "C"

int tfrg_stream_read(const void* d_bytes, uint64_t nbytes, uint32_t* d_sink, void* stream, int variant) {
  if (!d_bytes || !d_sink || (nbytes & 15u)) return TFRG_E_ARG;
  return tfrg::launch_stream_read(d_bytes, nbytes, d_sink, static_cast<hipStream_t>(stream), variant) == hipSuccess
             ? 0 : TFRG_E_HIP;
}

int tfrg_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
