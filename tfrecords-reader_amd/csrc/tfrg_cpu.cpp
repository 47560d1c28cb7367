// tfrg_cpu.cpp — host decode of single tf.train.Example payloads (include/tfrg.h, tfrg_host_*).
//
// The "cython" decoder type of the drop-in (reference: example/feature.py:104-106 ->
// cython/decoder.pyx:107 example_from_bytes) and the one-record calls of the "hip" type
// (decode(raw), example_from_bytes, ds[i]): a single record is far below the device's launch
// latency, so it is decoded here, on the calling thread, with the same exact walk the device's exact
// walker runs (tfrg_walk.h: decoder.pyx's level-by-level error precedence, dict semantics, varint
// compat mode) over host memory. Keys are interned per call (no schema): the dict keeps the first
// position of a key and its last value (decoder.pyx:141-150); a key that is not valid UTF-8 raises
// at its map entry (decoder.pyx:164), decided by a strict UTF-8 check (CPython's decoder rejects
// overlong forms, surrogates and code points above U+10FFFF).
#include <stdint.h>
#include <string.h>

#include <new>
#include <vector>

#include "../../include/tfrg.h"
#include "tfrg_walk.h"

namespace {

// payload bytes with the reference's out-of-range behaviour (index == L is CPython's NUL terminator)
struct HostSrc {
  const uint8_t* p;
  int64_t L;
  uint64_t p0 = 0;
  bool ub = false;
  uint32_t at(int64_t i) {
    if (i >= L) {
      ub |= (i > L);
      return 0u;
    }
    return p[i];
  }
  uint32_t u32(int64_t i) { return at(i) | (at(i + 1) << 8) | (at(i + 2) << 16) | (at(i + 3) << 24); }
};

bool utf8_valid(const uint8_t* s, uint64_t n) {
  uint64_t i = 0;
  while (i < n) {
    const uint8_t c = s[i];
    if (c < 0x80u) {
      ++i;
      continue;
    }
    uint32_t len, cp;
    if (c >= 0xC2u && c <= 0xDFu) {
      len = 2;
      cp = c & 0x1Fu;
    } else if (c >= 0xE0u && c <= 0xEFu) {
      len = 3;
      cp = c & 0x0Fu;
    } else if (c >= 0xF0u && c <= 0xF4u) {
      len = 4;
      cp = c & 0x07u;
    } else {
      return false;
    }
    if (n - i < len) return false;
    for (uint32_t k = 1; k < len; ++k) {
      const uint8_t d = s[i + k];
      if ((d & 0xC0u) != 0x80u) return false;
      cp = (cp << 6) | (d & 0x3Fu);
    }
    if (len == 3 && (cp < 0x800u || (cp >= 0xD800u && cp <= 0xDFFFu))) return false;
    if (len == 4 && (cp < 0x10000u || cp > 0x10FFFFu)) return false;
    i += len;
  }
  return true;
}

struct Ent {
  uint32_t koff, klen;
  int kind;
  int kid;
  int64_t lo, ll;
};

// hash of a key's bytes (8 at a time)
uint64_t key_hash(const uint8_t* s, uint32_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ n;
  uint32_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    memcpy(&w, s + i, 8);
    h = (h ^ w) * 0xBF58476D1CE4E5B9ull;
    h ^= h >> 31;
  }
  uint64_t w = 0;
  memcpy(&w, s + i, n - i);
  h = (h ^ w) * 0x94D049BB133111EBull;
  return h ^ (h >> 29);
}

}  // namespace

struct tfrg_host_ctx {
  // interned keys of the current call: (offset, length) into the payload, validity, hash; an
  // open-addressing table over them (key id + 1, 0 = empty), so a record of K distinct keys costs
  // O(K), as the reference's dict (decoder.pyx:141-150)
  std::vector<uint32_t> kof, kln;
  std::vector<uint8_t> kok;
  std::vector<uint64_t> khash;
  std::vector<uint32_t> kslot;  // key id -> its table slot
  std::vector<int32_t> ht = std::vector<int32_t>(64, 0);
  std::vector<int32_t> pos_of;  // key id -> dict entry, -1 absent
  std::vector<Ent> ents;        // the dict, in insertion order
  const uint8_t* p = nullptr;
  // result arrays (valid until the next call)
  std::vector<uint32_t> key_off, key_len, val_off, val_cnt, f32, b_off, b_len;
  std::vector<uint8_t> kind;
  std::vector<int64_t> i64;

  // ---- the dict sink of tfrg_walk.h
  void reset() {
    for (const Ent& e : ents) pos_of[e.kid] = -1;
    ents.clear();
  }
  void clear_keys() {  // (only the used slots: a table grown by one wide record is not swept per call)
    for (uint32_t sl : kslot) ht[sl] = 0;
    kof.clear();
    kln.clear();
    kok.clear();
    khash.clear();
    kslot.clear();
  }
  void grow() {
    const size_t m = ht.size() * 2;
    ht.assign(m, 0);
    for (size_t k = 0; k < kof.size(); ++k) {
      size_t i = khash[k] & (m - 1);
      while (ht[i]) i = (i + 1) & (m - 1);
      ht[i] = (int32_t)k + 1;
      kslot[k] = (uint32_t)i;
    }
  }
  template <class S>
  int lookup(S&, int64_t off, int64_t len) {
    if (len > 0xffffffffll) return -2;
    const uint32_t o = (uint32_t)off, n = (uint32_t)len;
    const uint64_t h = key_hash(p + o, n);
    const size_t m = ht.size() - 1;
    size_t i = h & m;
    for (; ht[i]; i = (i + 1) & m) {
      const int k = ht[i] - 1;
      if (khash[k] == h && kln[k] == n && memcmp(p + kof[k], p + o, n) == 0) return kok[k] ? k : -2;
    }
    const int k = (int)kof.size();
    kof.push_back(o);
    kln.push_back(n);
    kok.push_back(utf8_valid(p + o, (uint64_t)n) ? 1 : 0);
    khash.push_back(h);
    kslot.push_back((uint32_t)i);
    ht[i] = k + 1;
    pos_of.push_back(-1);
    if (2 * kof.size() > ht.size()) grow();
    return kok[k] ? k : -2;
  }
  void note_miss(int, int64_t, int64_t) {}
  int insert(int kid, int kind_, int64_t lo, int64_t ll, uint32_t, int64_t koff, int64_t klen) {
    const int at = pos_of[kid];
    if (at >= 0) {  // last value wins, the key keeps its first position
      ents[at].kind = kind_;
      ents[at].lo = lo;
      ents[at].ll = ll;
    } else {
      pos_of[kid] = (int)ents.size();
      ents.push_back(Ent{(uint32_t)koff, (uint32_t)klen, kind_, kid, lo, ll});
    }
    return TFRG_OK;
  }

  // ---- list_values sink
  struct Vals {
    tfrg_host_ctx* c;
    void bytes(int64_t off, int64_t len) {
      c->b_off.push_back((uint32_t)off);
      c->b_len.push_back((uint32_t)len);
    }
    void f32(uint32_t bits) { c->f32.push_back(bits); }
    void i64(int64_t v) { c->i64.push_back(v); }
  };

  template <bool COMPAT>
  int run(const uint8_t* payload, uint64_t len, int64_t& aux) {
    clear_keys();
    p = payload;
    pos_of.clear();
    ents.clear();
    key_off.clear();
    key_len.clear();
    kind.clear();
    val_off.clear();
    val_cnt.clear();
    i64.clear();
    f32.clear();
    b_off.clear();
    b_len.clear();
    HostSrc s{payload, (int64_t)len};
    int st = tfrg::walk_example<COMPAT>(s, *this, aux);
    if (st != TFRG_OK) return st;
    Vals out{this};
    for (const Ent& e : ents) {
      key_off.push_back(e.koff);
      key_len.push_back(e.klen);
      kind.push_back((uint8_t)e.kind);
      const size_t before = e.kind == TFRG_KIND_INT64 ? i64.size() : e.kind == TFRG_KIND_FLOAT ? f32.size() : b_off.size();
      tfrg::list_values<COMPAT>(s, e.kind, e.lo, e.ll, out);
      const size_t after = e.kind == TFRG_KIND_INT64 ? i64.size() : e.kind == TFRG_KIND_FLOAT ? f32.size() : b_off.size();
      val_off.push_back((uint32_t)before);
      val_cnt.push_back((uint32_t)(after - before));
    }
    return TFRG_OK;
  }
};

extern "C" {

int tfrg_host_ctx_create(tfrg_host_ctx** out) {
  if (!out) return TFRG_E_ARG;
  *out = new (std::nothrow) tfrg_host_ctx();
  return *out ? 0 : TFRG_E_NOMEM;
}

int tfrg_host_ctx_destroy(tfrg_host_ctx* c) {
  delete c;
  return 0;
}

int tfrg_host_decode(tfrg_host_ctx* c, const uint8_t* payload, uint64_t len, uint32_t flags, tfrg_host_record* out) {
  if (!c || !out || (len && !payload)) return TFRG_E_ARG;
  static const uint8_t empty[1] = {0};
  int64_t aux = 0;
  int st;
  try {
    st = (flags & TFRG_FLAG_SPEC_VARINT) ? c->run<false>(len ? payload : empty, len, aux)
                                         : c->run<true>(len ? payload : empty, len, aux);
  } catch (const std::bad_alloc&) {
    return TFRG_E_NOMEM;
  }
  memset(out, 0, sizeof(*out));
  out->status = st;
  out->aux = st == TFRG_OK ? 0 : aux;
  if (st == TFRG_OK) {
    out->n_entries = (uint32_t)c->key_off.size();
    out->key_off = c->key_off.data();
    out->key_len = c->key_len.data();
    out->kind = c->kind.data();
    out->val_off = c->val_off.data();
    out->val_cnt = c->val_cnt.data();
    out->i64 = c->i64.data();
    out->f32 = c->f32.data();
    out->b_off = c->b_off.data();
    out->b_len = c->b_len.data();
  }
  return 0;
}

}  // extern "C"
