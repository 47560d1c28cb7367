// tfrg_walk.h — the reference's exact Example walk (decoder.pyx:34-300), shared by the device's exact
// walker (k_tail_count role 1, tfrg_kernels.hip) and the host decode of single records
// (tfrg_cpu.cpp, the "cython" decoder type). Generic over a byte source S (s.at(i): payload byte i
// with the reference's out-of-range behaviour, s.L, s.ub) and a dict sink (reset / lookup /
// note_miss / insert), so both sides run the same code with their own memory and dict.
#pragma once
#include <stdint.h>
#include "crc32c.h"  // (TFRG_HD)
#include "../../include/tfrg_status.h"

#define TFRG_WALK TFRG_HD inline

namespace tfrg {

// decode_varint (decoder.pyx:34-50). COMPAT reproduces the reference's int-width shift:
// term = (int32)((b & 0x7F) << (shift & 31)), sign-extended.
template <bool COMPAT, class S>
TFRG_WALK int rd_varint(S& s, int64_t& pos, int64_t& val) {
  int64_t r = 0;
  int shift = 0;
  for (;;) {
    const uint32_t b = s.at(pos);
    ++pos;
    const uint32_t g = b & 0x7fu;
    if (COMPAT) {
      r |= (int64_t)(int32_t)(g << (shift & 31));
    } else if (shift < 64) {
      r |= (int64_t)((uint64_t)g << shift);
    }
    if (!(b & 0x80u)) break;
    shift += 7;
    if (shift >= 64) return TFRG_ERR_VARINT_TOO_MANY;
  }
  if (s.ub) return TFRG_UB_READ_PAST_END;
  val = r;
  return TFRG_OK;
}

// same control flow without assembling the value (counting passes)
template <class S>
TFRG_WALK int skip_varint(S& s, int64_t& pos) {
  int shift = 0;
  for (;;) {
    const uint32_t b = s.at(pos);
    ++pos;
    if (!(b & 0x80u)) break;
    shift += 7;
    if (shift >= 64) return TFRG_ERR_VARINT_TOO_MANY;
  }
  return s.ub ? TFRG_UB_READ_PAST_END : TFRG_OK;
}

struct Fld {
  int64_t fn = 0, wt = 0, off = 0, len = 0;
};

// One iteration of decode_message (decoder.pyx:69-104).
template <bool COMPAT, class S>
TFRG_WALK int rd_field(S& s, int64_t& pos, int64_t end, Fld& f, int64_t& aux) {
  int64_t key;
  int st = rd_varint<COMPAT>(s, pos, key);
  if (st) return st;
  f.fn = key >> 3;
  f.wt = key & 7;
  if (f.wt == 1) {
    if (pos + 8 > end) return TFRG_ERR_EOB_FIXED64;
    f.off = pos;
    f.len = 8;
    pos += 8;
    return TFRG_OK;
  }
  if (f.wt == 2) {
    int64_t len;
    st = rd_varint<COMPAT>(s, pos, len);
    if (st) return st;
    if (COMPAT) {
      if (pos + len > end) return TFRG_ERR_EOB_LEN;  // |len| < 2^31 here: no overflow
      if (len < 0) return TFRG_UB_NEGATIVE_LENGTH;   // passes the check, then pos moves back
    } else {
      if (pos > end || (uint64_t)len > (uint64_t)(end - pos)) return TFRG_ERR_EOB_LEN;
    }
    f.off = pos;
    f.len = len;
    pos += len;
    return TFRG_OK;
  }
  if (f.wt == 5) {
    if (pos + 4 > end) return TFRG_ERR_EOB_FIXED32;
    f.off = pos;
    f.len = 4;
    pos += 4;
    return TFRG_OK;
  }
  aux = f.wt;
  return TFRG_ERR_WIRE_TYPE;
}

// decode_message validation pass: every tag/length of one level before any child is parsed,
// which is the reference's level-by-level error precedence.
template <bool COMPAT, class S>
TFRG_WALK int scan_msg(S& s, int64_t pos, int64_t end, int64_t& aux) {
  Fld f;
  while (pos < end) {
    const int st = rd_field<COMPAT>(s, pos, end, f, aux);
    if (st) return st;
  }
  return TFRG_OK;
}

// bytes/float/int64 list (decoder.pyx:203-300): validation + element count.
template <bool COMPAT, class S>
TFRG_WALK int list_count(S& s, int kind, int64_t o, int64_t n, int64_t& aux, uint32_t& count) {
  const int64_t end = o + n;
  int st = scan_msg<COMPAT>(s, o, end, aux);
  if (st) return st;
  uint64_t c = 0;
  int64_t pos = o;
  Fld f;
  while (pos < end) {
    rd_field<COMPAT>(s, pos, end, f, aux);  // validated above
    if (f.fn != 1) continue;
    if (kind == TFRG_KIND_BYTES) {
      if (f.wt != 2) return TFRG_ERR_WT_BYTES_LIST;
      ++c;
    } else if (kind == TFRG_KIND_FLOAT) {
      if (f.wt == 2) c += (uint64_t)(f.len >> 2);  // floor(len/4): trailing bytes dropped
      else if (f.wt == 5) ++c;
      else return TFRG_ERR_WT_FLOAT_LIST;
    } else {
      if (f.wt != 2) return TFRG_ERR_WT_INT64_LIST;
      // packed varints until p >= chunk end; the last one may run past the chunk (no bound)
      int64_t p = f.off;
      const int64_t e = f.off + f.len;
      while (p < e) {
        st = skip_varint(s, p);
        if (st) return st;
        ++c;
      }
    }
  }
  count = (uint32_t)c;
  return TFRG_OK;
}

// feature_from_bytes (decoder.pyx:169-199): kind = field number of the FIRST field.
template <bool COMPAT, class S>
TFRG_WALK int walk_feature(S& s, int64_t o, int64_t n, int64_t& aux, int& kind, int64_t& lo,
                            int64_t& ll, uint32_t& count) {
  const int64_t end = o + n;
  int64_t pos = o;
  Fld f, g0;
  int cnt = 0;
  while (pos < end) {
    const int st = rd_field<COMPAT>(s, pos, end, f, aux);
    if (st) return st;
    if (cnt == 0) g0 = f;
    ++cnt;
  }
  if (cnt == 0) return TFRG_UB_EMPTY_FEATURE;
  if (g0.fn < 1 || g0.fn > 3) return TFRG_ERR_FEATURE_FIELD;
  kind = (int)g0.fn;
  lo = g0.off;
  ll = g0.len;
  return list_count<COMPAT>(s, kind, g0.off, g0.len, aux, count);
}

// parse_map_entry (decoder.pyx:153-166): positional fields[0] = key, fields[1] = value.
template <bool COMPAT, class S, class Sink>
TFRG_WALK int walk_entry(S& s, Sink& sink, int64_t o, int64_t n, int64_t& aux) {
  const int64_t end = o + n;
  int64_t pos = o;
  Fld f, f0, f1;
  int cnt = 0;
  while (pos < end) {
    const int st = rd_field<COMPAT>(s, pos, end, f, aux);
    if (st) return st;
    if (cnt == 0) f0 = f;
    else if (cnt == 1) f1 = f;
    ++cnt;
  }
  if (cnt < 2) return TFRG_UB_SHORT_MAP_ENTRY;
  const int kid = sink.lookup(s, f0.off, f0.len);
  // An unknown key may be invalid UTF-8, which would raise before the feature is parsed: report
  // it now (kind 0 = key only) so the next round can rank this record's errors correctly.
  if (kid == -1) sink.note_miss(0, f0.off, f0.len);
  if (kid == -2) {  // interned as invalid UTF-8: bytes(key).decode('utf-8') raises here
    aux = (int64_t)(((uint64_t)f0.off << 32) | (uint64_t)(uint32_t)f0.len);
    return TFRG_ERR_KEY_UTF8;
  }
  int kind = 0;
  int64_t lo = 0, ll = 0;
  uint32_t count = 0;
  const int st = walk_feature<COMPAT>(s, f1.off, f1.len, aux, kind, lo, ll, count);
  if (st) return st;
  return sink.insert(kid, kind, lo, ll, count, f0.off, f0.len);
}

// features_from_bytes (decoder.pyx:130-150)
template <bool COMPAT, class S, class Sink>
TFRG_WALK int walk_features(S& s, Sink& sink, int64_t o, int64_t n, int64_t& aux) {
  const int64_t end = o + n;
  int st = scan_msg<COMPAT>(s, o, end, aux);
  if (st) return st;
  sink.reset();  // a repeated Features field replaces the dict, never merges (decoder.pyx:121)
  int64_t pos = o;
  Fld f;
  while (pos < end) {
    rd_field<COMPAT>(s, pos, end, f, aux);
    if (f.fn != 1) continue;
    if (f.wt != 2) return TFRG_ERR_WT_FEATURE;
    st = walk_entry<COMPAT>(s, sink, f.off, f.len, aux);
    if (st) return st;
  }
  return TFRG_OK;
}

// example_from_bytes (decoder.pyx:107-127) + Feature(proto.features.feature) (feature.py:106)
template <bool COMPAT, class S, class Sink>
TFRG_WALK int walk_example(S& s, Sink& sink, int64_t& aux) {
  const int64_t L = s.L;
  int st = scan_msg<COMPAT>(s, 0, L, aux);
  if (st) return st;
  bool have = false;
  int64_t pos = 0;
  Fld f;
  while (pos < L) {
    rd_field<COMPAT>(s, pos, L, f, aux);
    if (f.fn != 1) continue;
    if (f.wt != 2) return TFRG_ERR_WT_FEATURES;
    st = walk_features<COMPAT>(s, sink, f.off, f.len, aux);
    if (st) return st;
    have = true;
  }
  return have ? TFRG_OK : TFRG_ERR_FEATURES_NONE;
}

// The values of a validated list message (decoder.pyx:203-300), in wire order: out.bytes(offset,
// length) per bytes element (payload-relative), out.f32(bits) per float (packed chunks floor(len/4),
// fixed32 fields one), out.i64(value) per packed varint.
template <bool COMPAT, class S, class V>
TFRG_WALK void list_values(S& s, int kind, int64_t lo, int64_t ll, V& out) {
  const int64_t end = lo + ll;
  int64_t pos = lo, aux = 0;
  Fld f;
  while (pos < end) {
    rd_field<COMPAT>(s, pos, end, f, aux);
    if (f.fn != 1) continue;
    if (kind == TFRG_KIND_BYTES) {
      out.bytes(f.off, f.len);
    } else if (kind == TFRG_KIND_FLOAT) {
      const int64_t m = f.wt == 2 ? (f.len >> 2) : 1;
      for (int64_t i = 0; i < m; ++i) out.f32(s.u32(f.off + 4 * i));
    } else {
      int64_t p = f.off;
      const int64_t e = f.off + f.len;
      while (p < e) {
        int64_t val = 0;
        rd_varint<COMPAT>(s, p, val);
        out.i64(val);
      }
    }
  }
}

}  // namespace tfrg
