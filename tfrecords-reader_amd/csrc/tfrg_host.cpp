// tfrg_host.cpp — host-side native pieces of libtfrg: the TFRecord framing index over an mmap'd
// file image (replaces cython/indexer.pyx:212-252, bit-exact), the .idx cache format
// (indexer.pyx:255-328), CRC-32C and the TFRecord writer framing.
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <string>
#include <unordered_set>
#include <vector>

#include <zlib.h>

#include "../../include/tfrg.h"
#include "crc32c.h"

namespace tfrg {
thread_local std::string g_last_error;
void set_error(const std::string& s) { g_last_error = s; }

// slice-by-8 host tables, built once
struct HostCrc {
  uint32_t t[8][256];
  HostCrc() {
    CrcTables T;
    crc_make_tables(&T);
    for (int v = 0; v < 256; ++v) t[0][v] = T.t[0][v];
    for (int v = 0; v < 256; ++v) {
      uint32_t c = t[0][v];
      for (int j = 1; j < 8; ++j) {
        c = (c >> 8) ^ t[0][c & 0xff];
        t[j][v] = c;
      }
    }
  }
  uint32_t update(uint32_t c, const uint8_t* p, uint64_t n) const {
    while (n && ((uintptr_t)p & 7)) {
      c = t[0][(c ^ *p++) & 0xff] ^ (c >> 8);
      --n;
    }
    while (n >= 8) {
      uint64_t w;
      memcpy(&w, p, 8);
      w ^= c;
      c = t[7][w & 0xff] ^ t[6][(w >> 8) & 0xff] ^ t[5][(w >> 16) & 0xff] ^ t[4][(w >> 24) & 0xff] ^
          t[3][(w >> 32) & 0xff] ^ t[2][(w >> 40) & 0xff] ^ t[1][(w >> 48) & 0xff] ^ t[0][w >> 56];
      p += 8;
      n -= 8;
    }
    while (n--) c = t[0][(c ^ *p++) & 0xff] ^ (c >> 8);
    return c;
  }
};
static const HostCrc& host_crc() {
  static const HostCrc h;
  return h;
}
}  // namespace tfrg

using namespace tfrg;

extern "C" {

int tfrg_abi_version(void) { return TFRG_ABI_VERSION; }
const char* tfrg_last_error(void) { return g_last_error.c_str(); }
void tfrg_free(void* p) { free(p); }

// Per-record status -> the exception the reference raises (decoder.pyx:49-297, feature.py:106,
// reader.py:48-49), for C / Cython callers that do not go through tfr_reader/_status.py.
const char* tfrg_status_exception(int status) {
  switch (status) {
    case TFRG_OK: return "";
    case TFRG_ERR_KEY_UTF8: return "UnicodeDecodeError";  // bytes(key).decode('utf-8'), decoder.pyx:164
    case TFRG_ERR_FEATURES_NONE: return "AttributeError";  // Example(features=None).feature, feature.py:106
    case TFRG_ERR_READ: return "OSError";                 // reader.py:48-49
    case TFRG_ERR_CRC: return "DataLossError";             // TFRG_FLAG_STRICT_CRC (OSError subclass)
    case TFRG_UB_EMPTY_FEATURE: case TFRG_UB_SHORT_MAP_ENTRY: case TFRG_UB_NEGATIVE_LENGTH:
    case TFRG_UB_READ_PAST_END: return "UndefinedRecordError";
    case TFRG_ST_SCHEMA_MISS: case TFRG_ST_LIMIT: case TFRG_ST_INTERNAL: return "RuntimeError";
    default: return status >= TFRG_ERR_VARINT_TOO_MANY && status <= TFRG_ERR_WT_INT64_LIST ? "Exception"
                                                                                             : "RuntimeError";
  }
}

const char* tfrg_status_message(int status, int64_t aux) {
  static thread_local char buf[256];
  const char* m = nullptr;
  switch (status) {
    case TFRG_OK: m = ""; break;
    case TFRG_ERR_VARINT_TOO_MANY: m = "Too many bytes when decoding varint."; break;                   // :49
    case TFRG_ERR_EOB_FIXED64: m = "Unexpected end of buffer when reading fixed64."; break;              // :79
    case TFRG_ERR_EOB_LEN: m = "Unexpected end of buffer when reading length-delimited field."; break;  // :89
    case TFRG_ERR_EOB_FIXED32: m = "Unexpected end of buffer when reading fixed32."; break;              // :98
    case TFRG_ERR_WIRE_TYPE:                                                                            // :104
      snprintf(buf, sizeof(buf), "Unsupported wire type: %lld", (long long)aux);
      return buf;
    case TFRG_ERR_WT_FEATURES: m = "Unexpected wire type for field features"; break;  // :123
    case TFRG_ERR_WT_FEATURE: m = "Unexpected wire type for field feature"; break;    // :147
    case TFRG_ERR_FEATURE_FIELD: m = "Unexpected field number in Feature"; break;     // :199
    case TFRG_ERR_WT_BYTES_LIST: m = "Unexpected wire type in BytesList"; break;      // :220
    case TFRG_ERR_WT_FLOAT_LIST: m = "Unexpected wire type in FloatList"; break;      // :264
    case TFRG_ERR_WT_INT64_LIST: m = "Unexpected wire type in Int64List"; break;      // :297
    case TFRG_ERR_KEY_UTF8:
      snprintf(buf, sizeof(buf), "'utf-8' codec can't decode the key at payload offset %llu (length %llu)",
               (unsigned long long)((uint64_t)aux >> 32), (unsigned long long)((uint64_t)aux & 0xffffffffu));
      return buf;
    case TFRG_ERR_FEATURES_NONE: m = "'NoneType' object has no attribute 'feature'"; break;
    case TFRG_ERR_READ: m = "Failed to read data for the record byte range!"; break;
    case TFRG_ERR_CRC:
      snprintf(buf, sizeof(buf),
               "corrupted record: length field / masked CRC-32C mismatch (verdict bits 0x%llx)",
               (unsigned long long)aux);
      return buf;
    case TFRG_UB_EMPTY_FEATURE:
      m = "Feature has no kind field (the reference reads fields[0] of an empty vector and crashes: "
          "decoder.pyx:177)";
      break;
    case TFRG_UB_SHORT_MAP_ENTRY:
      m = "map entry has fewer than two fields (the reference reads fields[1] out of range and crashes: "
          "decoder.pyx:163-165)";
      break;
    case TFRG_UB_NEGATIVE_LENGTH:
      m = "negative length-delimited size (undefined in the reference: decoder.pyx:85-92 moves the cursor "
          "backwards)";
      break;
    case TFRG_UB_READ_PAST_END:
      m = "varint runs past the end of the record (undefined in the reference: decoder.pyx:34-50 has no bound)";
      break;
    case TFRG_ST_LIMIT: m = "record exceeds a decoder limit (more than 65534 keys)"; break;
    case TFRG_ST_INTERNAL:
      snprintf(buf, sizeof(buf), "internal decoder error: list location of slot %lld outside its record",
               (long long)aux);
      return buf;
    default:
      snprintf(buf, sizeof(buf), "unexpected decoder status %d", status);
      return buf;
  }
  return m;
}

uint32_t tfrg_crc32c(const uint8_t* p, uint64_t n) { return ~host_crc().update(0xffffffffu, p, n); }
uint32_t tfrg_masked_crc32c(const uint8_t* p, uint64_t n) { return crc_mask(tfrg_crc32c(p, n)); }

// The reference loop, with stdio semantics made explicit:
//   start = ftell; fread(8) != 8 -> stop; fseek(+4) (past EOF is allowed);
//   push (start, start + 16 + len, len); fseek(+(long)(len + 4)) fails -> stop.
// A last record whose payload runs past EOF is therefore indexed (verified in the survey).
extern "C++" {
template <class Put>
static inline int64_t index_walk(const uint8_t* file, uint64_t size, int64_t cap, Put put) {
  int64_t n = 0, pos = 0;
  for (;;) {
    if ((uint64_t)pos + 8 > size) break;
    const uint64_t start = (uint64_t)pos;
    uint64_t length;
    memcpy(&length, file + pos, 8);
    pos += 12;
    if (n < cap) put(n, start, length);
    ++n;
    const int64_t off = (int64_t)(length + 4);  // fseek's long offset
    int64_t np;
    if (__builtin_add_overflow(pos, off, &np) || np < 0) break;
    pos = np;
  }
  return n;
}
}  // extern "C++"

int64_t tfrg_index_buffer(const uint8_t* file, uint64_t size, uint64_t* out, int64_t cap) {
  return index_walk(file, size, cap, [out](int64_t n, uint64_t start, uint64_t length) {
    out[3 * n] = start;
    out[3 * n + 1] = start + 16 + length;  // u64 arithmetic, as the reference
    out[3 * n + 2] = length;
  });
}

// The same walk writing the (start, end) columns of a batch directly, shifted by the piece's offset
// in the batch (the stream's staging index; internal, not part of the C-ABI).
int64_t tfrg_index_split(const uint8_t* file, uint64_t size, uint64_t base, uint64_t* starts, uint64_t* ends,
                         int64_t cap) {
  return index_walk(file, size, cap, [=](int64_t n, uint64_t start, uint64_t length) {
    starts[n] = start + base;
    ends[n] = start + 16 + length + base;
  });
}

int tfrg_index_file(const char* path, uint64_t** out_triples, int64_t* n) {
  *out_triples = nullptr;
  *n = 0;
  const int fd = open(path, O_RDONLY);
  if (fd < 0) {
    set_error(std::string("Cannot open file: ") + path);
    return TFRG_E_IO;
  }
  struct stat sb;
  if (fstat(fd, &sb) != 0) {
    close(fd);
    set_error("fstat failed");
    return TFRG_E_IO;
  }
  const uint64_t size = (uint64_t)sb.st_size;
  const uint8_t* img = nullptr;
  if (size) {
    void* m = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) {
      close(fd);
      set_error("mmap failed");
      return TFRG_E_IO;
    }
    madvise(m, size, MADV_SEQUENTIAL);
    img = (const uint8_t*)m;
  }
  close(fd);
  // count first (cheap: touches 8 bytes per record), then fill
  const int64_t cnt = tfrg_index_buffer(img, size, nullptr, 0);
  uint64_t* out = (uint64_t*)malloc(sizeof(uint64_t) * 3 * (size_t)(cnt > 0 ? cnt : 1));
  if (!out) {
    if (img) munmap((void*)img, size);
    set_error("out of memory");
    return TFRG_E_NOMEM;
  }
  tfrg_index_buffer(img, size, out, cnt);
  if (img) munmap((void*)img, size);
  *out_triples = out;
  *n = cnt;
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Compressed TFRecord files: TensorFlow's TFRecordOptions compression "ZLIB" / "GZIP" deflates the
// whole framed record stream (the reference's README.md:14 claims support; its code has none).
// ---------------------------------------------------------------------------------------------
static bool framing_exact(const uint8_t* img, uint64_t size) {
  uint64_t pos = 0;
  while (pos + 8 <= size) {
    uint64_t len;
    memcpy(&len, img + pos, 8);
    if (len > size || pos + 16 + len > size) return false;
    pos += 16 + len;
  }
  return pos == size;
}

int tfrg_compression_of(const uint8_t* img, uint64_t size) {
  int kind = TFRG_COMPRESSION_NONE;
  if (size >= 2 && img[0] == 0x1f && img[1] == 0x8b) kind = TFRG_COMPRESSION_GZIP;
  else if (size >= 2 && (img[0] & 0x0f) == 8 && (img[0] >> 4) <= 7 && (((uint32_t)img[0] << 8) | img[1]) % 31 == 0)
    kind = TFRG_COMPRESSION_ZLIB;
  // a header that looks compressed may still be the start of a plain image (a first record of
  // length 0x..9c78 begins 78 9c): a length chain that tiles the file exactly, or a first length
  // field whose masked CRC-32C (bytes 8..12) matches, means uncompressed (a deflate stream passing
  // that check by chance has odds of 2^-32)
  if (kind != TFRG_COMPRESSION_NONE) {
    if (size >= 12) {
      uint64_t len;
      uint32_t stored;
      memcpy(&len, img, 8);
      memcpy(&stored, img + 8, 4);
      if (len <= size && stored == tfrg_masked_crc32c(img, 8)) return TFRG_COMPRESSION_NONE;
    }
    if (framing_exact(img, size)) kind = TFRG_COMPRESSION_NONE;
  }
  return kind;
}

int tfrg_inflate(const uint8_t* in, uint64_t size, uint8_t** out, uint64_t* out_len) {
  *out = nullptr;
  *out_len = 0;
  z_stream zs;
  memset(&zs, 0, sizeof(zs));
  if (inflateInit2(&zs, 15 + 32) != Z_OK) {  // 15 + 32: zlib or gzip header, detected
    set_error("inflateInit2 failed");
    return TFRG_E_IO;
  }
  uint64_t cap = size * 4 + 4096, len = 0;
  uint8_t* buf = (uint8_t*)malloc(cap);
  const uint8_t* p = in;
  uint64_t left = size;
  int rc = Z_OK;
  while (buf) {
    if (len == cap) {
      cap *= 2;
      uint8_t* nb = (uint8_t*)realloc(buf, cap);
      if (!nb) {
        free(buf);
        buf = nullptr;
        break;
      }
      buf = nb;
    }
    const uInt in_chunk = left > (1u << 30) ? (1u << 30) : (uInt)left;
    const uInt out_chunk = cap - len > (1u << 30) ? (1u << 30) : (uInt)(cap - len);
    zs.next_in = const_cast<Bytef*>(p);
    zs.avail_in = in_chunk;
    zs.next_out = buf + len;
    zs.avail_out = out_chunk;
    rc = inflate(&zs, Z_NO_FLUSH);
    p += in_chunk - zs.avail_in;
    left -= in_chunk - zs.avail_in;
    len += out_chunk - zs.avail_out;
    if (rc == Z_STREAM_END) {
      // concatenated gzip members (e.g. `cat a.gz b.gz`) decode as one stream
      if (left >= 2 && p[0] == 0x1f && p[1] == 0x8b && inflateReset(&zs) == Z_OK) continue;
      break;
    }
    if (rc != Z_OK && rc != Z_BUF_ERROR) break;
    if (rc == Z_BUF_ERROR && left == 0 && len < cap) break;  // truncated input
  }
  inflateEnd(&zs);
  if (!buf) {
    set_error("out of memory while inflating");
    return TFRG_E_NOMEM;
  }
  if (rc != Z_STREAM_END) {
    free(buf);
    set_error(std::string("corrupt or truncated compressed TFRecord stream (zlib: ") + (zs.msg ? zs.msg : "error") + ")");
    return TFRG_E_IO;
  }
  *out = buf;
  *out_len = len;
  return 0;
}

uint64_t tfrg_gather_ranges(const uint8_t* src, const uint64_t* starts, const uint64_t* ends, int64_t n,
                            uint8_t* dst) {
  uint64_t at = 0;
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t len = ends[i] > starts[i] ? ends[i] - starts[i] : 0;
    if (dst && len) memcpy(dst + at, src + starts[i], len);
    at += len;
  }
  return at;
}

}  // extern "C"

// ---- key discovery (tfrg_scan_keys) -----------------------------------------------------------
namespace {
struct PbCur {  // bounded protobuf cursor over [p, e)
  const uint8_t* p;
  const uint8_t* e;
  bool varint(uint64_t& v) {
    v = 0;
    for (int s = 0; s < 64 && p < e; s += 7) {
      const uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7f) << s;
      if (!(b & 0x80)) return true;
    }
    return false;
  }
  // next field: number, wire type, and for wire type 2 its body [bp, bp + bl)
  bool field(uint64_t& fn, uint32_t& wt, const uint8_t*& bp, uint64_t& bl) {
    uint64_t tag;
    if (p >= e || !varint(tag)) return false;
    fn = tag >> 3;
    wt = (uint32_t)(tag & 7);
    uint64_t v;
    switch (wt) {
      case 0: return varint(v);
      case 1: if (e - p < 8) return false; p += 8; return true;
      case 5: if (e - p < 4) return false; p += 4; return true;
      case 2:
        if (!varint(bl) || bl > (uint64_t)(e - p)) return false;
        bp = p;
        p += bl;
        return true;
      default: return false;
    }
  }
};

// a list message of a well-formed value list (bytes: length-delimited elements; float: packed
// 4-byte multiples or fixed32; int64: packed or single varints of <= 10 bytes)
bool list_ok(uint64_t kind, const uint8_t* p, uint64_t n) {
  PbCur c{p, p + n};
  uint64_t fn, bl;
  uint32_t wt;
  const uint8_t* bp = nullptr;
  while (c.p < c.e) {
    const uint8_t* at = c.p;
    if (!c.field(fn, wt, bp, bl) || fn != 1) return false;
    if (kind == 1) {
      if (wt != 2) return false;
    } else if (kind == 2) {
      if (!(wt == 5 || (wt == 2 && bl % 4 == 0))) return false;
    } else {
      if (wt == 0) {
        if (c.p - at > 11) return false;  // tag + a varint of <= 10 bytes
      } else if (wt == 2) {
        PbCur v{bp, bp + bl};
        while (v.p < v.e) {
          const uint8_t* s0 = v.p;
          uint64_t x;
          if (!v.varint(x) || v.p - s0 > 10) return false;
        }
      } else {
        return false;
      }
    }
  }
  return true;
}
}  // namespace

extern "C" {

int64_t tfrg_scan_keys(const uint8_t* bytes, uint64_t nbytes, const uint64_t* start, const uint64_t* end, int64_t n,
                       uint32_t flags, uint64_t* out, int64_t cap) {
  const bool framed = !(flags & 1u);  // TFRG_FLAG_PAYLOAD_ONLY
  std::unordered_set<std::string> seen;
  std::vector<std::pair<std::string, uint64_t>> rec;  // this record's (key + kind, key offset)
  int64_t k = 0;
  for (int64_t i = 0; i < n && k < cap; ++i) {
    uint64_t a = start[i], b = end[i];
    if (b > nbytes || a > b) continue;
    if (framed) {
      if (b - a < 16) continue;
      a += 12;
      b -= 4;
    }
    // only a canonical record seeds keys (Example = features fields, Features = map entries of key
    // then value, a Feature = one list field): its keys and kinds are exactly what the reference
    // decoder meets; any other record is left to the device's schema-miss pass
    rec.clear();
    bool ok = true;
    PbCur ex{bytes + a, bytes + b};
    uint64_t fn, bl;
    uint32_t wt;
    const uint8_t* bp = nullptr;
    while (ok && ex.p < ex.e) {
      if (!ex.field(fn, wt, bp, bl) || fn != 1 || wt != 2) {
        ok = false;
        break;
      }
      PbCur fs{bp, bp + bl};
      const uint8_t* ep = nullptr;
      uint64_t el;
      while (ok && fs.p < fs.e) {
        if (!fs.field(fn, wt, ep, el) || fn != 1 || wt != 2) {
          ok = false;
          break;
        }
        PbCur en{ep, ep + el};
        const uint8_t *kp = nullptr, *vp = nullptr;
        uint64_t kl = 0, vl = 0, f2 = 0, ql = 0;
        uint32_t w2 = 0;
        const uint8_t* q = nullptr;
        if (!en.field(f2, w2, kp, kl) || f2 != 1 || w2 != 2 || !en.field(f2, w2, vp, vl) || f2 != 2 || w2 != 2 ||
            en.p != en.e) {
          ok = false;
          break;
        }
        PbCur fe{vp, vp + vl};
        if (!fe.field(f2, w2, q, ql) || f2 < 1 || f2 > 3 || w2 != 2 || fe.p != fe.e || !list_ok(f2, q, ql)) {
          ok = false;
          break;
        }
        std::string id((const char*)kp, kl);
        id.push_back((char)f2);
        rec.emplace_back(std::move(id), (uint64_t)(kp - bytes));
      }
    }
    if (!ok) continue;
    for (auto& [id, off] : rec) {
      if (k >= cap) break;
      if (!seen.insert(id).second) continue;
      out[3 * k] = off;
      out[3 * k + 1] = id.size() - 1;
      out[3 * k + 2] = (uint8_t)id.back();
      ++k;
    }
  }
  return k;
}

int tfrg_idx_save(const char* idx_path, const uint64_t* triples, int64_t n) {
  FILE* f = fopen(idx_path, "wb");
  if (!f) return TFRG_E_IO;
  const size_t cnt = (size_t)n;
  bool ok = fwrite(&cnt, sizeof(size_t), 1, f) == 1;
  if (ok && cnt) ok = fwrite(triples, sizeof(uint64_t) * 3, cnt, f) == cnt;
  fclose(f);
  return ok ? 0 : TFRG_E_IO;
}

int tfrg_idx_load(const char* idx_path, uint64_t** out_triples, int64_t* n) {
  *out_triples = nullptr;
  *n = 0;
  FILE* f = fopen(idx_path, "rb");
  if (!f) {
    set_error(std::string("Cannot open index file: ") + idx_path);
    return TFRG_E_IO;
  }
  size_t cnt = 0;
  if (fread(&cnt, sizeof(size_t), 1, f) != 1) {
    fclose(f);
    set_error("Failed to read index file header");
    return TFRG_E_IO;
  }
  uint64_t* out = (uint64_t*)malloc(sizeof(uint64_t) * 3 * (cnt ? cnt : 1));
  if (!out) {
    fclose(f);
    set_error("Failed to allocate memory for index");
    return TFRG_E_NOMEM;
  }
  if (cnt && fread(out, sizeof(uint64_t) * 3, cnt, f) != cnt) {
    free(out);
    fclose(f);
    set_error("Failed to read index pointers");
    return TFRG_E_IO;
  }
  fclose(f);
  *out_triples = out;
  *n = (int64_t)cnt;
  return 0;
}

int64_t tfrg_frame_records(const uint8_t* payloads, const uint64_t* offsets, int64_t n, int crc, uint8_t* out,
                           int64_t out_cap) {
  int64_t total = 0;
  for (int64_t i = 0; i < n; ++i) total += 16 + (int64_t)(offsets[i + 1] - offsets[i]);
  if (!out || total > out_cap) return total;
  uint8_t* p = out;
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t len = offsets[i + 1] - offsets[i];
    memcpy(p, &len, 8);
    const uint32_t lc = crc ? tfrg_masked_crc32c(p, 8) : 0u;
    memcpy(p + 8, &lc, 4);
    memcpy(p + 12, payloads + offsets[i], len);
    const uint32_t dc = crc ? tfrg_masked_crc32c(payloads + offsets[i], len) : 0u;
    memcpy(p + 12 + len, &dc, 4);
    p += 16 + len;
  }
  return total;
}

}  // extern "C"
