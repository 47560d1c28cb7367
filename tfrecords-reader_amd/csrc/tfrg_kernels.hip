// tfrg_kernels.hip — gfx950 kernels for the TFRecord -> tf.train.Example -> Feature path.
//
// Pipeline for one batch of framed records resident in HBM (launch_decode):
//   1. k_lane_count  : one LANE per record. Records <= lane_max: the wave's contiguous span staged
//                      in LDS, framing check, masked CRC-32C of length and payload (slice-by-4 LDS
//                      tables), single-pass canonical walk of Example -> Features -> map entries ->
//                      Feature -> list (decoder.pyx:53-300 on canonical input). Records above
//                      lane_max: the same walk straight from HBM (their payload CRC is step 3).
//                      Per-slot counts summed per 256-record tile. Everything else -> slow list.
//   2. k_slow_count  : the exact reference walk (level-by-level error precedence, dict semantics,
//                      schema misses) for the slow list, one lane per record.
//   3. k_big_crc     : payload CRC of records above lane_max, one workgroup per record, the four
//                      waves recombined with GF(2) shift operators (crc32c.h).
//   4. k_spine       : exclusive scan of the tile sums per (slot, chunk) with a decoupled look-back
//                      across chunks; per-kind column bases (last workgroup).
//   5. k_down_gather : row splits (tile prefix + in-tile scan) and inline single values.
//   6. k_list_gather / k_stage_gather / k_wave_gather : out-of-line lists of lane records and of
//                      records above lane_max.
//
// The canonical walker and the exact walker share the count/gather sinks, so both paths produce
// identical columns (tests/test_gpu_parity.py forces each path on the same inputs).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <type_traits>
#include "tfrg_internal.h"
#include "crc32c.h"
#include "tfrg_walk.h"
#include "../../include/tfrg_status.h"

namespace tfrg {

// Optional per-phase cycle accounting of the wavefront kernels (make prof -> libtfrg_prof.so);
// compiled out of the product library.
#ifdef TFRG_PHASE_PROF
__device__ unsigned long long g_phase[32];
#define PHASE_MARK(t) const uint64_t t = __builtin_readcyclecounter()
#define PHASE_ADD(i, a, b) \
  do {                     \
    if (lane == 0) atomicAdd(&g_phase[i], (unsigned long long)((b) - (a))); \
  } while (0)
#else
#define PHASE_MARK(t) (void)0
#define PHASE_ADD(i, a, b) (void)0
#endif

// ------------------------------------------------------------------------------------------------
// Byte source: payload bytes of one record with the reference's out-of-range behaviour
// (index == L reads the CPython NUL terminator, index > L is reference UB), read through a
// per-lane 16-byte aligned window so that sequential parsing issues one 16 B load per 16 bytes.
// ------------------------------------------------------------------------------------------------
struct Src {
  const uint8_t* buf;
  uint64_t p0;  // absolute payload start
  int64_t L;    // payload length
  uint64_t wb;  // window base (absolute, 16-aligned)
  uint4 w;
  bool ub;

  __device__ __forceinline__ void init(const uint8_t* b, uint64_t p, int64_t len) {
    buf = b;
    p0 = p;
    L = len;
    wb = ~0ull;
    ub = false;
  }
  __device__ __forceinline__ uint32_t raw(uint64_t a) {
    const uint64_t base = a & ~15ull;
    if (base != wb) {
      w = *reinterpret_cast<const uint4*>(buf + base);
      wb = base;
    }
    const uint32_t k = (uint32_t)(a >> 2) & 3u;
    const uint32_t d = k == 0 ? w.x : (k == 1 ? w.y : (k == 2 ? w.z : w.w));
    return (d >> ((a & 3u) * 8u)) & 0xffu;
  }
  __device__ __forceinline__ uint32_t at(int64_t i) {
    if (i >= L) {
      ub |= (i > L);
      return 0u;
    }
    return raw(p0 + (uint64_t)i);
  }
  // 4 payload bytes at i (caller guarantees i + 4 <= L)
  __device__ __forceinline__ uint32_t u32(int64_t i) {
    return at(i) | (at(i + 1) << 8) | (at(i + 2) << 16) | (at(i + 3) << 24);
  }
};

// The same payload view over a wave's LDS stage: lds[0] holds absolute byte `lo`.
struct LdsSrc {
  const uint8_t* lds;
  uint64_t lo;
  uint64_t p0;
  int64_t L;
  bool ub;

  __device__ __forceinline__ void init(const uint8_t* l, uint64_t lo_, uint64_t p, int64_t len) {
    lds = l;
    lo = lo_;
    p0 = p;
    L = len;
    ub = false;
  }
  __device__ __forceinline__ uint32_t at(int64_t i) {
    if (i >= L) {
      ub |= (i > L);
      return 0u;
    }
    return lds[(uint32_t)(p0 - lo) + (uint32_t)i];
  }
  __device__ __forceinline__ uint32_t u32(int64_t i) {
    return at(i) | (at(i + 1) << 8) | (at(i + 2) << 16) | (at(i + 3) << 24);
  }
};

// ------------------------------------------------------------------------------------------------
// Count sink: dict semantics (insertion order, last value wins, first position kept) over
// (key, kind) slots, with the per-record rank state in LDS.
// ------------------------------------------------------------------------------------------------
// L: the dict lives in LDS (ord + cnt, explicitly LDS-typed so every access is a ds_* instruction,
// never a flat one); !L: in the global order / count columns (key tables too large for LDS).
typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
// constant address space: loads at wave-uniform indices compile to scalar loads (s_load, SGPRs)
typedef __attribute__((address_space(4))) const uint32_t cu32;

// single value stored in the loc word by the count pass
__device__ __forceinline__ void put_inline(const DevOut& o, uint32_t kind, uint2 lc, uint64_t dst) {
  if (kind == TFRG_KIND_INT64) {
    if (dst < o.cap_i64) o.i64[dst] = (int64_t)(((uint64_t)lc.y << 32) | lc.x);
  } else if (kind == TFRG_KIND_FLOAT) {
    if (dst < o.cap_f32) o.f32[dst] = lc.x;
  } else if (dst < o.cap_b) {
    o.b_off[dst] = lc.x;
    o.b_len[dst] = lc.y;
  }
}

// Speculative placement target of one slot (DevSchema::spec), staged in LDS by the lane kernel's
// prologue: the value column addresses at n * rank and the records r < lim that fit its capacity.
// The stores then need no DevOut field (seven pointers and capacities, which the register allocator
// otherwise kept spilled in VGPR lanes and reloaded with v_readlane per stored value).
// Layout: 8 u32 words per slot: [0, 2) p1 = int64 / float column, or bytes_list offsets, [2, 4) p2 =
// bytes_list lengths, [4] lim (records r < lim are stored: capacity), [5] kind.
typedef uint32_t spec_u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) spec_u32x4 lds_spec_t;
constexpr uint32_t kSpecTgtWords = 8;

__device__ __forceinline__ void spec_target(uint32_t* dst, const DevOut& o, uint32_t sw, uint32_t n) {
  const uint32_t kind = sw & 3u;
  uint64_t p1 = 0, p2 = 0;
  uint32_t lim = 0;
  if (sw) {
    const uint64_t base = (uint64_t)n * ((sw >> 2) - 1u);
    const uint64_t cap = kind == TFRG_KIND_INT64 ? o.cap_i64 : kind == TFRG_KIND_FLOAT ? o.cap_f32 : o.cap_b;
    lim = cap > base ? (cap - base < n ? (uint32_t)(cap - base) : n) : 0u;
    if (kind == TFRG_KIND_INT64) {
      p1 = (uint64_t)(o.i64 + base);
    } else if (kind == TFRG_KIND_FLOAT) {
      p1 = (uint64_t)(o.f32 + base);
    } else {
      p1 = (uint64_t)(o.b_off + base);
      p2 = (uint64_t)(o.b_len + base);
    }
  }
  dst[0] = (uint32_t)p1;
  dst[1] = (uint32_t)(p1 >> 32);
  dst[2] = (uint32_t)p2;
  dst[3] = (uint32_t)(p2 >> 32);
  dst[4] = lim;
  dst[5] = kind;
  dst[6] = dst[7] = 0;
}

// put_inline at a staged target (record r of the batch)
__device__ __forceinline__ void put_spec(const lds_spec_t* t, uint2 lc, uint32_t r) {
  const spec_u32x4 a = t[0], b = t[1];
  if (r >= b.x) return;
  const uint64_t p1 = ((uint64_t)a.y << 32) | a.x;
  if (b.y == TFRG_KIND_INT64) {
    reinterpret_cast<uint64_t*>(p1)[r] = ((uint64_t)lc.y << 32) | lc.x;
  } else if (b.y == TFRG_KIND_FLOAT) {
    reinterpret_cast<uint32_t*>(p1)[r] = lc.x;
  } else {
    reinterpret_cast<uint32_t*>(p1)[r] = lc.x;
    reinterpret_cast<uint32_t*>(((uint64_t)a.w << 32) | a.z)[r] = lc.y;
  }
}

template <bool L>
struct CountSinkT {
  using ord_t = std::conditional_t<L, lds_u16, uint16_t>;
  using cnt_t = std::conditional_t<L, lds_u32, uint32_t>;
  static constexpr bool kLds = L;
  const DevSchema* sc;
  const DevOut* o;
  ord_t* ord;        // ord[slot * ostride]
  uint32_t ostride;
  uint32_t rank;
  uint32_t n, r;
  uint64_t p0;
  bool miss;
  bool leader;       // issues global writes and atomics
  cnt_t* cnt = nullptr;  // LDS value counts, same layout as ord (L only)
  const lds_u32* spec = nullptr;  // DevSchema::spec staged in LDS (L only; null = off)
  const lds_spec_t* spec_t = nullptr;  // its targets (kSpecTgtWords per slot)

  __device__ __forceinline__ void reset() {
    for (uint32_t k = 0; k < sc->n_slots; ++k) ord[(size_t)k * ostride] = 0;
    rank = 0;
  }

  // key bytes -> key id; -1 unknown, -2 interned as invalid UTF-8
  template <class S>
  __device__ int lookup(S& s, int64_t off, int64_t len) {
    if (sc->n_keys == 0 || len > 0xffffffffll) return -1;
    uint32_t w0 = 0, w1 = 0;
    for (int64_t i = 0; i < (len < 4 ? len : 4); ++i) w0 |= s.at(off + i) << (8 * i);
    if (len > 4)
      for (int64_t i = 0; i < 4; ++i) w1 |= s.at(off + len - 4 + i) << (8 * i);
    const uint32_t h = key_hash_words((uint32_t)len, w0, w1);
    uint32_t j = h & sc->ht_mask;
    for (uint32_t probe = 0; probe <= sc->ht_mask; ++probe) {
      const uint32_t e = sc->ht[j];
      if (!e) return -1;
      const uint32_t kid = e - 1;
      const uint32_t ko = sc->key_off[kid];
      if (sc->key_hash[kid] == h && (int64_t)(sc->key_off[kid + 1] - ko) == len &&
          sc->key_w[2 * kid] == w0 && sc->key_w[2 * kid + 1] == w1) {
        const uint8_t* kb = sc->key_blob + ko;
        bool eq = true;
        for (int64_t i = 4; i < len - 4 && eq; ++i) eq = s.at(off + i) == kb[i];
        if (eq) return (sc->key_slot[kid * 4] & 1) ? -2 : (int)kid;
      }
      j = (j + 1) & sc->ht_mask;
    }
    return -1;
  }

  __device__ void note_miss(int kind, int64_t koff, int64_t klen) {
    miss = true;
    if (leader) {
      const uint32_t i = atomicAdd(&o->info[kInfoMissEntries], 1u);
      if (i < o->miss_cap) {
        uint32_t* m = o->miss + 4ull * i;
        m[0] = r;
        m[1] = (uint32_t)kind;
        m[2] = (uint32_t)(p0 + (uint64_t)koff);
        m[3] = (uint32_t)klen;
      }
    }
  }

  __device__ int insert(int kid, int kind, int64_t lo, int64_t ll, uint32_t count, int64_t koff,
                        int64_t klen) {
    const int slot = kid >= 0 ? sc->key_slot[kid * 4 + kind] : -1;
    if (slot < 0) {  // schema miss: report the (key, kind) so the host can intern it
      note_miss(kind, koff, klen);
      return TFRG_OK;
    }
    uint32_t rk = 0;
    for (int k = 1; k <= 3; ++k) {  // duplicate key (any kind): keep its first position
      const int s2 = sc->key_slot[kid * 4 + k];
      if (s2 >= 0) {
        const uint32_t v = ord[(size_t)s2 * ostride];
        if (v) {
          rk = v;
          ord[(size_t)s2 * ostride] = 0;
        }
      }
    }
    if (!rk) {
      if (rank >= 65534u) return TFRG_ST_LIMIT;
      rk = ++rank;
    }
    ord[(size_t)slot * ostride] = (uint16_t)rk;
    if (count & kCountInline) return TFRG_ST_LIMIT;  // >= 2^31 values in one list
    if constexpr (L) cnt[(size_t)slot * ostride] = count;
    if (leader) {
      const size_t at = (size_t)slot * n + r;
      if constexpr (!L) o->count[at] = count;
      o->loc[at] = make_uint2((uint32_t)lo, (uint32_t)ll);
    }
    return TFRG_OK;
  }

  // canonical-walker interface (fast_walk)
  __device__ __forceinline__ void fast_reset(uint32_t S) {
    for (uint32_t k = 0; k < S; ++k) ord[(size_t)k * ostride] = 0;
  }
  __device__ __forceinline__ bool fast_taken(const uint32_t* kr) const {  // any kind of this key present
    bool t = false;
    for (int k = 0; k < 3; ++k) {
      const int s2 = (int)kr[kKrSlot1 + k];
      t |= s2 >= 0 && ord[(size_t)s2 * ostride] != 0;
    }
    return t;
  }
  __device__ __forceinline__ void fast_put(uint32_t slot, uint32_t rk, uint32_t cw, uint2 lv) {
    ord[(size_t)slot * ostride] = (uint16_t)rk;
    const size_t at = (size_t)slot * n + r;
    if constexpr (L) cnt[(size_t)slot * ostride] = cw;
    else o->count[at] = cw;
    if constexpr (L) {
      if (spec) {  // speculative placement of a single value (DevSchema::spec): no loc word (k_spine
                   // copies the value back into it if the slot's placement fails)
        const uint32_t sw = spec[slot];
        if (sw && (cw & kCountInline)) {
          put_spec(spec_t + 2u * slot, lv, r);
          return;
        }
      }
    }
    o->loc[at] = lv;
  }

  // final count of a present slot (LDS, or read back from this thread's own column write)
  __device__ __forceinline__ uint32_t count_of(uint32_t k) const {
    if constexpr (L) return cnt[(size_t)k * ostride];
    else return o->count[(size_t)k * n + r];
  }

  // dict -> order / count columns of a lane-per-record walk; present counts are added to the
  // record's tile sum (the row-split scan's first level)
  __device__ __forceinline__ void finalize(bool ok) {
    for (uint32_t k = 0; k < sc->n_slots; ++k) {
      const uint32_t v = ok ? ord[(size_t)k * ostride] : 0u;
      const uint32_t c = v ? count_of(k) : 0u;
      if (leader) {
        const size_t at = (size_t)k * n + r;
        o->order[at] = (uint16_t)v;
        o->count[at] = c;
        if (c & ~kCountInline) atomicAdd(&o->tsum[(size_t)k * o->tile_stride + (r >> kTileShift)], c & ~kCountInline);
      }
    }
  }
};

template <bool L>
__device__ __forceinline__ typename CountSinkT<L>::ord_t* dict_ord(uint16_t* global, uint16_t* shared) {
  if constexpr (L) return (lds_u16*)shared;
  else return global;
}

// Canonical-walker dict for schemas of <= 64 slots whose per-lane LDS dict does not fit: the order /
// count / loc columns are written as the walk goes, the present slots kept in a 64-bit mask, and the
// counts added to the wave's LDS tile sums (rolled back from the columns if the walk bails).
struct MaskSink {
  const DevOut* o;
  uint32_t n, r;
  lds_u32* tsl;  // [64] this wave's tile sums
  uint64_t pm = 0;
  uint32_t rank = 0;
  __device__ __forceinline__ void fast_reset(uint32_t) { pm = 0; }
  __device__ __forceinline__ bool fast_taken(const uint32_t* kr) const {
    bool t = false;
    for (int k = 0; k < 3; ++k) {
      const int s2 = (int)kr[kKrSlot1 + k];
      t |= s2 >= 0 && ((pm >> s2) & 1ull);
    }
    return t;
  }
  __device__ __forceinline__ void fast_put(uint32_t slot, uint32_t rk, uint32_t cw, uint2 lv) {
    const size_t at = (size_t)slot * n + r;
    o->order[at] = (uint16_t)rk;
    o->count[at] = cw;
    o->loc[at] = lv;
    pm |= 1ull << slot;
    __atomic_fetch_add(&tsl[slot], cw & ~kCountInline, __ATOMIC_RELAXED);
  }
  __device__ __forceinline__ void rollback() {  // this thread's own column writes, read back
    for (uint64_t m = pm; m; m &= m - 1) {
      const uint32_t k = (uint32_t)__builtin_ctzll(m);
      __atomic_fetch_sub(&tsl[k], o->count[(size_t)k * n + r] & ~kCountInline, __ATOMIC_RELAXED);
    }
    pm = 0;
  }
  __device__ __forceinline__ void zero_absent(uint32_t S) {
    for (uint32_t k = 0; k < S; ++k) {
      if ((pm >> k) & 1ull) continue;
      const size_t at = (size_t)k * n + r;
      o->order[at] = 0;
      o->count[at] = 0;
    }
  }
};

// ------------------------------------------------------------------------------------------------
// CRC-32C helpers
// ------------------------------------------------------------------------------------------------
// LDS table view with R-fold bank replication: entry (j, v) copy c at dword ((j*256+v)*R + c).
// Lane l reads copy l % R, so up to R lanes of a 32-lane group never collide on a bank.
// a ^ b ^ c in one VALU (gfx950 v_bitop3_b32, truth table 0x96; the compiler does not fuse XOR chains)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// ((x >> 8K) & 0xff) * 4 in one VALU: a shift with an SDWA byte select of its source
template <int K>
__device__ __forceinline__ uint32_t byte_x4(uint32_t x) {
  static_assert(K >= 0 && K < 4, "byte index");
  uint32_t r;
  const uint32_t two = 2u;
  if constexpr (K == 0)
    asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0"
        : "=v"(r) : "v"(two), "v"(x));
  else if constexpr (K == 1)
    asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
        : "=v"(r) : "v"(two), "v"(x));
  else if constexpr (K == 2)
    asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2"
        : "=v"(r) : "v"(two), "v"(x));
  else
    asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3"
        : "=v"(r) : "v"(two), "v"(x));
  return r;
}

template <int R>
struct LdsTab {
  const uint32_t* t;
  uint32_t c;
  __device__ __forceinline__ uint32_t operator()(uint32_t j, uint32_t v) const { return t[((j << 8) + v) * R + c]; }
  // entry of table j at byte offset bx4 = 4 * index
  __device__ __forceinline__ uint32_t at4(uint32_t j, uint32_t bx4) const {
    return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(t) + (j << 10) + bx4);
  }
  __device__ __forceinline__ uint32_t step4(uint32_t x) const {
    if constexpr (R == 1)  // table byte offsets in one SDWA instruction each (the lane kernel is VALU-bound)
      return xor3(at4(3, byte_x4<0>(x)), at4(2, byte_x4<1>(x)), at4(1, byte_x4<2>(x))) ^ at4(0, byte_x4<3>(x));
    return (*this)(3, x & 0xffu) ^ (*this)(2, (x >> 8) & 0xffu) ^ (*this)(1, (x >> 16) & 0xffu) ^ (*this)(0, x >> 24);
  }
  __device__ __forceinline__ uint32_t step1(uint32_t c_, uint32_t byte) const {
    return (*this)(0, (c_ ^ byte) & 0xffu) ^ (c_ >> 8);
  }
  // 8 bytes (x = state ^ first word, y = second word); needs the slice-by-8 table set
  __device__ __forceinline__ uint32_t step8(uint32_t x, uint32_t y) const {
    return (*this)(7, x & 0xffu) ^ (*this)(6, (x >> 8) & 0xffu) ^ (*this)(5, (x >> 16) & 0xffu) ^
           (*this)(4, x >> 24) ^ (*this)(3, y & 0xffu) ^ (*this)(2, (y >> 8) & 0xffu) ^
           (*this)(1, (y >> 16) & 0xffu) ^ (*this)(0, y >> 24);
  }
};

// Serial CRC-32C of absolute bytes [a, b) by one lane: aligned 16 B loads, slice-by-4 for whole
// words, byte steps at the unaligned edges.
template <int R>
__device__ uint32_t crc_serial(const uint8_t* buf, uint64_t a, uint64_t b, const LdsTab<R>& T) {
  uint32_t c = 0xffffffffu;
  for (uint64_t q = a & ~15ull; q < b; q += 16) {
    const uint4 w = *reinterpret_cast<const uint4*>(buf + q);
    const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t wa = q + 4ull * k;
      if (wa >= a && wa + 4 <= b) {
        c = T.step4(c ^ ws[k]);
      } else if (wa + 4 > a && wa < b) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint64_t ba = wa + j;
          if (ba >= a && ba < b) c = T.step1(c, ws[k] >> (8 * j));
        }
      }
    }
  }
  return ~c;
}

__device__ __forceinline__ uint32_t load_u32_unaligned(const uint8_t* buf, uint64_t a) {
  uint32_t v = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) v |= (uint32_t)buf[a + j] << (8 * j);
  return v;
}
__device__ __forceinline__ uint64_t load_u64_unaligned(const uint8_t* buf, uint64_t a) {
  return (uint64_t)load_u32_unaligned(buf, a) | ((uint64_t)load_u32_unaligned(buf, a + 4) << 32);
}

// ------------------------------------------------------------------------------------------------
// Per-record framing: payload range, verdict bits, read errors.
// ------------------------------------------------------------------------------------------------
struct RecView {
  uint64_t st, e;   // absolute [st, e) clamped to the buffer
  uint64_t en;      // end as given (unclamped; the framing length check compares against it)
  uint64_t p0;
  int64_t L;
  int status;
  uint32_t verdict;
};

__device__ __forceinline__ RecView rec_view_se(const DevBatch& B, uint64_t st, uint64_t en) {
  RecView v;
  v.st = st;
  v.en = en;
  v.status = TFRG_OK;
  v.verdict = 0;
  const bool framed = !(B.flags & kFlagPayloadOnly);
  if (st > en || (framed ? st >= B.nbytes : en > B.nbytes)) {  // reader.py:48-49 empty read
    v.status = TFRG_ERR_READ;
    v.e = st;
    v.p0 = st;
    v.L = 0;
    return v;
  }
  v.e = en < B.nbytes ? en : B.nbytes;
  if (en > B.nbytes) v.verdict |= TFRG_V_TRUNCATED;
  if (framed) {  // reader.py:55: data = example_data[12:-4]
    const uint64_t D = v.e - st;
    v.p0 = st + 12;
    v.L = D >= 16 ? (int64_t)(D - 16) : 0;
  } else {
    v.p0 = st;
    v.L = (int64_t)(v.e - st);
  }
  return v;
}

__device__ __forceinline__ RecView rec_view(const DevBatch& B, uint32_t r) {
  return rec_view_se(B, rec_start(B, r), rec_end(B, r));
}

// ------------------------------------------------------------------------------------------------
// Kernels
// ------------------------------------------------------------------------------------------------
constexpr int kLaneBlock = 256;
constexpr int kLaneCountBlock = 256;  // k_lane_count workgroup (its LDS tables are per workgroup)
constexpr int kWaveBlock = 256;
constexpr int kWavesPerBlock = kWaveBlock / 64;

__device__ __forceinline__ void record_result(const DevOut& o, uint32_t r, int status, int64_t aux,
                                              uint32_t verdict) {
  o.status[r] = status;
  if (status != TFRG_OK) o.aux[r] = aux;  // aux is defined only for failing records
  o.verdict[r] = (uint8_t)verdict;
  if (status == TFRG_ST_SCHEMA_MISS) {
    atomicAdd(&o.info[kInfoMissRecords], 1u);
  } else if (status != TFRG_OK) {
    atomicAdd(&o.info[kInfoErrors], 1u);
    atomicMax(&o.info[kInfoFirstError], ~r);  // stored inverted: zero-initialised with the rest
  }
}

// TFRG_FLAG_STRICT_CRC: a framed record is accepted only with a matching length field and masked
// CRC-32Cs (need_data = false while the payload CRC is still k_big_crc's work).
__device__ __forceinline__ bool strict_pass(const DevBatch& B, uint32_t verdict, bool need_data) {
  if (!(B.flags & kFlagStrictCrc) || (B.flags & kFlagPayloadOnly)) return true;
  const uint32_t need = TFRG_V_LEN_MATCH | TFRG_V_LEN_CRC | (need_data ? TFRG_V_DATA_CRC : 0u);
  return (verdict & need) == need;
}

// ------------------------------------------------------------------------------------------------
// Wave staging for the lane-per-record kernels: the 64 records of a wave are (in the common case of
// whole-file batches) one contiguous span of a few KiB. The wave copies that span into its LDS stage
// with coalesced 16-byte loads (1 KiB per wave-instruction) and every lane then parses its record
// from LDS instead of issuing scattered, latency-bound global loads.
// ------------------------------------------------------------------------------------------------
constexpr uint32_t kStageBytes = 4096;   // span capacity per wave
constexpr uint32_t kStageStride = kStageBytes + 64;   // + slack for aligned over-reads at the tail

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t x) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    const uint64_t y = __shfl_xor(x, m, 64);
    x = y < x ? y : x;
  }
  return x;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t x) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    const uint64_t y = __shfl_xor(x, m, 64);
    x = y > x ? y : x;
  }
  return x;
}

// Span [lo, hi) covering the records of the lanes with `in` set. Whole-file batches are ascending
// and contiguous, so the first / last participating lanes bound it; one ballot verifies that and
// the 64-bit shuffle reductions run only when it does not hold.
__device__ __forceinline__ void wave_span(bool in, uint64_t a, uint64_t b, uint64_t& lo, uint64_t& hi) {
  const uint64_t m = __ballot(in);
  if (!m) {
    lo = ~0ull;
    hi = 0;
    return;
  }
  const int f = __builtin_ctzll(m), l = 63 - __builtin_clzll(m);
  const uint64_t lo_c = __shfl(a, f, 64), hi_c = __shfl(b, l, 64);
  if (__ballot(in && (a < lo_c || b > hi_c)) == 0) {
    lo = lo_c;
    hi = hi_c;
    return;
  }
  lo = wave_min_u64(in ? a : ~0ull);
  hi = wave_max_u64(in ? b : 0ull);
}

// Memory writes of one wave made visible to its other lanes. A wavefront's memory instructions
// are processed in order, so wavefront scope needs no waits (workgroup scope would drain every
// outstanding global store, a multi-microsecond stall per call); this orders the compiler only.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr uint32_t kWStage = 12288;          // staged record bytes per wave (wavefront kernels)
constexpr uint32_t kWStageStride = kWStage + 64;

// copy absolute bytes [lo16, hi) (lo16 16-aligned, wave-uniform, hi - lo16 <= kStageBytes) into dst
__device__ __forceinline__ void stage_span(uint8_t* dst, const uint8_t* src, uint64_t lo16, uint64_t hi,
                                           uint32_t lane) {
  // scalar base + 32-bit lane offsets: the address arithmetic stays off the (busy) VALU
  const uint64_t l0 = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(lo16 >> 32)) << 32) |
                      __builtin_amdgcn_readfirstlane((uint32_t)lo16);
  const uint32_t n = __builtin_amdgcn_readfirstlane((uint32_t)(hi - lo16));
  const uint8_t* base = src + l0;
  // four 1 KiB wave-loads in flight per round, unconditional (clamped offsets) so that all four
  // are issued before the first wait, held in named registers (no scratch)
  for (uint32_t off = lane * 16u; off < n; off += 4096u) {
    const bool h1 = off + 1024u < n, h2 = off + 2048u < n, h3 = off + 3072u < n;
    const uint4 a = *reinterpret_cast<const uint4*>(base + off);
    const uint4 b = *reinterpret_cast<const uint4*>(base + (h1 ? off + 1024u : off));
    const uint4 c = *reinterpret_cast<const uint4*>(base + (h2 ? off + 2048u : off));
    const uint4 d = *reinterpret_cast<const uint4*>(base + (h3 ? off + 3072u : off));
    *reinterpret_cast<uint4*>(dst + off) = a;
    if (h1) *reinterpret_cast<uint4*>(dst + off + 1024u) = b;
    if (h2) *reinterpret_cast<uint4*>(dst + off + 2048u) = c;
    if (h3) *reinterpret_cast<uint4*>(dst + off + 3072u) = d;
  }
}

// 4 unaligned bytes at stage offset `off` (two aligned LDS dwords + a byte funnel shift)
__device__ __forceinline__ uint32_t lds_u32u(const uint8_t* l, uint32_t off) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(l);
  const uint32_t a = off >> 2;
  // always both dwords (one ds_read2_b32, no divergent branch); alignbyte by 0 returns the low one
  return __builtin_amdgcn_alignbyte(w[a + 1], w[a], off & 3u);
}

// CRC-32C of stage bytes [a, b): byte steps to 4-alignment, slice-by-4 words, byte tail
template <int R>
__device__ uint32_t crc_lds(const uint8_t* l, uint32_t a, uint32_t b, const LdsTab<R>& T) {
  uint32_t c = 0xffffffffu;
  while (a < b && (a & 3u)) c = T.step1(c, l[a++]);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(l);
  for (; a + 4 <= b; a += 4) c = T.step4(c ^ w[a >> 2]);
  while (a < b) c = T.step1(c, l[a++]);
  return ~c;
}

// as crc_lds, 8 bytes per dependent step (T holds the slice-by-8 set), with no byte loops: the
// k = a & 3 bytes before `a` in its dword are read as zeros and the start state is ~0 (x) x^(-8k)
// (prepending zero bytes to a message multiplies the state by x^8 each, crc32c.h), and the last
// m = b & 3 bytes take one partial slicing step T[m-1][x0] ^ ... ^ T[0][x(m-1)] ^ (c >> 8m).
__device__ __forceinline__ uint32_t crc_head_state(uint32_t k) {
  // ~0 (x) x^(-8k) for k = 0..3 (checked against crc32c("123456789") with k zero bytes prepended)
  return k == 0 ? 0xffffffffu : (k == 1 ? 0xa942e6bcu : (k == 2 ? 0x2804363bu : 0x96db52a8u));
}
constexpr int kLaneSlice = 4;  // slicing width of the lane kernel's CRC (4 KiB of tables)

template <int R>
__device__ __forceinline__ uint32_t crc_lds8(const uint8_t* l, uint32_t a, uint32_t b, const LdsTab<R>& T) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(l);
  const uint32_t k = a & 3u, bw = b & ~3u, m = b & 3u;
  uint32_t p = a & ~3u;
  uint32_t c = crc_head_state(k);
  uint32_t hm = 0xffffffffu << (8u * k);  // masks the bytes before a in the first dword
  for (; p + 12 <= bw; p += 8) {  // two words per iteration (one ds_read2, half the loop overhead)
    const uint32_t x0 = w[p >> 2], x1 = w[(p >> 2) + 1];
    c = T.step4(c ^ (x0 & hm));
    hm = 0xffffffffu;
    c = T.step4(c ^ x1);
  }
  if (p + 8 <= bw) {
    c = T.step4(c ^ (w[p >> 2] & hm));
    hm = 0xffffffffu;
    p += 4;
  }
  if (p + 4 <= bw) {
    c = T.step4(c ^ (w[p >> 2] & hm));
    hm = 0xffffffffu;
    p += 4;
  }
  if (m) {  // partial dword: m = 1..3 bytes
    const uint32_t x = c ^ (w[p >> 2] & hm);
    uint32_t t = T(m - 1u, x & 0xffu);
    const uint32_t t1 = T(m >= 2u ? m - 2u : 0u, (x >> 8) & 0xffu);
    const uint32_t t2 = T(0u, (x >> 16) & 0xffu);
    t ^= m >= 2u ? t1 : 0u;
    t ^= m == 3u ? t2 : 0u;
    c = t ^ (c >> (8u * m));
  }
  return ~c;
}

// ------------------------------------------------------------------------------------------------
// Fast walker for canonical, valid records in the LDS stage. Single pass, 32-bit positions,
// 4-byte varint reads, word-wise key match, terminator popcount for packed int64. It accepts only
// records whose reference result is unambiguous (every field where a serializer puts it, no
// error, no duplicate or unknown key, tag/length varints <= 4 bytes, no varint overrun) and
// returns kBail for anything else; the lane then re-walks that record with the exact walker.
// ------------------------------------------------------------------------------------------------
constexpr int kBail = -1;

struct FastSrc {
  const uint8_t* l;  // stage
  uint32_t p;        // payload offset in the stage
  uint32_t L;        // payload length
  uint64_t base;     // absolute offset of the payload in the input (bytes views)
  // 4 payload bytes at i (i <= L); bytes at index >= L read as 0 (the NUL terminator and beyond)
  __device__ __forceinline__ uint32_t w4(uint32_t i) const {
    uint32_t w = lds_u32u(l, p + i);
    const uint32_t rem = L - i;
    if (rem < 4) w &= (1u << (8 * rem)) - 1u;
    return w;
  }
  // as w4, any i (0 at and past L)
  __device__ __forceinline__ uint32_t w4s(uint32_t i) const { return i < L ? w4(i) : 0u; }
  // 4 bytes at payload offset i, unmasked (the canonical walker bounds-checks what it uses)
  __device__ __forceinline__ uint32_t u32(uint32_t i) const { return lds_u32u(l, p + i); }
  __device__ __forceinline__ void window(uint32_t) const {}  // (the stage is the window)
  __device__ __forceinline__ void prefetch(uint32_t) const {}
  __device__ __forceinline__ void advance() const {}
};

// The same payload view over HBM (records beyond the LDS stage): two aligned dword loads + a byte
// funnel shift, clamped to the readable end of the batch (round_up(nbytes, 16)).
// A 32-byte register window (two aligned 16-byte blocks) is loaded at the start of every map entry
// (window()): the entry's headers, a short key and the first list chunk header are then served
// from registers, one HBM round trip per entry instead of one per dependent header. WIN = false
// compiles the window out (the per-lane-dict kernel: its registers would cost C1 occupancy).
template <bool WIN>
struct FastSrcG {
  const uint8_t* buf;
  uint64_t base;  // absolute payload start
  uint32_t L;
  uint64_t lim;   // last readable dword
  mutable uint64_t wa = 0;  // window start (16-aligned absolute address)
  mutable bool wv = false;  // window loaded
  mutable uint4 b0, b1;
  mutable uint64_t pa = ~0ull;  // prefetched window of the next map entry (its start, validity, blocks)
  mutable bool pv = false;
  mutable uint4 p0, p1;
  __device__ __forceinline__ void window(uint32_t i) const {
    if (!WIN) return;
    const uint64_t a = (base + i) & ~15ull;
    wv = a + 32u <= lim + 4u;  // both blocks readable
    const uint64_t lb = lim - 12u;  // last readable 16-byte block
    wa = a;
    b0 = *reinterpret_cast<const uint4*>(buf + (a < lb ? a : lb));
    b1 = *reinterpret_cast<const uint4*>(buf + (a + 16u < lb ? a + 16u : lb));
  }
  // the next entry's window, requested as soon as this entry's extent is known (it then overlaps
  // this entry's key lookup and list-count loads instead of adding a round trip per entry), made the
  // window by advance() at the end of the entry (plain register moves, no condition)
  __device__ __forceinline__ void advance() const {
    if (!WIN) return;
    wa = pa;
    wv = pv;
    b0 = p0;
    b1 = p1;
  }
  __device__ __forceinline__ void prefetch(uint32_t i) const {
    if (!WIN) return;
    const uint64_t a = (base + i) & ~15ull;
    pv = a + 32u <= lim + 4u;
    const uint64_t lb = lim - 12u;
    pa = a;
    p0 = *reinterpret_cast<const uint4*>(buf + (a < lb ? a : lb));
    p1 = *reinterpret_cast<const uint4*>(buf + (a + 16u < lb ? a + 16u : lb));
  }
  __device__ __forceinline__ uint32_t u32(uint32_t i) const {
    const uint64_t a = base + i;
    const uint64_t off = a - wa;
    if (WIN && wv && off <= 27u) {  // words k, k+1 of the window: select chains (no dynamic register index)
      const uint32_t k = (uint32_t)off >> 2;
      const uint32_t e0 = (k & 1u) ? b0.y : b0.x, e1 = (k & 1u) ? b0.w : b0.z;
      const uint32_t e2 = (k & 1u) ? b1.y : b1.x, e3 = (k & 1u) ? b1.w : b1.z;
      const uint32_t lo = k < 4u ? ((k & 2u) ? e1 : e0) : ((k & 2u) ? e3 : e2);
      const uint32_t k1 = k + 1u;
      const uint32_t f0 = (k1 & 1u) ? b0.y : b0.x, f1 = (k1 & 1u) ? b0.w : b0.z;
      const uint32_t f2 = (k1 & 1u) ? b1.y : b1.x, f3 = (k1 & 1u) ? b1.w : b1.z;
      const uint32_t hi = k1 < 4u ? ((k1 & 2u) ? f1 : f0) : ((k1 & 2u) ? f3 : f2);
      return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(a & 3u));
    }
    const uint64_t a0 = a & ~3ull;
    const uint32_t w0 = *reinterpret_cast<const uint32_t*>(buf + (a0 < lim ? a0 : lim));
    const uint32_t w1 = *reinterpret_cast<const uint32_t*>(buf + (a0 + 4 < lim ? a0 + 4 : lim));
    return __builtin_amdgcn_alignbyte(w1, w0, (uint32_t)(a & 3u));
  }
};

// 7-bit groups of the bytes of w selected by byte mask m, compacted (a varint of <= 4 bytes)
__device__ __forceinline__ uint32_t vgroups(uint32_t w, uint32_t m) {
  w &= m;
  return (w & 0x7fu) | ((w >> 1) & 0x3f80u) | ((w >> 2) & 0x1fc000u) | ((w >> 3) & 0xfe00000u);
}
// byte mask of the first nb (1..4) bytes: shifts only (a multiply by 7 would be quarter rate)
__device__ __forceinline__ uint32_t bytes_mask(uint32_t nb) { return nb >= 4u ? 0xffffffffu : (1u << (nb << 3)) - 1u; }

// varint of <= 4 bytes (values < 2^28: identical in compat and spec mode); false = bail
__device__ __forceinline__ bool fv32(const FastSrc& s, uint32_t& pos, uint32_t& v) {
  if (pos > s.L) return false;
  const uint32_t w = s.w4(pos);
  const uint32_t term = ~w & 0x80808080u;
  if (!term) return false;
  const uint32_t nb = (__builtin_ctz(term) >> 3) + 1u;
  v = vgroups(w, term ^ (term - 1u));  // bytes up to the first terminator
  pos += nb;
  return true;
}

// a length-delimited field inside [pos, end): returns its field number, payload offset and length.
// Common case: 1-byte tag + 1..3-byte length, decoded from ONE 4-byte stage read.
__device__ __forceinline__ bool ffield(const FastSrc& s, uint32_t& pos, uint32_t end, uint32_t& fn, uint32_t& off,
                                       uint32_t& len) {
  if (pos > s.L) return false;
  const uint32_t w = s.w4(pos);
  if ((w & 0x87u) != 0x02u) {  // tag longer than 1 byte, or not wire type 2
    uint32_t key;
    if (!fv32(s, pos, key) || (key & 7u) != 2u) return false;
    fn = key >> 3;
    if (!fv32(s, pos, len) || pos > end || len > end - pos) return false;
    off = pos;
    pos += len;
    return true;
  }
  fn = (w & 0x7fu) >> 3;
  uint32_t l, hb;
  if (!(w & 0x8000u)) {
    l = (w >> 8) & 0x7fu;
    hb = 2;
  } else if (!(w & 0x800000u)) {
    l = ((w >> 8) & 0x7fu) | ((w >> 9) & 0x3f80u);
    hb = 3;
  } else if (!(w & 0x80000000u)) {
    l = ((w >> 8) & 0x7fu) | ((w >> 9) & 0x3f80u) | ((w >> 10) & 0x1fc000u);
    hb = 4;
  } else {
    return false;
  }
  const uint32_t q = pos + hb;
  if (q > end || l > end - q) return false;
  off = q;
  len = l;
  pos = q + l;
  return true;
}

// number of varints in a packed chunk [o, e) that ends on a terminator, with no varint longer
// than 10 bytes (else bail: 'Too many bytes' / overrun semantics are the exact walker's)
template <class S>
__device__ __forceinline__ bool count_packed(const S& s, uint32_t o, uint32_t e, uint32_t& cnt) {
  uint32_t run = 0, terms = 0, last = 0x80u;
  for (uint32_t i = o; i < e; i += 4) {
    const uint32_t w = s.u32(i);
    const uint32_t rem = e - i;
    const uint32_t valid = rem >= 4 ? 0x80808080u : (0x80808080u & ((1u << (8 * rem)) - 1u));
    const uint32_t term = ~w & valid;
    const uint32_t nvalid = __popc(valid);
    if (!term) {
      run += nvalid;
      if (run >= 10) return false;
    } else {
      if (run + (__builtin_ctz(term) >> 3) >= 10) return false;
      run = nvalid - 1u - ((31u - __builtin_clz(term)) >> 3);
      terms += __popc(term);
    }
    last = (w >> (8 * (nvalid - 1u))) & 0x80u;
  }
  if (e > o && last) return false;  // the last varint runs past the chunk
  cnt = terms;
  return true;
}

// bit 7 of the 16 bytes of a block, byte i -> bit i
__device__ __forceinline__ uint32_t cont16(uint4 b) {
  auto nib = [](uint32_t w) {
    w = (w >> 7) & 0x01010101u;
    return (w | (w >> 7) | (w >> 14) | (w >> 21)) & 0xfu;
  };
  return nib(b.x) | (nib(b.y) << 4) | (nib(b.z) << 8) | (nib(b.w) << 12);
}
// One 16-byte block of a packed chunk, bytes [lo, hi) of it inside the chunk: its terminators added,
// the run of continuation bytes carried in / out, `bad` set by a varint of more than 10 bytes (runs
// of >= 10 continuation bytes after a terminator found by a 10-fold AND of shifts)
__device__ __forceinline__ void packed_block(uint4 blk, uint32_t lo, uint32_t hi, uint32_t& run, uint32_t& terms,
                                             bool& bad) {
  const uint32_t valid = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
  const uint32_t m = cont16(blk), t = ~m & valid, cm = m & valid;
  const uint32_t a = cm & (cm >> 1), b = a & (a >> 2), c = b & (b >> 4);
  bad |= ((c & (a >> 8)) & (t << 1)) != 0u;
  if (!t) {
    run += hi - lo;
  } else {
    bad |= run + (uint32_t)__builtin_ctz(t) - lo >= 10u;  // the run carried in, ended here
    run = hi - 1u - (31u - (uint32_t)__builtin_clz(t));
    terms += (uint32_t)__popc(t);
  }
  bad |= run >= 10u;
}
// count_packed over HBM (records walked from HBM): aligned 16-byte blocks, two loads in flight per
// round instead of one dependent dword pair per word (a packed list of 300 bytes was 75 serial
// round trips; four blocks per round would cost the staged path its occupancy in VGPRs)
// (NB blocks per round: k_body_count, whose lanes count independent bodies, takes 8: one round for
// a body of up to ~112 bytes)
template <int NB = 2, bool WIN>
__device__ __forceinline__ bool count_packed(const FastSrcG<WIN>& s, uint32_t o, uint32_t e, uint32_t& cnt) {
  uint32_t run = 0, terms = 0;
  const uint64_t a0 = s.base + o, a1 = s.base + e;
  // last block to load: the chunk's last one (spare loads of a round re-read it: no line past the
  // chunk is fetched), never past the last readable 16-byte block
  const uint64_t lb0 = s.lim - 12, lbc = a1 > a0 ? (a1 - 1) & ~15ull : a0 & ~15ull;
  const uint64_t lb = lbc < lb0 ? lbc : lb0;
  for (uint64_t q = a0 & ~15ull; q < a1; q += 16 * NB) {
    uint4 blk[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const uint64_t qq = q + 16u * j;
      blk[j] = *reinterpret_cast<const uint4*>(s.buf + (qq < lb ? qq : lb));
    }
    if constexpr (NB > 2) {  // (k_body_count: a block at a time)
      bool bad = false;
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const uint64_t qb = q + 16u * j;
        if (qb >= a1) break;
        const uint32_t lo = a0 > qb ? (uint32_t)(a0 - qb) : 0u;
        const uint32_t hi = a1 - qb < 16u ? (uint32_t)(a1 - qb) : 16u;
        packed_block(blk[j], lo, hi, run, terms, bad);
      }
      if (bad) return false;
    } else {  // (the lane kernel's walk: a word at a time, fewer live registers)
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const uint32_t ws[4] = {blk[j].x, blk[j].y, blk[j].z, blk[j].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint64_t wa = q + 16u * j + 4u * k;
          if (wa >= a1 || wa + 4 <= a0) continue;
          const uint32_t lo = wa < a0 ? (uint32_t)(a0 - wa) : 0u;  // valid bytes [lo, hi) of this word
          const uint32_t hi = wa + 4 <= a1 ? 4u : (uint32_t)(a1 - wa);
          const uint32_t vm = bytes_mask(hi) & ~((1u << (lo << 3)) - 1u);
          const uint32_t term = ~ws[k] & vm & 0x80808080u;
          if (!term) {
            run += hi - lo;
            if (run >= 10) return false;
          } else {
            if (run + (__builtin_ctz(term) >> 3) - lo >= 10) return false;
            run = hi - 1u - ((31u - __builtin_clz(term)) >> 3);
            terms += __popc(term);
          }
        }
      }
    }
  }
  if (e > o && run) return false;  // the last varint runs past the chunk
  cnt = terms;
  return true;
}

__device__ __forceinline__ bool fast_list_count(const FastSrc& s, uint32_t kind, uint32_t lo, uint32_t ll,
                                                uint32_t& cnt) {
  uint32_t q = lo, c = 0;
  const uint32_t le = lo + ll;
  while (q < le) {
    uint32_t fn, co, cl;
    if (!ffield(s, q, le, fn, co, cl) || fn != 1u) return false;
    if (kind == TFRG_KIND_BYTES) {
      ++c;
    } else if (kind == TFRG_KIND_FLOAT) {
      if (cl & 3u) return false;
      c += cl >> 2;
    } else {
      uint32_t k;
      if (!count_packed(s, co, co + cl, k)) return false;
      c += k;
    }
  }
  cnt = c;
  return true;
}

// LDS copy of the key table for the fast path: hash table + packed key records
struct LdsKeys {
  const uint32_t* ht;    // [mask+1] key id + 1
  const uint32_t* rec;   // [n_keys][kKrWords]
  uint32_t mask;
  const uint8_t* blob = nullptr;   // global key bytes + offsets: the middle of keys longer than 8 bytes
  const uint32_t* koff = nullptr;
};

// key id for key bytes at [ko, ko+kl) of the payload; -1 = not a plain hit (bail)
template <class S>
__device__ __forceinline__ int fast_lookup(const S& s, const LdsKeys& K, uint32_t ko, uint32_t kl) {
  if (kl > 256u) return -1;  // very long keys: exact walker
  uint32_t w0 = s.u32(ko);
  if (kl < 4) w0 &= (1u << (8 * kl)) - 1u;
  const uint32_t w1 = kl > 4 ? s.u32(ko + kl - 4) : 0u;
  const uint32_t h = key_hash_words(kl, w0, w1);
  uint32_t j = h & K.mask;
  for (uint32_t probe = 0; probe <= K.mask; ++probe) {
    const uint32_t e = K.ht[j];
    if (!e) return -1;
    const uint32_t* r = K.rec + (e - 1) * kKrWords;
    const uint4 q = *reinterpret_cast<const uint4*>(r);  // (hash, len, w0, w1): one 16-byte read
    static_assert(kKrHash == 0 && kKrLen == 1 && kKrW0 == 2 && kKrW1 == 3, "record head layout");
    if ((q.x == h) & (q.y == kl) & (q.z == w0) & (q.w == w1)) {
      // (length, first 4, last 4) identify keys of <= 8 bytes; longer ones compare the middle too
      bool eq = true;
      if (kl > 8u) {
        const uint8_t* kb = K.blob + K.koff[e - 1];
        for (uint32_t i = 4; eq && i < kl - 4u; i += 4) {
          const uint32_t jj = i + 4u <= kl - 4u ? i : kl - 8u;
          eq = s.u32(ko + jj) == load_u32_unaligned(kb, jj);
        }
      }
      if (eq) return (r[kKrFlags] & 1u) ? -1 : (int)(e - 1);
    }
    j = (j + 1) & K.mask;
  }
  return -1;
}

// One packed int64 varint at `pos` of a validated chunk ending at `e` (fast gather path); false = bail.
template <bool COMPAT>
__device__ __forceinline__ bool fast_value(const FastSrc& s, uint32_t& pos, uint32_t e, int64_t& val) {
  const uint32_t w = s.w4(pos);
  const uint32_t term = ~w & 0x80808080u;
  if (term) {
    const uint32_t nb = (__builtin_ctz(term) >> 3) + 1u;
    if (pos + nb > e) return false;
    val = (int64_t)vgroups(w, term ^ (term - 1u));
    pos += nb;
    return true;
  }
  // 5..10 bytes: two more words, terminator found by bit scan, groups combined branch-free (no
  // dependent byte-at-a-time chain: a long varint costs one extra LDS round trip)
  const uint32_t w1 = s.w4s(pos + 4), w2 = s.w4s(pos + 8);
  const uint32_t t1 = ~w1 & 0x80808080u, t2 = ~w2 & 0x00008080u;
  uint32_t nb;
  if (t1) nb = 5u + (__builtin_ctz(t1) >> 3);
  else if (t2) nb = 9u + (__builtin_ctz(t2) >> 3);
  else return false;  // > 10 bytes: "Too many bytes when decoding varint." (exact path)
  if (pos + nb > e) return false;
  const uint32_t x = (w & 0x7fu) | ((w >> 1) & 0x3f80u) | ((w >> 2) & 0x1fc000u) | ((w >> 3) & 0xfe00000u);
  const uint32_t g4 = w1 & 0x7fu;
  const uint32_t g5 = nb > 5u ? (w1 >> 8) & 0x7fu : 0u;
  const uint32_t g6 = nb > 6u ? (w1 >> 16) & 0x7fu : 0u;
  const uint32_t g7 = nb > 7u ? (w1 >> 24) & 0x7fu : 0u;
  const uint32_t g8 = nb > 8u ? w2 & 0x7fu : 0u;
  const uint32_t g9 = nb > 9u ? (w2 >> 8) & 0x7fu : 0u;
  pos += nb;
  if (COMPAT) {  // term_k = (int32)(g_k << (7k & 31)), sign-extended, OR-ed (decoder.pyx:34-50)
    const uint32_t lo32 = x | (g4 << 28) | (g5 << 3) | (g6 << 10) | (g7 << 17) | (g8 << 24) | (g9 << 31);
    const bool neg = ((g4 >> 3) | g9) & 1u;
    val = (int64_t)(((uint64_t)(neg ? 0xffffffffu : 0u) << 32) | lo32);
  } else {
    val = (int64_t)((uint64_t)x | ((uint64_t)g4 << 28) | ((uint64_t)g5 << 35) | ((uint64_t)g6 << 42) |
                    ((uint64_t)g7 << 49) | ((uint64_t)g8 << 56) | ((uint64_t)g9 << 63));
  }
  return true;
}

// A list holding exactly one value: the value itself, packed into the 8-byte loc word (int64 bits,
// float bits in .x, or the bytes element's absolute (offset, length)). The gather then writes it
// without touching the record again. false = keep the list location.
template <bool COMPAT>
__device__ __forceinline__ bool fast_single(const FastSrc& s, uint32_t kind, uint32_t lo, uint32_t ll, uint2& val) {
  uint32_t q = lo, fn, co, cl;
  if (!ffield(s, q, lo + ll, fn, co, cl) || fn != 1u || q != lo + ll) return false;
  if (kind == TFRG_KIND_BYTES) {
    val = make_uint2((uint32_t)(s.base + co), cl);
    return true;
  }
  if (kind == TFRG_KIND_FLOAT) {
    if (cl != 4u) return false;
    val = make_uint2(lds_u32u(s.l, s.p + co), 0u);
    return true;
  }
  // int64: one varint of <= 4 bytes filling the chunk (values < 2^28, same in both varint modes)
  if (cl == 0u || cl > 4u) return false;
  const uint32_t w = s.w4(co);
  const uint32_t term = ~w & 0x80808080u;
  if (!term || (__builtin_ctz(term) >> 3) + 1u != cl) return false;
  val = make_uint2(vgroups(w, bytes_mask(cl)), 0u);
  return true;
}


// Branch-free header of a length-delimited field at `pos` inside [pos, end): 1-byte tag with wire
// type 2, 1..3-byte length, body inside `end`. Anything else is not canonical (ok = false); the
// outputs are then garbage but positions stay inside the record, so the caller may keep computing
// and decide once.
template <class S>
__device__ __forceinline__ bool hdr2(const S& s, uint32_t pos, uint32_t end, uint32_t& fn, uint32_t& off,
                                     uint32_t& len) {
  pos = pos < s.L ? pos : s.L;
  const uint32_t w = s.u32(pos);
  if (__builtin_expect((w & 0x8087u) == 0x0002u, 1)) {  // 1-byte length (< 128): a third of the VALU
    fn = (w >> 3) & 0xfu;
    off = pos + 2u;
    len = (w >> 8) & 0x7fu;
    return off + len <= end;  // (pos <= L < 2^31: no wrap)
  }
  const uint32_t b1 = (w >> 8) & 0xffu, b2 = (w >> 16) & 0xffu, b3 = w >> 24;
  const uint32_t c1 = b1 >> 7, c12 = c1 & (b2 >> 7);
  uint32_t l = b1 & 0x7fu;
  l |= c1 ? (b2 & 0x7fu) << 7 : 0u;
  l |= c12 ? b3 << 14 : 0u;
  fn = (w >> 3) & 0xfu;
  off = pos + 2u + c1 + c12;
  len = l;
  return ((w & 0x87u) == 0x02u) & !(c12 & (b3 >> 7)) & (off <= end) & (l <= end - off);
}

// Returns TFRG_OK with the dict in sink.ord / cnt (or count) / loc, or kBail (exact walker).
// Every level is a single canonical pass: one Features field spanning the Example, map entries of
// exactly (key #1, value #2), one kind field spanning the Feature, list chunks of field #1.
// Deferred counting of packed int64 bodies (records walked from HBM). Counting a list's packed
// chunk on the spot costs the lane a dependent HBM round trip per 32 bytes of every body, one list
// after the other: 58 % of C3's count pass (0.72 -> 0.30 ms in a build that skipped those loads).
// Instead the lane lists (record, slot, absolute body offset, length) in its record's row and leaves
// the count word 0; k_body_count then counts every listed body in one flat pass, all of them
// independent (bandwidth, not latency), and writes the count words and tile sums. A body that does
// not count canonically sends its record to the exact walker, which withdraws its columns first.
struct NoDefer {
  __device__ __forceinline__ bool push(uint32_t, uint64_t, uint32_t) const { return false; }
};
struct BodyDefer {
  uint4* row;  // entry 0 of this lane's record (nullptr: count on the spot); entry j at row[64 j]
  uint32_t r;
  mutable uint32_t n = 0;
  __device__ __forceinline__ bool push(uint32_t slot, uint64_t at, uint32_t len) const {
    if (!row || n >= kDeferK) return false;
    row[64u * n++] = make_uint4(r, slot, (uint32_t)at, len);  // (a batch is < 4 GiB)
    return true;
  }
};

template <bool COMPAT, class Sink, class S, class D = NoDefer>
__device__ __forceinline__ int fast_walk(const S& s, const LdsKeys& K, Sink& sink, const D& dfr = D{}) {
  const uint32_t L = s.L;
  uint32_t fn, fo, fl;
  bool ok = hdr2(s, 0, L, fn, fo, fl) & (fn == 1u) & (fo + fl == L);
  uint64_t seen = 0;  // key ids < 64 already in the dict (a duplicate key bails)
  uint32_t rank = 0;
  const uint32_t fe = fo + fl;
  if (ok && fo < fe) s.window(fo);  // (later entries' windows are prefetched)
  for (uint32_t q = fo; ok && q < fe;) {
    uint32_t en, eo, el, kn, ko, kl, vn, vo, vl, kind, lo, ll;
    ok = hdr2(s, q, fe, en, eo, el) & (en == 1u);
    const uint32_t ee = eo + el;
    q = ee;
    s.prefetch(q);
    ok &= hdr2(s, eo, ee, kn, ko, kl) & (kn == 1u);
    ok &= hdr2(s, ko + kl, ee, vn, vo, vl) & (vn == 2u) & (vo + vl == ee);
    ok &= hdr2(s, vo, ee, kind, lo, ll) & (lo + ll == ee) & (kind - 1u < 3u);
    if (!ok) break;
    const int kid = fast_lookup(s, K, ko, kl);
    // list chunks (field #1, packed); the first chunk's single value is kept for the inline path
    uint32_t cnt = 0, nch = 0, c0o = 0, c0l = 0, c0w = 0;
    const uint32_t le = lo + ll;
    for (uint32_t g = lo; ok && g < le;) {
      uint32_t cf, co, cl;
      ok = hdr2(s, g, le, cf, co, cl) & (cf == 1u);
      g = co + cl;
      if (kind == TFRG_KIND_BYTES) {
        ++cnt;
      } else if (kind == TFRG_KIND_FLOAT) {
        ok &= (cl & 3u) == 0u;
        cnt += cl >> 2;
      } else if (cl <= 4u) {  // one word: its terminators; the chunk must end on one
        const uint32_t m = bytes_mask(cl);
        const uint32_t w = s.u32(co) & m;
        const uint32_t tm = ~w & 0x80808080u & m;
        ok &= cl == 0u || ((tm >> ((cl << 3) - 1u)) & 1u);
        cnt += __popc(tm);
        if (nch == 0) c0w = w;
      } else {
        // the list's only chunk, of a known key: its count can wait for k_body_count
        const int dslot = (nch == 0 && g == le && kid >= 0) ? (int)K.rec[(uint32_t)kid * kKrWords + kKrSlot1 + 2u] : -1;
        if (!(dslot >= 0 && dfr.push((uint32_t)dslot, s.base + co, cl))) {
          uint32_t k = 0;
          ok &= count_packed(s, co, co + cl, k);
          cnt += k;
        }
      }
      if (nch == 0) {
        c0o = co;
        c0l = cl;
      }
      ++nch;
    }
    ok &= kid >= 0;
    if (!ok) break;
    const uint32_t* kr = K.rec + (uint32_t)kid * kKrWords;
    const int slot = (int)kr[kKrSlot1 + kind - 1];
    if (kid < 64) {
      const uint64_t bit = 1ull << kid;
      ok &= !(seen & bit);
      seen |= bit;
    } else {
      ok &= !sink.fast_taken(kr);
    }
    ok &= (slot >= 0) & (rank < 65534u);
    if (!ok) break;
    ++rank;
    // a single value goes inline into the loc word (int64 bits, float bits, bytes view)
    uint2 lv = make_uint2(lo, ll);
    uint32_t cw = cnt;
    if (cnt == 1u && nch == 1u) {
      if (kind == TFRG_KIND_BYTES) {
        lv = make_uint2((uint32_t)(s.base + c0o), c0l);
        cw = 1u | kCountInline;
      } else if (kind == TFRG_KIND_FLOAT) {
        lv = make_uint2(s.u32(c0o), 0u);
        cw = 1u | kCountInline;
      } else if (c0l <= 4u) {  // one varint of <= 4 bytes: value < 2^28, same in both varint modes
        lv = make_uint2(vgroups(c0w, 0xffffffffu), 0u);  // (the chunk's word, masked to c0l bytes)
        cw = 1u | kCountInline;
      }
    }
    sink.fast_put((uint32_t)slot, rank, cw, lv);
    s.advance();
  }
  sink.rank = rank;
  return ok ? TFRG_OK : kBail;
}

// Framing verdicts of one record: length field vs the given range, masked CRC-32C of the 8 length
// bytes and of the payload (the TFRecord spec; absent from the reference), from the
// wave's LDS stage (STAGED) or from HBM.
// payload_crc = false leaves the payload CRC of a record above lane_max to k_wave_count.
template <int R, bool STAGED>
__device__ __forceinline__ void frame_verdicts(const DevBatch& B, RecView& v, const LdsTab<R>& T, const uint8_t* stage,
                                               uint64_t lo16, bool payload_crc = true) {
  if (B.flags & kFlagPayloadOnly) return;
  const bool do_crc = !(B.flags & kFlagNoCrc);
  const uint64_t D = v.e - v.st;
  if (D < 8) return;
  uint64_t lenf;
  uint32_t lw0 = 0, lw1 = 0;
  if constexpr (STAGED) {
    const uint32_t o0 = (uint32_t)(v.st - lo16);
    lw0 = lds_u32u(stage, o0);
    lw1 = lds_u32u(stage, o0 + 4);
    lenf = (uint64_t)lw0 | ((uint64_t)lw1 << 32);
  } else {
    lenf = load_u64_unaligned(B.bytes, v.st);
  }
  if (lenf == v.en - v.st - 16) v.verdict |= TFRG_V_LEN_MATCH;
  if (do_crc && D >= 12) {
    uint32_t want, stored;
    if constexpr (STAGED) {
      stored = lds_u32u(stage, (uint32_t)(v.st - lo16) + 8);
      // the two words just read: two slicing steps at any alignment
      want = crc_mask(~T.step4(T.step4(0xffffffffu ^ lw0) ^ lw1));
    } else {
      want = crc_mask(crc_serial<R>(B.bytes, v.st, v.st + 8, T));
      stored = load_u32_unaligned(B.bytes, v.st + 8);
    }
    if (want == stored) v.verdict |= TFRG_V_LEN_CRC;
  }
  if (do_crc && payload_crc && D >= 16) {
    uint32_t c, stored;
    if constexpr (STAGED) {
      c = crc_lds8<R>(stage, (uint32_t)(v.p0 - lo16), (uint32_t)(v.e - 4 - lo16), T);
      stored = lds_u32u(stage, (uint32_t)(v.e - 4 - lo16));
    } else {
      c = crc_serial<R>(B.bytes, v.p0, v.e - 4, T);
      stored = load_u32_unaligned(B.bytes, v.e - 4);
    }
    if (crc_mask(c) == stored) v.verdict |= TFRG_V_DATA_CRC;
  }
}

// Inclusive prefix sum over the wave (every lane active) in seven DPP adds, no LDS: rows of 16 by
// row_shr 1, 2, 3 of the value, then 4 and 8 of the partial sums (bank masks: only the lanes that
// still miss a part), then the row totals by row_bcast 15 / 31 (gfx9 DPP; lanes a mask leaves out
// read `old` = 0). Replaces six ds_bpermute round trips of __shfl_up.
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v, uint32_t) {
  uint32_t s = v + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);  // row_shr:1
  s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);             // row_shr:2
  s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x113, 0xf, 0xf, true);             // row_shr:3
  s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x114, 0xf, 0xe, true);             // row_shr:4
  s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x118, 0xf, 0xc, true);             // row_shr:8
  s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x142, 0xa, 0xf, false);            // row_bcast:15
  s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x143, 0xc, 0xf, false);            // row_bcast:31
  return s;
}

// wave total (every lane active), wave-uniform: the scan's last lane
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan_u32(x, 0u), 63);
}

// XOR of every lane's value (every lane active), wave-uniform: the scan above with XOR
__device__ __forceinline__ uint32_t wave_xor_u32(uint32_t v) {
  uint32_t s = v ^ (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);
  s ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);
  s ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x113, 0xf, 0xf, true);
  s ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x114, 0xf, 0xe, true);
  s ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x118, 0xf, 0xc, true);
  s ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x142, 0xa, 0xf, false);
  s ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x143, 0xc, 0xf, false);
  return (uint32_t)__builtin_amdgcn_readlane((int)s, 63);
}

// 1 KiB rounds (64 lanes x aligned 16-byte chunks) covering the payload [a, b), b > a
__device__ __forceinline__ uint32_t crc_rounds_of(uint64_t a, uint64_t b) {
  return (uint32_t)((((b - 1) >> 4) - (a >> 4) + 64) >> 6);
}

// Lists this wave's accepted large records (j = their round count, 0 = none) for the streaming
// payload CRC (k_tail_count role 2). ONE 64-bit atomic per wave returns both the list index and
// the flat round base, so list order and round order agree: entry i owns the flat rounds
// [crc_base[i], crc_base[i + 1]).
__device__ __forceinline__ void crc_list_append(const DevOut& o, uint32_t r, uint32_t j, uint32_t lane) {
  const uint64_t m = __ballot(j != 0);
  if (!m) return;
  const uint32_t incl = wave_incl_scan_u32(j, lane);
  const uint32_t tot = __shfl(incl, 63, 64);
  unsigned long long t = 0;
  if (lane == 0)
    t = atomicAdd(reinterpret_cast<unsigned long long*>(o.info + kInfoCrcCtr),
                  ((unsigned long long)__popcll(m) << kCrcIdxShift) | tot);
  const uint64_t tu = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(t >> 32), 0, 64) << 32) |
                      (uint32_t)__shfl((int)(uint32_t)t, 0, 64);
  if (j) {
    const uint32_t idx = (uint32_t)(tu >> kCrcIdxShift) + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    o.crc_rec[idx] = r;
    o.crc_base[idx] = (tu & kCrcRoundMask) + incl - j;
    o.crc_part[idx] = 0;
  }
}

// Wave-uniform values loaded with VECTOR loads: a laundered (VGPR) index keeps the compiler from
// turning the load into a scalar one, whose lgkmcnt would be drained by every LDS wait of the walk.
__device__ __forceinline__ uint32_t vgpr_launder(uint32_t x) {
  uint32_t y;
  asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "s"(x));
  return y;
}
__device__ __forceinline__ uint32_t rfl32(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t rfl64(uint64_t x) {
  return ((uint64_t)rfl32((uint32_t)(x >> 32)) << 32) | rfl32((uint32_t)x);
}

// Lane-per-record kernel, the general path. Each wave copies the contiguous span of its 64 records
// into its LDS stage, then every lane checks its record's framing + CRC and runs the single-pass
// canonical walker (fast_walk). Records the fast walker does not accept (non-canonical, erroneous,
// unknown keys) and framing errors are listed for the exact walker (k_tail_count role 1); records
// above lane_max, and the lane records of a wave whose span does not fit the stage, are walked from
// HBM. The per-slot value counts of the accepted records are summed per 256-record tile (first level
// of the row-split scan).
// Residual mode (DevOut::rlist set): only the records k_tpl_lane did not take, i.e. the 64-record
// groups it listed, each with its miss mask (DevOut::lmask).
// MODE: 0 = per-lane dict in LDS, 1 = MaskSink (<= 64 slots), 2 = dict in the global columns.
template <int R, bool COMPAT, int MODE>
__global__ __launch_bounds__(kLaneCountBlock, MODE == 0 ? 6 : 4) void k_lane_count(DevBatch B, DevSchema sc, DevOut o,
                                                                                  const uint32_t* __restrict__ crc_tab,
                                                                                  uint32_t lane_max, uint32_t wave_stage,
                                                                                  uint32_t defer_big) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  // slicing tables at a static LDS address: lookups fold the table base into the ds_read offset
  __shared__ uint32_t tab[256 * kLaneSlice * R];
  constexpr uint32_t kWaves = kLaneCountBlock / 64;
  uint32_t* cnt = lds;                                       // [n_slots][kLaneCountBlock]
  constexpr bool GORD = MODE != 0;  // no per-lane LDS dict
  const uint32_t S = sc.n_slots;
  const uint32_t cnt_words = GORD ? 0u : S * kLaneCountBlock;
  uint16_t* ord = reinterpret_cast<uint16_t*>(cnt + cnt_words);              // [n_slots][kLaneCountBlock]
  const uint32_t ord_bytes = GORD ? 0u : ((S * kLaneCountBlock * 2u + 15u) & ~15u);
  const uint32_t lane = threadIdx.x & 63u, wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // residual mode: a workgroup with no listed group exits before loading its tables (block-uniform)
  const bool resid = o.rlist != nullptr;
  if (blockIdx.x == 0 && threadIdx.x < kInfoCount) o.info_next[threadIdx.x] = 0u;  // (the next decode's)
  const uint32_t nres = resid ? rfl32(o.info[kInfoResid]) : 0u;
  if (resid && blockIdx.x * kWaves >= nres) return;
  uint8_t* stage_all = reinterpret_cast<uint8_t*>(ord) + ord_bytes;
  uint8_t* stage = stage_all + wib * kStageStride;
  uint32_t* kht = reinterpret_cast<uint32_t*>(stage_all + kWaves * kStageStride);
  uint32_t* krec = kht + ((sc.ht_mask + 4u) & ~3u);
  lds_u32* tsl = (lds_u32*)(krec + sc.n_keys * kKrWords) + wib * 64u;  // MODE 1: this wave's tile sums
  uint32_t* spec_l = krec + sc.n_keys * kKrWords + (MODE == 1 ? kWaves * 64u : 0u);  // MODE 0: DevSchema::spec
  uint32_t* spec_tl = spec_l + ((S + 7u) & ~7u);  // MODE 0: its targets (16-byte aligned)
  // 64-record groups: group g of the batch, or (residual mode) the g-th listed group with its mask
  const uint32_t nw = gridDim.x * kWaves;
  auto group = [&](uint32_t g, uint64_t& gb, uint64_t& gm) -> bool {
    if (resid) {
      if (g >= nres) return false;
      const uint32_t w = rfl32(o.rlist[g]);
      gb = (uint64_t)w * 64u;
      gm = rfl64(o.lmask[w]);
      return true;
    }
    gb = (uint64_t)g * 64u;
    gm = ~0ull;
    return gb < B.n;
  };
  uint32_t g = blockIdx.x * kWaves + wib;
  uint64_t base = 0, gmask = 0;
  bool more = group(g, base, gmask);
  // the next group's offsets are requested before this group's stores (one HBM round trip less on
  // the critical path of the next group); the first group's before the workgroup's table copy, so
  // that its round trip overlaps the copy
  uint64_t nst = 0, nen = 0;
  if (more && base + lane < B.n) {
    nst = rec_start(B, (uint32_t)(base + lane));
    nen = rec_end(B, (uint32_t)(base + lane));
  }

  for (uint32_t i = threadIdx.x; i < 256u * kLaneSlice * R; i += kLaneCountBlock) tab[i] = crc_tab[2048 + i / R];
  if constexpr (MODE == 1) {
    tsl[lane] = 0;
  }
  const bool fast_ok = sc.n_keys <= kLdsMaxKeys && sc.ht_mask + 1 <= kLdsMaxHt;  // else every record is slow
  if (fast_ok) {
    for (uint32_t i = threadIdx.x; i <= sc.ht_mask; i += kLaneCountBlock) kht[i] = sc.ht[i];
    for (uint32_t i = threadIdx.x; i < sc.n_keys * kKrWords; i += kLaneCountBlock) krec[i] = sc.krec[i];
  }
  const bool spec_on = MODE == 0 && fast_ok && sc.spec != nullptr;
  if (spec_on)
    for (uint32_t i = threadIdx.x; i < S; i += kLaneCountBlock) {
      spec_l[i] = sc.spec[i];
      spec_target(spec_tl + kSpecTgtWords * i, o, sc.spec[i], B.n);
    }
  __syncthreads();
  const LdsKeys K{kht, krec, sc.ht_mask, sc.key_blob, sc.key_off};
  const LdsTab<R> T{tab, threadIdx.x & (R - 1)};
  while (more) {
    PHASE_MARK(p0);
    const uint64_t ri = base + lane;
    const bool valid = ri < B.n && ((gmask >> lane) & 1ull);
    const uint32_t r = (uint32_t)ri;
    const uint32_t tile = (uint32_t)(base >> kTileShift);
    const uint64_t cst0 = nst, cen0 = nen;
    g += nw;
    more = group(g, base, gmask);
    if (more && base + lane < B.n) {
      nst = rec_start(B, (uint32_t)(base + lane));
      nen = rec_end(B, (uint32_t)(base + lane));
    }
    RecView v{};
    bool mine = false, big = false;
    if (valid) {
      v = rec_view_se(B, cst0, cen0);
      big = v.status == TFRG_OK && v.e - v.st > lane_max;  // (listed for the wave gathers below)
      mine = !big;
    }
    // (defer_big: a record above lane_max is walked by k_tail_count beside the streaming CRC,
    // role_big_walk; here it is only listed for the CRC and its verdict byte cleared)
    const bool deferred = defer_big && big;
    {
      const uint64_t bm = __ballot(big);
      if (bm && lane == 0) atomicAdd(&o.info[kInfoBigRecs], (uint32_t)__popcll(bm));
    }
    // wave-uniform staging decision over the span of this wave's records
    const bool span_rec = fast_ok && mine && v.status == TFRG_OK;
    uint64_t lo, hi;
    wave_span(span_rec, v.st, v.e, lo, hi);
    const uint64_t lo16 = lo & ~15ull;
    const bool staged = hi > lo && hi - lo16 <= kStageBytes;
    if (staged) {
      stage_span(stage, B.bytes, lo16, hi, lane);
      wave_lds_sync();
    }
    PHASE_MARK(p1);
    PHASE_ADD(16, p0, p1);
    using SinkT = std::conditional_t<MODE == 1, MaskSink, CountSinkT<MODE == 0>>;
    SinkT sink = [&]() {
      if constexpr (MODE == 1) {
        return MaskSink{&o, B.n, r, tsl};
      } else {
        CountSinkT<MODE == 0> c{&sc, &o, dict_ord<MODE == 0>(o.order + r, ord + threadIdx.x),
                                GORD ? B.n : (uint32_t)kLaneCountBlock, 0, B.n, r, v.p0, false, true};
        if constexpr (MODE == 0) {
          c.cnt = (lds_u32*)(cnt + threadIdx.x);
          if (spec_on) {
            c.spec = (const lds_u32*)spec_l;
            c.spec_t = (const lds_spec_t*)spec_tl;
          }
        }
        return c;
      }
    }();
    bool done = false;
    bool tried = false;
    uint32_t nd = 0;  // packed int64 bodies of this record deferred to k_body_count
    if (staged && span_rec) {
      const FastSrc fs{stage, (uint32_t)(v.p0 - lo16), (uint32_t)v.L, v.p0};
      frame_verdicts<R, true>(B, v, T, stage, lo16, true);
      PHASE_MARK(p2);
      PHASE_ADD(17, p1, p2);
      sink.fast_reset(S);
      if (strict_pass(B, v.verdict, true)) {  // (strict mode: a CRC failure is the slow kernel's)
        done = fast_walk<COMPAT>(fs, K, sink) == TFRG_OK;
        tried = true;
      }
      PHASE_MARK(p3);
      PHASE_ADD(18, p2, p3);
    }
    // records above lane_max, and lane records of a wave whose span does not fit the stage: the
    // canonical walk straight from HBM, one record per lane (64 latency chains in flight per wave).
    // The payload CRC of records above lane_max is the streaming CRC's (k_tail_count role 2); the
    // others' is computed here, serially per lane from HBM.
    const bool bigw = fast_ok && valid && !deferred && (!mine || (span_rec && !staged));
    if (__ballot(bigw)) {
      // one block of deferred-body rows per wave (k_body_count), while the batch has room
      uint32_t blk = ~0u;
      if (MODE != 0 && o.dq) {  // (MODE 0, narrow schemas: its register budget keeps the in-place count)
        if (lane == 0) blk = atomicAdd(&o.info[kInfoDefer], 1u);
        blk = rfl32((uint32_t)__shfl((int)blk, 0, 64));
        if (blk >= o.dq_blocks) blk = ~0u;
      }
      if (bigw) {
        // (the payload CRC of a large record is role 2's stream, unless it is shorter than one round)
        const bool crc_here = mine || (uint64_t)v.L < kCrcListMin;
        frame_verdicts<R, false>(B, v, T, nullptr, 0, crc_here);
        sink.fast_reset(S);
        if (strict_pass(B, v.verdict, crc_here)) {
          const FastSrcG<MODE != 0> fg{B.bytes, v.p0, (uint32_t)v.L, ((B.nbytes + 15) & ~15ull) - 4};
          if constexpr (MODE != 0) {
            const BodyDefer dfr{blk != ~0u ? o.dq + (size_t)blk * 64u * kDeferK + lane : nullptr, r};
            done = fast_walk<COMPAT>(fg, K, sink, dfr) == TFRG_OK;
            nd = dfr.n;
          } else {
            done = fast_walk<COMPAT>(fg, K, sink) == TFRG_OK;
          }
          tried = true;
        }
      }
      if (MODE != 0 && blk != ~0u) o.dq_cnt[(size_t)blk * 64u + lane] = (uint8_t)(bigw && done ? nd : 0u);
    }
    PHASE_MARK(p4);
    // everything else of this wave's records goes to the exact walker
    const bool slow = valid && !done && !deferred;
    const uint64_t sm = __ballot(slow);
    if (sm) {
      uint32_t b0 = 0;
      if (lane == (uint32_t)__builtin_ctzll(sm)) b0 = atomicAdd(&o.info[kInfoSlow], (uint32_t)__popcll(sm));
      b0 = __shfl(b0, __builtin_ctzll(sm), 64);
      if (slow) {
        o.slow_list[b0 + (uint32_t)__popcll(sm & ((1ull << lane) - 1ull))] = r;
        o.verdict[r] = (uint8_t)kVerdictPending;
      }
    }
    if (done) {
      o.status[r] = TFRG_OK;
      o.verdict[r] = (uint8_t)v.verdict;
    } else if (deferred) {
      o.verdict[r] = 0;  // (bits OR-ed in by role_big_walk and role 2)
    }
    // the payload CRC of an accepted (or deferred) large record: one entry of the streaming CRC list
    const bool crc_on = !(B.flags & (kFlagPayloadOnly | kFlagNoCrc));
    const uint32_t crc_j =
        (done || deferred) && !mine && crc_on && v.e - v.st >= 16 && (uint64_t)v.L >= kCrcListMin ? crc_rounds_of(v.p0, v.e - 4) : 0u;
    // order / count columns of the accepted records + the tile sums (one atomic per slot and wave)
    if constexpr (MODE == 1) {
      if (tried && !done) sink.rollback();
      if (done) sink.zero_absent(S);
      wave_lds_sync();
      if (lane < S) {
        const uint32_t t = tsl[lane];
        if (t) {
          atomicAdd(&o.tsum[(size_t)lane * o.tile_stride + tile], t);
          tsl[lane] = 0;
        }
      }
    }
    bool ool = MODE == 1;  // the record has an out-of-line list (MODE 1: not tracked, assumed)
    if constexpr (MODE != 1) {
      for (uint32_t k = 0; k < S; ++k) {
        const uint32_t ov = done ? (uint32_t)sink.ord[(size_t)k * sink.ostride] : 0u;
        const uint32_t c = ov ? sink.count_of(k) : 0u;
        ool |= c != 0u && !(c & kCountInline);
        if (done) {
          const size_t at = (size_t)k * B.n + r;
          o.order[at] = (uint16_t)ov;
          o.count[at] = c;
        }
        const uint32_t x = c & ~kCountInline;
        const uint64_t nz = __ballot(x != 0u);
        if (nz) {  // counts of 0/1 (single values): the sum is a popcount of the ballot (scalar)
          const uint32_t t = __ballot(x > 1u) ? wave_sum_u32(x) : (uint32_t)__popcll(nz);
          if (lane == 0) atomicAdd(&o.tsum[(size_t)k * o.tile_stride + tile], t);
        }
        if (spec_on && spec_l[k]) {  // (wave-uniform) speculative row split r; irregular records counted
          // (the row splits of a final placement are implicit for the first 64 slots:
          // tfrg_info.placed_slots; a failed placement has them all rewritten by k_down_gather)
          if (valid && k >= 64u) o.rs[(size_t)k * (B.n + 1) + r] = r;
          const uint64_t irm = __ballot(valid && !deferred && !(done && c == (1u | kCountInline)));
          if (irm && lane == 0) atomicAdd(&o.irr[k], (uint32_t)__popcll(irm));
        }
      }
    }
    crc_list_append(o, r, crc_j, lane);
    // a large record goes to the wave gathers (staged ones from the front of big_list, huge ones
    // from the back) if it has a list k_down_gather does not write: out-of-line or deferred lists, or
    // any list of a record the exact walker takes (C2's single image views and labels need none)
    if (big && !deferred && (!done || ool || nd)) {
      if (v.e - (v.st & ~15ull) <= wave_stage) {
        const uint32_t i = atomicAdd(&o.info[kInfoBig], 1u);
        o.big_list[i] = r;
      } else {
        const uint32_t i = atomicAdd(&o.info[kInfoHuge], 1u);
        o.big_list[B.n - 1u - i] = r;
      }
    }
    wave_lds_sync();  // the stage is rewritten by the next iteration
    PHASE_MARK(p5);
    PHASE_ADD(19, p4, p5);
    PHASE_ADD(20, p0, p5);
  }
}

// The columns a record accepted by the lane kernel wrote, withdrawn before the exact walker redoes it:
// order / count of every slot cleared, the counts taken back from the tile sums, and every present
// slot counted irregular (a speculatively placed value of the record is then re-placed by the scan).
__device__ void withdraw_record(const DevOut& o, uint32_t n, uint32_t n_slots, uint32_t r) {
  for (uint32_t k = 0; k < n_slots; ++k) {
    const size_t at = (size_t)k * n + r;
    const uint32_t c = o.count[at];
    if (o.order[at]) o.order[at] = 0;
    if (!c) continue;
    o.count[at] = 0;
    atomicAdd(&o.irr[k], 1u);
    if (c & ~kCountInline) atomicSub(&o.tsum[(size_t)k * o.tile_stride + (r >> kTileShift)], c & ~kCountInline);
  }
}

// Counts of the deferred packed int64 bodies (BodyDefer). A block holds the rows of one lane-kernel
// wave: 64 consecutive records (one tile), entry j of every row side by side ([block][j][lane]). A
// wave takes a quarter of a block's entry columns, lane l its record's entries one after the other:
// the lanes of one step are 64 records' j-th bodies, usually one slot of one tile, so the tile sum is
// usually one atomic per step. Each body: count_packed over HBM with 8 blocks of 16 bytes in flight
// (one round for most bodies), the count word written. A body that does not count canonically (a
// varint of more than 10 bytes, or one running past the chunk) marks its record kStatusRedo (once)
// and lists it for the exact walker (k_tail_count role 1), which withdraws the record's columns and
// re-walks it.
constexpr int kBodyBlock = 256;
constexpr uint32_t kBodyParts = 4;  // waves per block of rows (kDeferK / kBodyParts columns each)
__global__ __launch_bounds__(kBodyBlock) void k_body_count(DevBatch B, DevOut o) {
  const uint32_t nblk = o.info[kInfoDefer] < o.dq_blocks ? o.info[kInfoDefer] : o.dq_blocks;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t lim = ((B.nbytes + 15) & ~15ull) - 4;
  const uint32_t nw = gridDim.x * (kBodyBlock / 64u);
  for (uint32_t t = blockIdx.x * (kBodyBlock / 64u) + rfl32(threadIdx.x >> 6); t < nblk * kBodyParts; t += nw) {
    const uint32_t blk = t / kBodyParts, j0 = (t % kBodyParts) * (kDeferK / kBodyParts);
    const uint32_t nrow = o.dq_cnt[(size_t)blk * 64u + lane];
    uint32_t jmax = nrow;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      const uint32_t y = (uint32_t)__shfl_xor((int)jmax, m, 64);
      jmax = y > jmax ? y : jmax;
    }
    jmax = rfl32(jmax);
    const uint32_t j1 = j0 + kDeferK / kBodyParts < jmax ? j0 + kDeferK / kBodyParts : jmax;
    for (uint32_t j = j0; j < j1; ++j) {  // (wave-uniform: the reductions below see every lane)
      bool has = j < nrow, ok = true;
      uint32_t r = 0, slot = 0, cnt = 0;
      if (has) {
        const uint4 q = o.dq[((size_t)blk * kDeferK + j) * 64u + lane];
        r = q.x;
        slot = q.y;
        const FastSrcG<false> s{B.bytes, (uint64_t)q.z, q.w, lim};
        ok = count_packed<8>(s, 0u, q.w, cnt);
      }
      if (has && ok) o.count[(size_t)slot * B.n + r] = cnt;
      if (has && !ok && atomicCAS(&o.status[r], TFRG_OK, kStatusRedo) == TFRG_OK) {
        const uint32_t si = atomicAdd(&o.info[kInfoSlow], 1u);
        o.slow_list[si] = r;
      }
      // tile sums: one atomic per run of lanes with the same slot (the rows share one tile)
      bool pend = has && ok && cnt != 0u;
      for (uint64_t m = __ballot(pend); m; m = __ballot(pend)) {
        const int l0 = __builtin_ctzll(m);
        const uint32_t s0 = (uint32_t)__shfl((int)slot, l0, 64), t0 = (uint32_t)__shfl((int)r, l0, 64) >> kTileShift;
        const bool mine = pend && slot == s0 && (r >> kTileShift) == t0;
        const uint32_t sum = wave_sum_u32(mine ? cnt : 0u);
        if (lane == (uint32_t)l0) atomicAdd(&o.tsum[(size_t)s0 * o.tile_stride + t0], sum);
        pend &= !mine;
      }
    }
  }
}

// Exact reference walk (decoder.pyx:107-300 in its own level-by-level error precedence), one lane per
// record of the slow list, reading the record from HBM; also the framing errors and schema misses.
template <int R, bool COMPAT, bool GORD, uint32_t BLK>
__device__ __forceinline__ void role_slow_count(const DevBatch& B, const DevSchema& sc, const DevOut& o,
                                const uint32_t* __restrict__ crc_tab, uint32_t lane_max) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const uint32_t nslow = o.info[kInfoSlow];
  if (blockIdx.x * BLK >= nslow) return;  // block-uniform
  uint32_t* tab = lds;                            // 2048 * R dwords (slice-by-8 set; step4 uses 0..3)
  uint32_t* cnt = lds + 2048 * R;
  const uint32_t S = sc.n_slots;
  uint16_t* ord = reinterpret_cast<uint16_t*>(cnt + (GORD ? 0u : S * BLK));
  for (uint32_t i = threadIdx.x; i < 2048u * R; i += BLK) tab[i] = crc_tab[2048 + i / R];
  __syncthreads();
  const LdsTab<R> T{tab, threadIdx.x & (R - 1)};
  for (uint32_t i = blockIdx.x * BLK + threadIdx.x; i < nslow; i += gridDim.x * BLK) {
    const uint32_t r = o.slow_list[i];
    if (o.status[r] == kStatusRedo) withdraw_record(o, B.n, S, r);  // (a body k_body_count rejected)
    RecView v = rec_view(B, r);
    int64_t aux = 0;
    CountSinkT<!GORD> sink{&sc, &o, dict_ord<!GORD>(o.order + r, ord + threadIdx.x),
                           GORD ? B.n : (uint32_t)BLK, 0, B.n, r, v.p0, false, true};
    if constexpr (!GORD) sink.cnt = (lds_u32*)(cnt + threadIdx.x);
    int status = v.status;
    if (status == TFRG_OK) {
      // (the payload CRC of a large record too: role 2 skips the records of this role)
      frame_verdicts<R, false>(B, v, T, nullptr, 0, true);
      sink.reset();
      Src s;
      s.init(B.bytes, v.p0, v.L);
      status = walk_example<COMPAT>(s, sink, aux);
      if (sink.miss) status = TFRG_ST_SCHEMA_MISS;
      if (status == TFRG_OK && !strict_pass(B, v.verdict, true)) {
        status = TFRG_ERR_CRC;
        aux = v.verdict;
      }
    }
    sink.finalize(status == TFRG_OK);
    record_result(o, r, status, aux, v.verdict);
  }
}

// ------------------------------------------------------------------------------------------------
// Records above lane_max: payload CRC (k_big_crc) and the helpers of their wavefront gathers.
// ------------------------------------------------------------------------------------------------

// Scalar read of a canonical length-delimited field-1 header at `q`: tag 0x0a + length varint of
// <= 3 bytes; sets the body offset/length (body inside the payload) or returns false (bail).
__device__ __forceinline__ bool hdr_0a(const FastSrc& s, uint32_t q, uint32_t& bo, uint32_t& bl) {
  if (q + 2 > s.L) return false;
  const uint32_t w = __builtin_amdgcn_readfirstlane(s.w4(q));
  if ((w & 0xffu) != 0x0au) return false;
  const uint32_t b1 = (w >> 8) & 0xffu, b2 = (w >> 16) & 0xffu, b3 = w >> 24;
  uint32_t h, len;
  if (b1 < 0x80u) {
    h = 2;
    len = b1;
  } else if (b2 < 0x80u) {
    h = 3;
    len = (b1 & 0x7fu) | (b2 << 7);
  } else if (b3 < 0x80u) {
    h = 4;
    len = (b1 & 0x7fu) | ((b2 & 0x7fu) << 7) | (b3 << 14);
  } else {
    return false;
  }
  bo = q + h;
  bl = len;
  return bo <= s.L && len <= s.L - bo;
}

// Streaming payload CRC of the large records (k_tail_count role 2). The lane kernel lists every
// accepted record above lane_max (crc_list_append) with its 1 KiB rounds counted into ONE flat
// round space: list entry i owns the flat rounds [base_i, base_{i+1}); round j of a record,
// counted from its end, is its aligned 16-byte chunks c1 - 64 j - lane. Every wave of the launch
// takes an equal contiguous slice of the flat space, so the large payloads of a batch stream
// through the chip with kCrcDepth rounds of loads in flight per wave whatever the record sizes
// (one record per wave or workgroup left latency chains per record and the load imbalance of
// lognormal sizes). A lane's state advances by x^8192 per round (Horner, A1 tables); a record's
// rounds inside one wave are lane-combined (x^(128 l)) and shifted by x^(8192 jlo) to their place;
// the slices of a record split over waves XOR together in crc_part (CRC-32C is linear, crc32c.h)
// and the wave whose rounds complete the record finishes it.
constexpr int kCrcDepth = 4;  // rounds of loads in flight per wave
[[maybe_unused]] constexpr uint32_t kCstUnshift = 64;     // consts: [0, 64) x^(128 l), [64, 80) x^(-8z),
[[maybe_unused]] constexpr uint32_t kCstRoundPow = 96;    // [96, 128) x^(8192 * 2^k)
constexpr uint32_t kPowTabOff = 26624;   // crc_tab: [24][4][256] multiply by x^(8192 * 2^k) (split-slice shifts)
constexpr uint32_t kNumCst = 128;

// U(0, 16-byte chunk at q) of the payload [a, b): bytes outside zeroed, the first 4 payload bytes
// inverted (the ~0 initial state)
template <class TabT>
__device__ __forceinline__ uint32_t chunk_u(uint4 w, uint64_t q, uint64_t a, uint64_t b, const TabT& T) {
  uint32_t ws[4] = {w.x, w.y, w.z, w.w};
  if (q < a + 4 || q + 16 > b) {
    // chunk-relative byte bounds in [0, 16]: keep [lo, hi), invert [lo, li) (the payload's first 4)
    const int64_t la = (int64_t)(a - q), lb = (int64_t)(b - q);
    const uint32_t lo = la <= 0 ? 0u : (la >= 16 ? 16u : (uint32_t)la);
    const uint32_t hi = lb <= 0 ? 0u : (lb >= 16 ? 16u : (uint32_t)lb);
    const uint32_t li = la + 4 <= 0 ? 0u : (la + 4 >= 16 ? 16u : (uint32_t)(la + 4));  // end of the first 4
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2) {
      auto upto = [](uint32_t x, int k) {  // bytes of word k below chunk byte x
        const uint32_t n = x <= 4u * k ? 0u : (x - 4u * k >= 4u ? 4u : x - 4u * k);
        return n >= 4u ? 0xffffffffu : (1u << (8u * n)) - 1u;
      };
      const uint32_t below_lo = upto(lo, k2);
      const uint32_t keep = upto(hi, k2) & ~below_lo;
      const uint32_t inv = upto(li, k2) & ~below_lo & keep;
      ws[k2] = (ws[k2] & keep) ^ inv;
    }
  }
  // slice-by-16: byte i of the chunk is followed by 15 - i bytes (T holds the 16 tables), so the
  // 16 lookups are independent (no serial step chain per chunk)
  uint32_t r0 = 0, r1 = 0;
#pragma unroll
  for (int k2 = 0; k2 < 4; ++k2) {
    const uint32_t x = ws[k2];
    r0 ^= T.at4(15 - 4 * k2, byte_x4<0>(x)) ^ T.at4(14 - 4 * k2, byte_x4<1>(x));
    r1 ^= T.at4(13 - 4 * k2, byte_x4<2>(x)) ^ T.at4(12 - 4 * k2, byte_x4<3>(x));
  }
  return r0 ^ r1;
}

// The masking of chunk_u alone: bytes outside the payload [a, b) zeroed, its first 4 bytes inverted.
__device__ __forceinline__ uint4 chunk_mask(uint4 w, uint64_t q, uint64_t a, uint64_t b) {
  uint32_t ws[4] = {w.x, w.y, w.z, w.w};
  const int64_t la = (int64_t)(a - q), lb = (int64_t)(b - q);
  const uint32_t lo = la <= 0 ? 0u : (la >= 16 ? 16u : (uint32_t)la);
  const uint32_t hi = lb <= 0 ? 0u : (lb >= 16 ? 16u : (uint32_t)lb);
  const uint32_t li = la + 4 <= 0 ? 0u : (la + 4 >= 16 ? 16u : (uint32_t)(la + 4));
#pragma unroll
  for (int k2 = 0; k2 < 4; ++k2) {
    auto upto = [](uint32_t x, int k) {
      const uint32_t n = x <= 4u * k ? 0u : (x - 4u * k >= 4u ? 4u : x - 4u * k);
      return n >= 4u ? 0xffffffffu : (1u << (8u * n)) - 1u;
    };
    const uint32_t below_lo = upto(lo, k2);
    const uint32_t keep = upto(hi, k2) & ~below_lo;
    const uint32_t inv = upto(li, k2) & ~below_lo & keep;
    ws[k2] = (ws[k2] & keep) ^ inv;
  }
  return make_uint4(ws[0], ws[1], ws[2], ws[3]);
}

// x << 2 with an SDWA byte select of x: a table byte offset in one VALU (the multiply-table lookups)
#define TFRG_SDWA(o, two, src, k) "v_lshlrev_b32_sdwa %" #o ", %" #two ", %" #src " dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_" #k "\n\t"

// Bank-conflict-free slice-by-16 (the streaming CRC's LDS layout): the 16 tables are laid out in
// rows of 64 dwords, row e = entry e, column c holding T[(c + 1) & 15][e] (c < 47). Lane l reads its
// chunk ROTATED by rho = l & 15 bytes: at instruction t its byte t is chunk byte (t + rho) & 15, whose
// table 15 - ((t + rho) & 15) sits in column 15 - rho + 16 h + 15 - t, h = (l >> 4) & 1. The bank
// ((a / 4) mod 32) is then 15 - rho + 16 h + 15 - t mod 32: the 32 lanes of a ds_read_b32 group hit 32
// different banks whatever the data (random-byte lookups into one shared table conflicted ~3x,
// profiles/r02/pmc_c2_k_tail_count.json). The address (e << 8) | lane base is ONE v_perm_b32; the
// table base and the column's t part are the instruction's immediate offset.
constexpr uint32_t kRotTabOff = 12288;  // byte offset of the rotated table in LDS (after A1, A2, A4)
struct CrcRot {
  uint64_t m1, m2;  // lanes whose rho has bit 2 / bit 3 set (dword rotation by 1 / 2)
  uint32_t s;       // rho & 3 (byte funnel)
  uint32_t basel;   // 4 * (15 - rho + 16 h)
};
__device__ __forceinline__ CrcRot crc_rot_init(uint32_t lane) {
  const uint32_t rho = lane & 15u;
  CrcRot r;
  r.m1 = __ballot((rho >> 2) & 1u);
  r.m2 = __ballot((rho >> 3) & 1u);
  r.s = rho & 3u;
  r.basel = 4u * (15u - rho + 16u * ((lane >> 4) & 1u));
  return r;
}
__device__ __forceinline__ uint32_t crc_perm(uint32_t x, uint32_t basel, uint32_t sel) {
  return __builtin_amdgcn_perm(x, basel, sel);
}
__device__ __forceinline__ uint32_t chunk_rot(uint4 w, const CrcRot& R, uint32_t lane) {
  const uint64_t bit = 1ull << lane;
  const bool b2 = (R.m2 & bit) != 0, b1 = (R.m1 & bit) != 0;
  // dword rotation by q = rho >> 2: E[i] = D[(i + q) & 3]
  uint32_t e0 = b2 ? w.z : w.x, e1 = b2 ? w.w : w.y, e2 = b2 ? w.x : w.z, e3 = b2 ? w.y : w.w;
  const uint32_t f0 = b1 ? e1 : e0, f1 = b1 ? e2 : e1, f2 = b1 ? e3 : e2, f3 = b1 ? e0 : e3;
  // byte funnel by rho & 3: R[i] = bytes (4i + rho ..) of the chunk
  const uint32_t r0 = __builtin_amdgcn_alignbyte(f1, f0, R.s), r1 = __builtin_amdgcn_alignbyte(f2, f1, R.s);
  const uint32_t r2 = __builtin_amdgcn_alignbyte(f3, f2, R.s), r3 = __builtin_amdgcn_alignbyte(f0, f3, R.s);
  // v_perm selectors: byte 0 from the lane base (src1 byte 0), byte 1 = byte k of x (src0), rest 0
  constexpr uint32_t S0 = 0x0c0c0400u, S1 = 0x0c0c0500u, S2 = 0x0c0c0600u, S3 = 0x0c0c0700u;
  const uint32_t bl = R.basel;
  uint32_t v[16];
  v[0] = crc_perm(r0, bl, S0); v[1] = crc_perm(r0, bl, S1); v[2] = crc_perm(r0, bl, S2); v[3] = crc_perm(r0, bl, S3);
  v[4] = crc_perm(r1, bl, S0); v[5] = crc_perm(r1, bl, S1); v[6] = crc_perm(r1, bl, S2); v[7] = crc_perm(r1, bl, S3);
  v[8] = crc_perm(r2, bl, S0); v[9] = crc_perm(r2, bl, S1); v[10] = crc_perm(r2, bl, S2); v[11] = crc_perm(r2, bl, S3);
  v[12] = crc_perm(r3, bl, S0); v[13] = crc_perm(r3, bl, S1); v[14] = crc_perm(r3, bl, S2); v[15] = crc_perm(r3, bl, S3);
  // all 16 reads issued before the one wait; instruction t's immediate = table base + 4 (15 - t)
  asm volatile(
      "ds_read_b32 %0, %0 offset:12348\n\t"
      "ds_read_b32 %1, %1 offset:12344\n\t"
      "ds_read_b32 %2, %2 offset:12340\n\t"
      "ds_read_b32 %3, %3 offset:12336\n\t"
      "ds_read_b32 %4, %4 offset:12332\n\t"
      "ds_read_b32 %5, %5 offset:12328\n\t"
      "ds_read_b32 %6, %6 offset:12324\n\t"
      "ds_read_b32 %7, %7 offset:12320\n\t"
      "ds_read_b32 %8, %8 offset:12316\n\t"
      "ds_read_b32 %9, %9 offset:12312\n\t"
      "ds_read_b32 %10, %10 offset:12308\n\t"
      "ds_read_b32 %11, %11 offset:12304\n\t"
      "ds_read_b32 %12, %12 offset:12300\n\t"
      "ds_read_b32 %13, %13 offset:12296\n\t"
      "ds_read_b32 %14, %14 offset:12292\n\t"
      "ds_read_b32 %15, %15 offset:12288\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]),
        "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]), "+v"(v[14]), "+v"(v[15]));
  return xor3(xor3(xor3(v[0], v[1], v[2]), xor3(v[3], v[4], v[5]), xor3(v[6], v[7], v[8])),
              xor3(v[9], v[10], v[11]), xor3(v[12], v[13], v[14])) ^ v[15];
}
// table j's entry at byte offset bx4 = 4 * index, read from the rotated layout (masked edge chunks)
struct RotTabView {
  const uint8_t* l;  // LDS base
  __device__ __forceinline__ uint32_t at4(uint32_t j, uint32_t bx4) const {
    return *reinterpret_cast<const uint32_t*>(l + kRotTabOff + (bx4 << 6) + 4u * ((j + 15u) & 15u));
  }
};

__device__ __forceinline__ uint32_t mul_tab(const uint32_t* M, uint32_t S) {
  return M[S & 0xffu] ^ M[256 + ((S >> 8) & 0xffu)] ^ M[512 + ((S >> 16) & 0xffu)] ^ M[768 + (S >> 24)];
}

// mul_tab of the x^8192 table A1 at LDS byte 0 (before the rotated slice-by-16 table), with SDWA
// byte offsets and immediate table offsets: 4 VALU + 4 LDS reads + 2 XOR
#define TFRG_MUL_LDS(NAME, O0, O1, O2, O3)                                                        \
  __device__ __forceinline__ uint32_t NAME(uint32_t S) {                                          \
    uint32_t m0, m1, m2, m3;                                                                      \
    const uint32_t two = 2u;                                                                      \
    asm volatile(TFRG_SDWA(0, 4, 5, 0) TFRG_SDWA(1, 4, 5, 1) TFRG_SDWA(2, 4, 5, 2) TFRG_SDWA(3, 4, 5, 3) \
                 "ds_read_b32 %0, %0 offset:" #O0 "\n\t"                                        \
                 "ds_read_b32 %1, %1 offset:" #O1 "\n\t"                                        \
                 "ds_read_b32 %2, %2 offset:" #O2 "\n\t"                                        \
                 "ds_read_b32 %3, %3 offset:" #O3 "\n\t"                                        \
                 "s_waitcnt lgkmcnt(0)"                                                           \
                 : "=&v"(m0), "=&v"(m1), "=&v"(m2), "=&v"(m3)                                     \
                 : "v"(two), "v"(S));                                                             \
    return xor3(m0, m1, m2) ^ m3;                                                                 \
  }
// (x) x^16384 and x^32768 at LDS bytes 4096 and 8192: a group of 4 rounds of one record is summed as
// S A^4 + (rc0 A + rc1) A^2 + (rc2 A + rc3): two dependent LDS round trips instead of four
TFRG_MUL_LDS(mul_a2_lds, 4096, 5120, 6144, 7168)
TFRG_MUL_LDS(mul_a4_lds, 8192, 9216, 10240, 11264)

__device__ __forceinline__ uint32_t mul_a1_lds(uint32_t S) {
  uint32_t m0, m1, m2, m3;
  const uint32_t two = 2u;
  asm volatile(
      TFRG_SDWA(0, 4, 5, 0) TFRG_SDWA(1, 4, 5, 1) TFRG_SDWA(2, 4, 5, 2) TFRG_SDWA(3, 4, 5, 3)
      "ds_read_b32 %0, %0\n\t"
      "ds_read_b32 %1, %1 offset:1024\n\t"
      "ds_read_b32 %2, %2 offset:2048\n\t"
      "ds_read_b32 %3, %3 offset:3072\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(m0), "=&v"(m1), "=&v"(m2), "=&v"(m3)
      : "v"(two), "v"(S));
  return xor3(m0, m1, m2) ^ m3;
}

// TFRG_FLAG_STRICT_CRC, payload CRC of a record above lane_max failed: the record becomes an error
// (status TFRG_ERR_CRC, aux = verdict) and its counts are withdrawn from the columns and the tile
// sums before k_spine scans them. `t` indexes the slots with stride `nt` (the calling wave / group).
__device__ void strict_reject(const DevOut& o, uint32_t n, uint32_t n_slots, uint32_t r, uint32_t verdict,
                              uint32_t t, uint32_t nt) {
  if (__hip_atomic_load(&o.status[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != TFRG_OK) return;
  for (uint32_t k = t; k < n_slots; k += nt) {
    const size_t at = (size_t)k * n + r;
    const uint32_t c = o.count[at];
    if (o.order[at]) o.order[at] = 0;  // (present slots with empty lists have count 0)
    if (!c) continue;
    o.count[at] = 0;
    atomicAdd(&o.irr[k], 1u);  // (a speculatively placed value is withdrawn: k_down_gather places the slot)
    if (c & ~kCountInline) atomicSub(&o.tsum[(size_t)k * o.tile_stride + (r >> kTileShift)], c & ~kCountInline);
  }
  if (t == 0) {
    o.status[r] = TFRG_ERR_CRC;
    o.aux[r] = verdict;
    atomicAdd(&o.info[kInfoErrors], 1u);
    atomicMax(&o.info[kInfoFirstError], ~r);  // stored inverted: zero-initialised with the rest
  }
}

__device__ __forceinline__ uint64_t rl64(uint64_t x, uint32_t k) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), (int)k) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, (int)k);
}
__device__ __forceinline__ uint32_t rl32(uint32_t x, uint32_t k) {
  return (uint32_t)__builtin_amdgcn_readlane((int)x, (int)k);
}

// The streaming-CRC window: lane k < 63 describes list entry win0 + k, lane 63 holds the next
// window's first flat round (the bound of this one). Three 64-bit values per lane; everything else
// about an entry is derived in scalar registers (crc_ent) or loaded at its flush: the fewer VGPRs,
// the more group loads in flight without spills.
struct CrcWin {
  uint64_t base;  // first flat round (entry k's rounds: [base[k], base[k + 1]))
  uint64_t a, b;  // payload [a, b)
  uint32_t e32;   // E of entry k (crc_ent) mod 2^32: the byte offset of its chunk for flat round R and
                  // lane l is (e32 + 64 R - l) << 4 (batches are < 4 GiB)
};

__device__ __forceinline__ CrcWin crc_win_load(const DevBatch& B, const DevOut& o, uint32_t win0, uint32_t nrec,
                                               uint64_t TR, uint32_t lane) {
  CrcWin w{};
  const uint32_t idx = win0 + lane;
  w.base = idx < nrec ? o.crc_base[idx] : TR;
  if (idx < nrec && lane < 63u) {
    const RecView v = rec_view(B, o.crc_rec[idx]);
    w.a = v.p0;
    w.b = v.e - 4;
  }
  {  // E = c1 - 64 (J - 1) - 64 base[k] = c1 - 64 base[k + 1] + 64
    const uint32_t nb = (uint32_t)__shfl_down((int)(uint32_t)w.base, 1, 64);
    w.e32 = (uint32_t)((w.b - 1u) >> 4) - 64u * nb + 64u;
  }
  // the window's loads retired here: the group loads issued after it then carry no false wait on
  // them (a merged loop-header state otherwise drains vmcnt before every group)
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  return w;
}

// (scalar) window entry k: first round, round count J, chunk of its round R for lane l (E + 64 R - l;
// the rounds end at the payload's last chunk c1), first payload chunk c0
struct CrcEnt {
  uint64_t bas, J, E, c0;
};
__device__ __forceinline__ CrcEnt crc_ent(const CrcWin& w, uint32_t k) {
  CrcEnt e;
  e.bas = rl64(w.base, k);
  e.J = rl64(w.base, k + 1u) - e.bas;
  const uint64_t c1 = (rl64(w.b, k) - 1u) >> 4;
  e.E = c1 - 64ull * (e.J - 1u) - 64ull * e.bas;
  e.c0 = rl64(w.a, k) >> 4;
  return e;
}

// Per-record flushes of the streaming CRC, deferred and done 64 at a time, one per lane. A wave
// flushes a record each time its slice leaves one (C3: ~32 records per wave): the x^(8192 jlo)
// shift of a split slice, the 64-bit compare-and-swap that combines the slices of a record, the
// load of its stored CRC and the verdict OR are each a round trip to L2 or HBM, and done at once by
// the wave they cost ~12 us of C2's 98 us CRC and ~70 us of C3's 390 (flush-less timing builds).
// Queued here instead (the wave-uniform part, the lane combine of the Horner sums, at once: it needs
// the lanes' sums), the rest by lane i for the i-th queued record when 64 are pending and at the end
// of the wave's slice: all the round trips of 64 records in flight together.
struct CrcFlushQ {
  uint32_t t, idx, jlo, jtop, J;  // lane i: queued record i (the combined slice value, list entry, rounds)
  uint32_t n = 0;                 // (wave-uniform) records queued
};

// lane < q.n: finish queued record `lane` (see crc_flush_push)
__device__ void crc_flush_run(CrcFlushQ& q, const uint8_t* lbase, const uint32_t* __restrict__ ptab,
                              const DevBatch& B, const DevOut& o, uint32_t n_slots, uint32_t lane) {
  if (lane < q.n) {
    uint32_t t = q.t;
    const uint32_t idx = q.idx, jlo = q.jlo, jtop = q.jtop, J = q.J;
    for (uint32_t kb = 0, jj = jlo; jj; ++kb, jj >>= 1) {  // x x^(8192 jlo): one table multiply per set bit
      if (!(jj & 1u)) continue;
      const uint32_t* M = ptab + (size_t)kb * 1024u;
      t = M[t & 0xffu] ^ M[256u + ((t >> 8) & 0xffu)] ^ M[512u + ((t >> 16) & 0xffu)] ^ M[768u + (t >> 24)];
    }
    bool complete = true;
    if (jlo != 0u || jtop != J - 1u) {  // a slice of a record split over waves
      // (rounds done << 32 | XOR of the slices) updated in ONE 64-bit compare-and-swap: the wave that
      // completes the rounds sees every other slice in the value it replaced, with no fence (an
      // agent-scope fence per slice wrote back and invalidated L2 under the streaming loads)
      const uint32_t n_r = jtop - jlo + 1u;
      unsigned long long* p = reinterpret_cast<unsigned long long*>(o.crc_part + idx);
      unsigned long long cur = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (;;) {
        const unsigned long long nv = ((cur >> 32) + n_r) << 32 | (uint32_t)((uint32_t)cur ^ t);
        const unsigned long long prev = atomicCAS(p, cur, nv);
        if (prev == cur) break;
        cur = prev;
      }
      complete = (uint32_t)(cur >> 32) + n_r == J;  // (else another wave finishes the record)
      t ^= (uint32_t)cur;
    }
    if (complete) {
      const uint32_t r = o.crc_rec[idx];
      const uint64_t b = rec_view(B, r).e - 4;
      const uint32_t verdict = o.verdict[r];
      const uint32_t z = (uint32_t)(16ull * (((b - 1) >> 4) + 1ull) - b);  // zero bytes padding the last chunk
      // t is the state after the payload and z zero bytes: the stored CRC's state is advanced by the
      // same z zero bytes through the slicing tables of the rotated layout and compared with t
      const uint32_t um = load_u32_unaligned(B.bytes, b) - kCrcMaskDelta;
      uint32_t v = ~((um << 15) | (um >> 17));  // ~crc_mask^-1(stored)
      auto rt = [&](uint32_t col, uint32_t e) {
        return *reinterpret_cast<const uint32_t*>(lbase + kRotTabOff + (e << 8) + 4u * col);
      };
      uint32_t zz = z;
      for (; zz >= 4u; zz -= 4u)  // 4 zero bytes: slice-by-4 (tables 3, 2, 1, 0 in columns 2, 1, 0, 15)
        v = xor3(rt(2u, v & 0xffu), rt(1u, (v >> 8) & 0xffu), rt(0u, (v >> 16) & 0xffu)) ^ rt(15u, v >> 24);
      for (; zz; --zz) v = (v >> 8) ^ rt(15u, v & 0xffu);
      if (v == t) {
        // one atomic OR on the byte's aligned word: a record k_body_count sent back to the exact walker
        // (role 1 of the same launch) may have its verdict byte written by role 1 at the same time
        atomicOr(reinterpret_cast<uint32_t*>(o.verdict + (r & ~3u)), (uint32_t)TFRG_V_DATA_CRC << (8u * (r & 3u)));
      } else if (B.flags & kFlagStrictCrc) {
        strict_reject(o, B.n, n_slots, r, verdict, 0u, 1u);
      }
    }
  }
  q.n = 0;
}

// the rounds [Rf, Rl] of window entry k, Horner sum S per lane: combined over the lanes and queued
// (crc_flush_run when 64 are pending)
__device__ __forceinline__ void crc_flush_push(CrcFlushQ& q, const uint8_t* lbase, const uint32_t* __restrict__ ptab,
                                               const DevBatch& B, const DevOut& o, const CrcWin& w, uint32_t win0,
                                               uint32_t k, uint64_t Rf, uint64_t Rl, uint32_t S, const uint32_t* cst,
                                               uint32_t n_slots, uint32_t lane) {
  const uint64_t bas = rl64(w.base, k);
  const uint32_t J = (uint32_t)(rl64(w.base, k + 1u) - bas);
  const uint32_t jtop = J - 1u - (uint32_t)(Rf - bas), jlo = J - 1u - (uint32_t)(Rl - bas);
  const uint32_t t = wave_xor_u32(gf_mul(S, cst[lane]));
  if (lane == q.n) {
    q.t = t;
    q.idx = win0 + k;
    q.jlo = jlo;
    q.jtop = jtop;
    q.J = J;
  }
  if (++q.n == 64u) crc_flush_run(q, lbase, ptab, B, o, n_slots, lane);
}

// (wb: the launch's first wb workgroups walk large records instead, role_big_walk)
template <uint32_t BLK>
__device__ __forceinline__ void role_crc_stream(const DevBatch& B, const DevOut& o, const uint32_t* __restrict__ crc_tab,
                                const uint32_t* __restrict__ consts, uint32_t n_slots, uint32_t wb) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  if (B.flags & (kFlagPayloadOnly | kFlagNoCrc)) return;
  const uint64_t ctr = *reinterpret_cast<const uint64_t*>(o.info + kInfoCrcCtr);
  const uint32_t nrec = (uint32_t)(ctr >> kCrcIdxShift);
  const uint64_t TR = ctr & kCrcRoundMask;
  if (!nrec) return;  // (grid-uniform)
  uint32_t* A1 = lds;           // [4][256] (x) x^8192, then (x) x^16384, (x) x^32768
  uint32_t* rot = lds + 3072;   // [256][64] rotated slice-by-16 (chunk_rot)
  uint32_t* cst = lds + 19456;  // [kNumCst]
  // the 77 KiB of tables are loaded into registers first and written to LDS only after this wave's
  // search for its first list entry and its window load: those dependent HBM round trips overlap
  // the table loads instead of following them (every wave of the launch starts with them)
  static_assert(3072u % BLK == 0u && 4096u % BLK == 0u && kNumCst <= BLK, "table copy shape");
  uint32_t ta[3072u / BLK];
  uint4 tr[4096u / BLK];
#pragma unroll
  for (uint32_t j = 0; j < 3072u / BLK; ++j) {
    const uint32_t i = j * BLK + threadIdx.x;
    ta[j] = i < 1024u ? crc_tab[1024 + i] : crc_tab[24576 + (i - 1024u)];
  }
#pragma unroll
  for (uint32_t j = 0; j < 4096u / BLK; ++j) tr[j] = reinterpret_cast<const uint4*>(crc_tab + 8192)[j * BLK + threadIdx.x];
  const uint32_t tc = threadIdx.x < kNumCst ? consts[threadIdx.x] : 0u;
  const RotTabView T{reinterpret_cast<const uint8_t*>(lds)};
  const bool tab_at0 = (uint32_t)(uintptr_t)lds == 0u;  // (the asm chunk path addresses LDS 0)
  // the batch's readable bytes (round_up(nbytes, 16), at most 2^32 - 1: batches are < 4 GiB) as a
  // buffer resource
  const uint64_t readable = (B.nbytes + 15u) & ~15ull;
  const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(B.bytes), (short)0, (int)(uint32_t)(readable < 0xffffffffull ? readable : 0xffffffffull),
      0x00020000);
  const uint32_t lane = threadIdx.x & 63u, wib = rfl32(threadIdx.x >> 6);
  const CrcRot RR = crc_rot_init(lane);
  const uint64_t W = (uint64_t)(gridDim.x - wb) * (BLK / 64), wv = (uint64_t)(blockIdx.x - wb) * (BLK / 64) + wib;
  const uint64_t R0 = TR * wv / W, R1 = TR * (wv + 1) / W;
  const bool work = R0 < R1;  // (wave-uniform)
  PHASE_MARK(q0);
  // the list entry holding flat round R0: 64-ary search over the ascending bases
  uint32_t lo = 0, hi = work ? nrec : 1u;  // base[lo] <= R0 < base[hi] (base[nrec] = TR)
  while (hi - lo > 1u) {
    const uint32_t step = (hi - lo + 63u) >> 6;
    const uint32_t k = lo + lane * step;
    const uint64_t bk = k < hi ? o.crc_base[k] : ~0ull;
    lo = rfl32(lo + ((uint32_t)__popcll(__ballot(bk <= R0)) - 1u) * step);
    hi = rfl32(lo + step < hi ? lo + step : hi);
  }
  uint32_t win0 = lo;
  CrcWin w{};
  if (work) w = crc_win_load(B, o, win0, nrec, TR, lane);
#pragma unroll
  for (uint32_t j = 0; j < 3072u / BLK; ++j) A1[j * BLK + threadIdx.x] = ta[j];
#pragma unroll
  for (uint32_t j = 0; j < 4096u / BLK; ++j) reinterpret_cast<uint4*>(rot)[j * BLK + threadIdx.x] = tr[j];
  if (threadIdx.x < kNumCst) cst[threadIdx.x] = tc;
  __syncthreads();
  if (!work) return;  // (no barrier follows)
  uint64_t lim = rl64(w.base, 63);
  lim = lim < R1 ? lim : R1;
  PHASE_MARK(q1);
  PHASE_ADD(21, q0, q1);
  int cur = -1;  // window entry of the open slice
  CrcFlushQ fq;  // records whose slices this wave finished, flushed 64 at a time
  uint64_t Rf = 0;
  uint32_t S = 0;
  // Groups of kCrcDepth rounds, double-buffered: the loads of group k+1 are in flight while group k
  // is summed (a group never crosses the window; the pipeline drains at a window change).
  struct Grp {
    uint4 wd[kCrcDepth];
    uint64_t rd[kCrcDepth];  // (scalar) flat round of load d
    uint32_t kd[kCrcDepth];  // (scalar) its window entry
    uint32_t n;              // rounds in the group (0: none before the window bound)
    uint64_t r0;
  };
  auto issue = [&](Grp& g, uint64_t Rs) {
    g.r0 = Rs;
    g.n = Rs < lim ? (uint32_t)(lim - Rs < (uint64_t)kCrcDepth ? lim - Rs : (uint64_t)kCrcDepth) : 0u;
    if (!g.n) return;
    const uint64_t rl = Rs + g.n - 1u;
    const uint32_t k0 = (uint32_t)__popcll(__ballot(w.base <= Rs)) - 1u;
    const uint32_t kl = (uint32_t)__popcll(__ballot(w.base <= rl)) - 1u;
    // Chunk loads through a buffer resource over the batch with 32-bit offsets: a chunk before the
    // batch (a negative offset, i.e. a huge one) reads zeros, a chunk of the previous record is
    // read as it is; both occur only in a record's edge rounds, whose masked path (process) never
    // uses those lanes' bytes. Loads past the group's rounds re-read later bytes and are unused.
    if (k0 == kl) {  // (scalar) the whole group inside one record: its entry once
      const uint32_t vo = (rl32(w.e32, k0) + 64u * (uint32_t)Rs - lane) << 4;
#pragma unroll
      for (int d = 0; d < kCrcDepth; ++d) {  // every load of the group in flight before any use
        g.rd[d] = Rs + ((uint32_t)d < g.n ? (uint32_t)d : g.n - 1u);
        g.kd[d] = k0;
        g.wd[d] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(brs, vo + 1024u * d, 0, 0));
      }
      return;
    }
#pragma unroll
    for (int d = 0; d < kCrcDepth; ++d) {  // every load of the group in flight before any use
      g.rd[d] = Rs + ((uint32_t)d < g.n ? (uint32_t)d : g.n - 1u);
      g.kd[d] = (uint32_t)__popcll(__ballot(w.base <= g.rd[d])) - 1u;
      const uint32_t vo = (rl32(w.e32, g.kd[d]) + 64u * (uint32_t)g.rd[d] - lane) << 4;
      g.wd[d] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(brs, vo, 0, 0));
    }
  };
  auto process = [&](const Grp& g) {
    // chunk sums of the whole group, unconditionally (a conditional use lets the compiler sink each
    // load to it: one round trip per round); only the edge rounds (scalar test) take the masked path
    uint32_t rc[kCrcDepth];
    // (scalar) a round that needs masks in the group: a record's first two rounds (its first 4 payload
    // bytes, inverted, may run into the chunk after a's: that chunk opens the second round when the
    // first holds only a's chunk) and its last round
    bool edge = false;
    if (g.kd[0] == g.kd[kCrcDepth - 1]) {  // (scalar) one record: its first two rounds or its last
      const uint64_t bas = rl64(w.base, g.kd[0]);
      edge = g.r0 <= bas + 1u || g.r0 + g.n >= rl64(w.base, g.kd[0] + 1u);
    } else {
#pragma unroll
      for (int d = 0; d < kCrcDepth; ++d) {
        const uint64_t bas = rl64(w.base, g.kd[d]);
        edge |= g.rd[d] <= bas + 1u || g.rd[d] == rl64(w.base, g.kd[d] + 1u) - 1u;
      }
    }
    if (!edge && tab_at0) {  // interior group: one LDS round trip per chunk
#pragma unroll
      for (int d = 0; d < kCrcDepth; ++d) rc[d] = chunk_rot(g.wd[d], RR, lane);
    } else if (!edge) {
#pragma unroll
      for (int d = 0; d < kCrcDepth; ++d) rc[d] = chunk_u(g.wd[d], 64, 0, ~0ull, T);
    } else if (tab_at0 && g.kd[0] == g.kd[kCrcDepth - 1]) {  // edge rounds of one record: its entry once
      const CrcEnt e = crc_ent(w, g.kd[0]);
      const uint64_t a = rl64(w.a, g.kd[0]), b = rl64(w.b, g.kd[0]);
#pragma unroll
      for (int d = 0; d < kCrcDepth; ++d) {
        uint4 x = g.wd[d];
        if (g.rd[d] <= e.bas + 1u || g.rd[d] == e.bas + e.J - 1u) {
          const uint64_t ch = e.E + 64ull * g.rd[d] - lane;
          x = (int64_t)ch >= (int64_t)e.c0 ? chunk_mask(x, ch << 4, a, b) : make_uint4(0, 0, 0, 0);
        }
        rc[d] = chunk_rot(x, RR, lane);
      }
    } else if (tab_at0) {  // edge rounds: masked chunks, the same conflict-free lookups
#pragma unroll
      for (int d = 0; d < kCrcDepth; ++d) {
        const CrcEnt e = crc_ent(w, g.kd[d]);
        uint4 x = g.wd[d];
        if (g.rd[d] <= e.bas + 1u || g.rd[d] == e.bas + e.J - 1u) {
          const uint64_t ch = e.E + 64ull * g.rd[d] - lane;
          const uint64_t a = rl64(w.a, g.kd[d]), b = rl64(w.b, g.kd[d]);
          x = (int64_t)ch >= (int64_t)e.c0 ? chunk_mask(x, ch << 4, a, b) : make_uint4(0, 0, 0, 0);
        }
        rc[d] = chunk_rot(x, RR, lane);
      }
    } else {
#pragma unroll
      for (int d = 0; d < kCrcDepth; ++d) {
        const CrcEnt e = crc_ent(w, g.kd[d]);
        if (g.rd[d] <= e.bas + 1u || g.rd[d] == e.bas + e.J - 1u) {
          const uint64_t ch = e.E + 64ull * g.rd[d] - lane;
          const uint64_t a = rl64(w.a, g.kd[d]), b = rl64(w.b, g.kd[d]);
          rc[d] = (int64_t)ch >= (int64_t)e.c0 ? chunk_u(g.wd[d], ch << 4, a, b, T) : 0u;
        } else {
          rc[d] = chunk_u(g.wd[d], 64, 0, ~0ull, T);  // (interior: no masks)
        }
      }
    }
    static_assert(kCrcDepth == 4, "the split Horner sum below is spelled out for 4 rounds");
    if (tab_at0 && g.n == 4u && (int)g.kd[0] == cur && g.kd[3] == g.kd[0]) {  // (scalar) whole group, open record
      const uint32_t a = mul_a1_lds(rc[0]) ^ rc[1], b = mul_a1_lds(rc[2]) ^ rc[3];
      S = mul_a4_lds(S) ^ mul_a2_lds(a) ^ b;
      return;
    }
    // the group one record at a time: a record change ends the pass at `stop` (one flush site)
    for (uint32_t d0 = 0;;) {
      uint32_t stop = g.n;
      int next = cur;
#pragma unroll
      for (int d = 0; d < kCrcDepth; ++d) {
        if ((uint32_t)d < d0 || (uint32_t)d >= stop) continue;  // (wave-uniform)
        if ((int)g.kd[d] != cur) {
          stop = (uint32_t)d;
          next = (int)g.kd[d];
          continue;
        }
        S = (tab_at0 ? mul_a1_lds(S) : mul_tab(A1, S)) ^ rc[d];
      }
      if (stop == g.n) break;
      if (cur >= 0) crc_flush_push(fq, reinterpret_cast<const uint8_t*>(lds), crc_tab + kPowTabOff, B, o, w, win0, (uint32_t)cur, Rf, g.r0 + stop - 1, S, cst, n_slots, lane);
      cur = next;
      Rf = g.r0 + stop;
      S = 0;
      d0 = stop;
    }
  };
  uint64_t R = R0;
  while (R < R1) {
    if (R >= lim) {  // next window (R is its first entry's first round)
      if (cur >= 0) crc_flush_push(fq, reinterpret_cast<const uint8_t*>(lds), crc_tab + kPowTabOff, B, o, w, win0, (uint32_t)cur, Rf, R - 1, S, cst, n_slots, lane);
      cur = -1;
      win0 += 63u;
      w = crc_win_load(B, o, win0, nrec, TR, lane);
      lim = rl64(w.base, 63);
      lim = lim < R1 ? lim : R1;
      continue;
    }
    Grp ga, gb;
    issue(ga, R);
    R += ga.n;
    for (;;) {
      issue(gb, R);
      R += gb.n;
      process(ga);
      if (!gb.n) break;
      issue(ga, R);
      R += ga.n;
      process(gb);
      if (!ga.n) break;
    }
  }
  if (cur >= 0) crc_flush_push(fq, reinterpret_cast<const uint8_t*>(lds), crc_tab + kPowTabOff, B, o, w, win0, (uint32_t)cur, Rf, R1 - 1, S, cst, n_slots, lane);
  if (fq.n) crc_flush_run(fq, reinterpret_cast<const uint8_t*>(lds), crc_tab + kPowTabOff, B, o, n_slots, lane);
  PHASE_MARK(q9);
  PHASE_ADD(25, q0, q9);
}

// The exception paths before the row-split scan in ONE launch (usually both empty: a workgroup leaves
// at once when it has nothing to do): the exact walker for the slow list (role 1), then the streaming
// payload CRC of the listed large records (role 2). The lane kernel lists only records it accepted,
// but a listed record whose deferred packed body k_body_count rejected (kStatusRedo) is on role 1's
// list too: role 2 then sets its DATA_CRC bit with an atomic OR on the verdict word (role 1 writes the
// whole byte, with the same bit, at any time of the launch), and its strict rejection applies only to
// a status still TFRG_OK (strict_reject), i.e. never to role 1's records.
// (Role 2 as its own kernel at 5 instead of 4 waves per SIMD measured the same on C2: 0.129 vs 0.130
// ms; its own launch cost every batch ~6.5 us.)
// 512-thread blocks: the streaming CRC's 70 KiB of LDS tables then still leave 4 waves per SIMD.
constexpr uint32_t kTailBlock = 512;
constexpr uint32_t kTailFinishWord = 19456 + kNumCst;  // two LDS words of the finishing workgroup

// The end of an optimistic decode without record shapes (launch_all, `finish`: every slot placed
// speculatively, records above lane_max possible), by the last workgroup of k_tail_count. When the
// lane kernel placed every record's every slot (no irregular record, irr[k] = 0), sent none to the
// exact walker, missed no key and listed no record for the wave gathers, the passes after this one
// (k_spine, k_down_gather, k_tail_gather) would only do their bookkeeping: done here, as
// tpl_quiet_finish does for k_tpl_lane. Anything else: kInfoResid = 1 and the host re-runs the
// decode with every pass (tfrg_result_info). (The tile sums the lane kernel wrote are cleared by the
// host before the next decode.)
// (s_ok: a word of the dynamic LDS; a static __shared__ object would move the dynamic region off LDS
// address 0, which role 2's table lookups address directly)
__device__ __forceinline__ void tail_quiet_finish(const DevOut& o, const uint8_t* slot_kind, uint32_t n_slots, uint32_t n,
                                  volatile uint32_t& s_ok) {
  if (threadIdx.x == 0) {
    s_ok = o.info[kInfoSlow] == 0u && o.info[kInfoMissRecords] == 0u && o.info[kInfoErrors] == 0u &&
           o.info[kInfoBig] == 0u && o.info[kInfoHuge] == 0u && o.info[kInfoDefer] == 0u &&
           o.info[kInfoWalkMiss] == 0u;
  }
  __syncthreads();
  if (threadIdx.x < n_slots && o.irr[threadIdx.x] != 0u) s_ok = 0u;  // (benign race: only zeroes)
  for (uint32_t k = threadIdx.x + kTailBlock; k < n_slots; k += kTailBlock)
    if (o.irr[k] != 0u) s_ok = 0u;
  __syncthreads();
  if (!s_ok) {
    if (threadIdx.x == 0) o.info[kInfoResid] = 1u;
    return;
  }
  for (uint32_t k = threadIdx.x; k < n_slots; k += kTailBlock) {
    o.totals[k] = n;
    o.rs[(size_t)k * (n + 1u) + n] = n;
  }
  if (threadIdx.x == 0) {
    uint64_t acc[4] = {0, 0, 0, 0};
    for (uint32_t k = 0; k < n_slots; ++k) {
      const uint32_t kd = slot_kind[k] & 3u;
      o.slot_base[k] = acc[kd];
      acc[kd] += n;
    }
    for (int k = 0; k < 4; ++k) o.kind_totals[k] = acc[k];
    if (acc[TFRG_KIND_INT64] > o.cap_i64 || acc[TFRG_KIND_FLOAT] > o.cap_f32 || acc[TFRG_KIND_BYTES] > o.cap_b)
      o.info[kInfoOverflow] = 1u;
    const uint64_t pm = n_slots >= 64u ? ~0ull : (1ull << n_slots) - 1ull;
    o.info[kInfoPlacedLo] = (uint32_t)pm;
    o.info[kInfoPlacedHi] = (uint32_t)(pm >> 32);
  }
}

// Optimistic decodes without record shapes (k_tail_count's first `walk_blocks` workgroups): the
// records above lane_max, walked while the other workgroups stream their payload CRC (role 2) instead
// of by k_lane_count before it. C2's records are all above lane_max: walking them one per lane is a
// chain of dependent HBM round trips per map entry (~27 us on 128 waves) that left the CRC waiting.
// k_lane_count (defer_big) listed them for the CRC and cleared their verdict bytes; the framing bits
// are OR-ed in here, the payload CRC's by role 2, into the same words. The columns, tile sums and
// irregular counts are those k_lane_count MODE 0 writes for a record it walks from HBM (with the
// 32-byte register window: this launch's register budget has room for it). A record the canonical
// walker does not take, or one with an out-of-line list, flags the batch for a full re-run
// (kInfoWalkMiss, read by tail_quiet_finish).
template <bool COMPAT>
__device__ __forceinline__ void role_big_walk(const DevBatch& B, const DevSchema& sc, const DevOut& o, const uint32_t* __restrict__ crc_tab,
                              uint32_t lane_max, uint32_t walk_blocks) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  constexpr uint32_t BLK = kTailBlock, kW = BLK / 64;
  const uint32_t S = sc.n_slots;
  // layout (launch_all: walk_lds): slicing tables, per-lane dict (counts, ranks), keys, spec targets
  uint32_t* tab = lds;
  uint32_t* cnt = tab + 256u * kLaneSlice;
  uint16_t* ord = reinterpret_cast<uint16_t*>(cnt + S * BLK);
  uint32_t* kht = cnt + S * BLK + ((S * BLK * 2u + 15u) & ~15u) / 4u;
  uint32_t* krec = kht + ((sc.ht_mask + 4u) & ~3u);
  uint32_t* spec_l = krec + sc.n_keys * kKrWords;
  uint32_t* spec_tl = spec_l + ((S + 7u) & ~7u);  // (16-byte aligned)
  for (uint32_t i = threadIdx.x; i < 256u * kLaneSlice; i += BLK) tab[i] = crc_tab[2048 + i];
  for (uint32_t i = threadIdx.x; i <= sc.ht_mask; i += BLK) kht[i] = sc.ht[i];
  for (uint32_t i = threadIdx.x; i < sc.n_keys * kKrWords; i += BLK) krec[i] = sc.krec[i];
  for (uint32_t i = threadIdx.x; i < S; i += BLK) {
    spec_l[i] = sc.spec[i];
    spec_target(spec_tl + kSpecTgtWords * i, o, sc.spec[i], B.n);
  }
  __syncthreads();
  const LdsKeys K{kht, krec, sc.ht_mask, sc.key_blob, sc.key_off};
  const LdsTab<1> T{tab, 0u};
  const uint32_t lane = threadIdx.x & 63u, wib = rfl32(threadIdx.x >> 6);
  const uint32_t ng = (B.n + 63u) >> 6, nw = walk_blocks * kW;
  uint32_t miss = 0;
  for (uint32_t g = blockIdx.x * kW + wib; g < ng; g += nw) {  // (wave-uniform)
    const uint32_t r = g * 64u + lane;
    const uint32_t tile = (g * 64u) >> kTileShift;
    RecView v{};
    bool big = false;
    if (r < B.n) {
      v = rec_view(B, r);
      big = v.status == TFRG_OK && v.e - v.st > lane_max;
    }
    if (!__ballot(big)) continue;
    CountSinkT<true> sink{&sc, &o, (lds_u16*)(ord + threadIdx.x), BLK, 0, B.n, r, v.p0, false, true};
    sink.cnt = (lds_u32*)(cnt + threadIdx.x);
    sink.spec = (const lds_u32*)spec_l;
    sink.spec_t = (const lds_spec_t*)spec_tl;
    bool done = false;
    if (big) {
      // (the payload CRC is role 2's unless the payload is shorter than one round: k_lane_count's rule)
      frame_verdicts<1, false>(B, v, T, nullptr, 0, (uint64_t)v.L < kCrcListMin);
      sink.fast_reset(S);
      const FastSrcG<true> fg{B.bytes, v.p0, (uint32_t)v.L, ((B.nbytes + 15) & ~15ull) - 4};
      done = fast_walk<COMPAT>(fg, K, sink) == TFRG_OK;
    }
    bool ool = false;
    for (uint32_t k = 0; k < S; ++k) {
      const uint32_t ov = done ? (uint32_t)sink.ord[(size_t)k * BLK] : 0u;
      const uint32_t c = ov ? sink.count_of(k) : 0u;
      ool |= c != 0u && !(c & kCountInline);
      if (done) {
        const size_t at = (size_t)k * B.n + r;
        o.order[at] = (uint16_t)ov;
        o.count[at] = c;
      }
      const uint32_t x = c & ~kCountInline;
      const uint64_t nz = __ballot(x != 0u);
      if (nz) {
        const uint32_t t = __ballot(x > 1u) ? wave_sum_u32(x) : (uint32_t)__popcll(nz);
        if (lane == 0) atomicAdd(&o.tsum[(size_t)k * o.tile_stride + tile], t);
      }
      if (spec_l[k]) {  // (wave-uniform)
        const uint64_t irm = __ballot(big && !(done && c == (1u | kCountInline)));
        if (irm && lane == 0) atomicAdd(&o.irr[k], (uint32_t)__popcll(irm));
      }
    }
    if (done) {
      o.status[r] = TFRG_OK;
      atomicOr(reinterpret_cast<uint32_t*>(o.verdict + (r & ~3u)), (uint32_t)v.verdict << (8u * (r & 3u)));
    }
    miss += (uint32_t)__popcll(__ballot(big && (!done || ool)));
  }
  if (miss && lane == 0) atomicAdd(&o.info[kInfoWalkMiss], miss);
}

// finish: (optimistic decode without shapes) the last workgroup ends the decode, tail_quiet_finish;
// walk_blocks: its first workgroups walk the records above lane_max (role_big_walk), the others
// stream the CRC
template <bool COMPAT, bool GORD>
__global__ __launch_bounds__(kTailBlock, 2) void k_tail_count(DevBatch B, DevSchema sc, DevOut o,
                                                           const uint32_t* __restrict__ crc_tab,
                                                           const uint32_t* __restrict__ consts, uint32_t lane_max,
                                                           uint32_t finish, uint32_t walk_blocks) {
  role_slow_count<1, COMPAT, GORD, kTailBlock>(B, sc, o, crc_tab, lane_max);
  __syncthreads();  // (the LDS tables are reloaded by role 2)
  if (blockIdx.x < walk_blocks)  // (block-uniform)
    role_big_walk<COMPAT>(B, sc, o, crc_tab, lane_max, walk_blocks);
  else
    role_crc_stream<kTailBlock>(B, o, crc_tab, consts, sc.n_slots, walk_blocks);
  if (finish) {  // (uniform)
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    volatile uint32_t* sh = lds + kTailFinishWord;  // (after role 2's tables)
    __syncthreads();
    if (threadIdx.x == 0) sh[0] = atomicAdd(&o.info[kInfoTplDone], 1u) == gridDim.x - 1u;
    __syncthreads();
    if (sh[0]) tail_quiet_finish(o, sc.slot_kind, sc.n_slots, B.n, sh[1]);
  }
}

// Record queue of a staged wavefront kernel, three stages deep: bytes of the next record (in
// registers), start/end(/status) of the one after, the big_list index of the one after that.
struct RecPipe {
  uint32_t r1, r2;
  uint64_t s1, e1;
  int32_t t1;
  uint32_t r3v;       // vector-loaded, in flight
  uint64_t s2v, e2v;  // vector-loaded, in flight
  int32_t t2v;
};

// Software pipeline of the staged wavefront kernels: the next record's bytes are loaded into
// registers (12 x 16 B per lane) while the current one is walked from LDS, so HBM latency hides
// behind the walk. Loads are unconditional (clamped addresses) so the wait counts stay static.
constexpr int kPrefWords = (int)(kWStage / 1024);
struct Pref {  // named fields, returned by value: an array or an out-parameter is kept in scratch
  uint4 w0, w1, w2, w3, w4, w5, w6, w7, w8, w9, w10, w11;
};

#define TFRG_PREF_LOAD(j)                                                        \
  if constexpr ((j) < kPrefWords) {                                              \
    const uint64_t q = lo16 + lane * 16u + (uint32_t)(j)*1024u;                  \
    p.w##j = *reinterpret_cast<const uint4*>(src + (q < hi ? q : lo16c));         \
  }
#define TFRG_PREF_STORE(j)                                                       \
  if constexpr ((j) < kPrefWords) {                                              \
    const uint32_t off = lane * 16u + (uint32_t)(j) * 1024u;                     \
    if (lo16 + off < hi) *reinterpret_cast<uint4*>(dst + off) = p.w##j;          \
  }

__device__ __forceinline__ Pref pref_load_v(const uint8_t* src, uint64_t lo16, uint64_t hi, uint32_t lane) {
  // the loads past the record re-read its first 16 bytes (one line, already requested): clamping
  // them to the batch start put every wave's spare loads on the same few lines of one L2 channel
  const uint64_t lo16c = hi > lo16 ? lo16 : 0ull;
  Pref p;
  static_assert(kPrefWords <= 12 && kWStage % 1024 == 0, "pref_load is spelled out for up to 12 words");
  TFRG_PREF_LOAD(0) TFRG_PREF_LOAD(1) TFRG_PREF_LOAD(2) TFRG_PREF_LOAD(3) TFRG_PREF_LOAD(4) TFRG_PREF_LOAD(5)
  TFRG_PREF_LOAD(6) TFRG_PREF_LOAD(7) TFRG_PREF_LOAD(8) TFRG_PREF_LOAD(9) TFRG_PREF_LOAD(10) TFRG_PREF_LOAD(11)
  return p;
}

__device__ __forceinline__ void pref_store(const Pref& p, uint8_t* dst, uint64_t lo16, uint64_t hi, uint32_t lane) {
  TFRG_PREF_STORE(0) TFRG_PREF_STORE(1) TFRG_PREF_STORE(2) TFRG_PREF_STORE(3) TFRG_PREF_STORE(4)
  TFRG_PREF_STORE(5) TFRG_PREF_STORE(6) TFRG_PREF_STORE(7) TFRG_PREF_STORE(8) TFRG_PREF_STORE(9)
  TFRG_PREF_STORE(10) TFRG_PREF_STORE(11)
}
#undef TFRG_PREF_LOAD
#undef TFRG_PREF_STORE

// ------------------------------------------------------------------------------------------------
// Row-split scan, second level: the tile sums of every slot in chunks of 4096 tiles (1 M records),
// one 256-thread workgroup per (slot, chunk), 16 tiles per thread, with a decoupled look-back
// across the chunks of a slot: each workgroup publishes its chunk total (flag 1) at once, sums
// its predecessors' totals back to the first inclusive prefix (flag 2), publishes its own
// inclusive prefix and writes full exclusive prefixes over the tile sums in place. Chunks are
// taken in ticket order, so every workgroup waited on has started. The last workgroup to finish
// derives the per-kind column bases from the slot totals.
// ------------------------------------------------------------------------------------------------
constexpr int kSpineBlock = 256;
constexpr int kSpineItems = 16;
static_assert(kSpineBlock * kSpineItems == (1 << kSpineChunkShift), "one chunk per spine workgroup");

// exclusive prefix of chunk `chunk` from its predecessors' look-back words (lb[0..chunk)), by one
// wave: lane l reads predecessor chunk - 1 - l (64 words per round trip, not one), the nearest
// inclusive prefix (flag 2) ends the sum; a predecessor in range that has not published its total
// yet (flag 0; it has started: ticket order) makes the wave read the window again
__device__ __forceinline__ uint32_t spine_look_back(const uint64_t* lb, uint32_t chunk, uint32_t lane) {
  uint32_t excl = 0;
  for (int64_t base = (int64_t)chunk - 1; base >= 0;) {  // (wave-uniform)
    const int64_t j = base - (int64_t)lane;
    const uint64_t w = j >= 0 ? __hip_atomic_load(&lb[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                              : (2ull << 32);  // (before the first chunk: an inclusive prefix of 0)
    const uint32_t flag = (uint32_t)(w >> 32);
    const uint64_t inc = __ballot(flag == 2u), unset = __ballot(flag == 0u);
    const uint32_t stop = inc ? (uint32_t)__builtin_ctzll(inc) : 64u;  // lanes [0, stop] are summed
    const uint64_t range = stop >= 63u ? ~0ull : (2ull << stop) - 1ull;
    if (unset & range) {
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    uint32_t v = lane <= stop ? (uint32_t)w : 0u;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += (uint32_t)__shfl_xor((int)v, m, 64);
    excl += v;
    if (stop < 64u) break;
    base -= 64;
  }
  return excl;
}

// DevSchema::spec: the speculative placement of slot k is not final -- some record of it or of an
// earlier slot of its kind (all speculative: they form a prefix) was irregular. Otherwise every such
// slot holds n values at rows 0..n-1, so the column base of slot k is n * rank, as placed.
__device__ __forceinline__ bool spec_failed(const uint32_t* spec, const DevOut& o, uint32_t k) {
  const uint32_t sw = spec ? spec[k] : 0u;
  if (!sw) return false;
  for (uint32_t j = 0; j <= k; ++j) {
    const uint32_t sj = spec[j];
    if (sj && ((sj ^ sw) & 3u) == 0u && o.irr[j]) return true;
  }
  return false;
}
__device__ __forceinline__ bool spec_placed(const uint32_t* spec, const DevOut& o, uint32_t k) {
  return spec && spec[k] && !spec_failed(spec, o, k);
}

// grid n_chunks * n_slots (1-D). With DevSchema::spec, a workgroup of a slot whose speculative
// placement failed first copies the placed single values of its chunk's records back into their loc
// words (value columns -> loc: no overlap with k_down_gather's writes, which follow this kernel).
__global__ __launch_bounds__(kSpineBlock) void k_spine(DevOut o, const uint8_t* __restrict__ slot_kind, uint32_t n_slots,
                                                       uint32_t n_tiles, const uint32_t* __restrict__ spec, uint32_t n) {
  __shared__ uint32_t s_w[kSpineBlock / 64];
  __shared__ uint32_t s_ticket, s_excl, s_last;
  __shared__ uint32_t s_w2[kSpineBlock];  // last workgroup: slot totals of one pass
  __shared__ uint8_t s_kind[kSpineBlock];
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  if (threadIdx.x == 0) s_ticket = atomicAdd(&o.info[kInfoSpineTicket], 1u);
  // Every slot's placement final (a templated batch): no scan, no look-back and no last-workgroup
  // pass, since the placement fixes every total (n) and column base. Read beside the ticket: one
  // round trip to the device-scope words instead of three.
  const bool allp = spec && n_slots <= (uint32_t)kSpineBlock &&
                    __syncthreads_and(threadIdx.x >= n_slots || spec_placed(spec, o, threadIdx.x));
  __syncthreads();
  const uint32_t slot = s_ticket / o.n_chunks, chunk = s_ticket % o.n_chunks;
  if (allp) {  // (workgroup-uniform) this chunk's tile sums zeroed for the next decode
    uint32_t* t = o.tsum + (size_t)slot * o.tile_stride;
    const uint32_t i0 = (chunk << kSpineChunkShift) + threadIdx.x * kSpineItems;
#pragma unroll
    for (int j = 0; j < kSpineItems; j += 4)
      if (i0 + j < n_tiles) *reinterpret_cast<uint4*>(t + i0 + j) = make_uint4(0, 0, 0, 0);
    if (s_ticket == 0u && threadIdx.x == 0) {  // totals, column bases, kind totals (as the last pass)
      uint64_t acc[4] = {0, 0, 0, 0};
      for (uint32_t k = 0; k < n_slots; ++k) {
        const uint32_t kd = slot_kind[k] & 3u;
        o.totals[k] = n;
        o.slot_base[k] = acc[kd];
        acc[kd] += n;
      }
      for (int k = 0; k < 4; ++k) o.kind_totals[k] = acc[k];
      if (acc[TFRG_KIND_INT64] > o.cap_i64 || acc[TFRG_KIND_FLOAT] > o.cap_f32 || acc[TFRG_KIND_BYTES] > o.cap_b)
        o.info[kInfoOverflow] = 1u;
    }
    return;
  }
  if (spec_failed(spec, o, slot)) {  // (workgroup-uniform; rare: an irregular batch)
    const uint32_t sw = spec[slot];
    const uint64_t sb = (uint64_t)n * ((sw >> 2) - 1u);
    const uint64_t r0 = (uint64_t)chunk << (kSpineChunkShift + kTileShift);
    const uint64_t r1 = r0 + (1ull << (kSpineChunkShift + kTileShift)) < n ? r0 + (1ull << (kSpineChunkShift + kTileShift)) : n;
    for (uint64_t r = r0 + threadIdx.x; r < r1; r += kSpineBlock) {
      const size_t at = (size_t)slot * n + r;
      if (o.lmask && !((o.lmask[r >> 6] >> (r & 63u)) & 1ull)) {
        o.count[at] = 1u | kCountInline;  // a k_tpl_lane record (placed, its count word not written)
      } else if (o.count[at] != (1u | kCountInline)) {
        continue;
      }
      const uint64_t p = sb + r;
      uint2 lv = make_uint2(0, 0);
      if ((sw & 3u) == TFRG_KIND_INT64) {
        if (p < o.cap_i64) {
          const uint64_t v = (uint64_t)o.i64[p];
          lv = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
        }
      } else if ((sw & 3u) == TFRG_KIND_FLOAT) {
        if (p < o.cap_f32) lv.x = o.f32[p];
      } else if (p < o.cap_b) {
        lv = make_uint2(o.b_off[p], o.b_len[p]);
      }
      o.loc[at] = lv;
    }
  }
  uint32_t* t = o.tsum + (size_t)slot * o.tile_stride;
  uint64_t* lb = o.spine_lb + (size_t)slot * o.n_chunks;
  const uint32_t i0 = (chunk << kSpineChunkShift) + threadIdx.x * kSpineItems;
  if (spec_placed(spec, o, slot)) {  // (workgroup-uniform) n values at rows 0..n-1 (spec_failed): no scan
    // (k_down_gather skips the slot): its tile sums zeroed for the next decode, its look-back words
    // never written
#pragma unroll
    for (int j = 0; j < kSpineItems; j += 4)
      if (i0 + j < n_tiles) *reinterpret_cast<uint4*>(t + i0 + j) = make_uint4(0, 0, 0, 0);
    if (chunk == o.n_chunks - 1u && threadIdx.x == 0) o.totals[slot] = n;
  } else {
  uint32_t v[kSpineItems];
#pragma unroll
  for (int j = 0; j < kSpineItems; j += 4) {  // tile_stride is a multiple of 4: whole uint4s are in bounds
    uint4 q = make_uint4(0, 0, 0, 0);
    if (i0 + j < n_tiles) q = *reinterpret_cast<const uint4*>(t + i0 + j);
    v[j] = q.x;
    v[j + 1] = i0 + j + 1 < n_tiles ? q.y : 0u;
    v[j + 2] = i0 + j + 2 < n_tiles ? q.z : 0u;
    v[j + 3] = i0 + j + 3 < n_tiles ? q.w : 0u;
  }
  uint32_t sum = 0;
#pragma unroll
  for (int j = 0; j < kSpineItems; ++j) sum += v[j];
  const uint32_t incl = wave_incl_scan_u32(sum, lane);
  if (lane == 63) s_w[wid] = incl;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kSpineBlock / 64; ++w) {
    const uint32_t x = s_w[w];
    pre += (uint32_t)w < wid ? x : 0u;
    tot += x;
  }
  if (threadIdx.x < 64u) {  // wave 0
    if (threadIdx.x == 0)
      __hip_atomic_store(&lb[chunk], ((uint64_t)(chunk ? 1u : 2u) << 32) | tot, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t excl = spine_look_back(lb, chunk, lane);
    if (threadIdx.x == 0) {
      if (chunk) __hip_atomic_store(&lb[chunk], (2ull << 32) | (excl + tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (chunk == o.n_chunks - 1u) o.totals[slot] = excl + tot;
      s_excl = excl;
    }
  }
  __syncthreads();
  uint32_t run = s_excl + pre + incl - sum;
#pragma unroll
  for (int j = 0; j < kSpineItems; j += 4) {
    uint32_t w[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      w[m] = run;
      run += v[j + m];
    }
    if (i0 + j < n_tiles) *reinterpret_cast<uint4*>(t + i0 + j) = make_uint4(w[0], w[1], w[2], w[3]);
  }
  }
  if (threadIdx.x == 0) {
    __threadfence();
    s_last = atomicAdd(&o.info[kInfoSpineDone], 1u) == gridDim.x - 1u;
  }
  __syncthreads();
  if (!s_last) return;  // workgroup-uniform
  __threadfence();      // every slot total is visible
  // per pass of 256 slots, thread 0 derives the per-kind column bases from LDS copies
  uint64_t acc[4] = {0, 0, 0, 0};  // thread 0
  for (uint32_t b = 0; b < n_slots; b += kSpineBlock) {
    const uint32_t k = b + threadIdx.x;
    if (k < n_slots) {
      s_w2[threadIdx.x] = __hip_atomic_load(&o.totals[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_kind[threadIdx.x] = slot_kind[k] & 3u;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t m = n_slots - b < (uint32_t)kSpineBlock ? n_slots - b : (uint32_t)kSpineBlock;
      for (uint32_t j = 0; j < m; ++j) {
        const uint32_t kd = s_kind[j];
        o.slot_base[b + j] = acc[kd];
        acc[kd] += s_w2[j];
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    for (int k = 0; k < 4; ++k) o.kind_totals[k] = acc[k];
    // capacities bound the values of disjoint ranges; overlapping / repeated ranges can exceed
    // them (stores past a capacity are dropped): the host reports TFRG_E_LIMIT
    if (acc[TFRG_KIND_INT64] > o.cap_i64 || acc[TFRG_KIND_FLOAT] > o.cap_f32 || acc[TFRG_KIND_BYTES] > o.cap_b)
      o.info[kInfoOverflow] = 1u;
  }
}

// ------------------------------------------------------------------------------------------------
// Gather: decode the (validated) list message of every present slot into its column.
// ------------------------------------------------------------------------------------------------
// list_values into the value columns from element dst on (stores past a capacity dropped)
struct ColOut {
  const DevOut& o;
  uint64_t base;  // absolute payload start (bytes views)
  uint64_t dst;
  __device__ __forceinline__ void bytes(int64_t off, int64_t len) {
    if (dst < o.cap_b) {
      o.b_off[dst] = (uint32_t)(base + (uint64_t)off);
      o.b_len[dst] = (uint32_t)len;
    }
    ++dst;
  }
  __device__ __forceinline__ void f32(uint32_t bits) {
    if (dst < o.cap_f32) o.f32[dst] = bits;
    ++dst;
  }
  __device__ __forceinline__ void i64(int64_t v) {
    if (dst < o.cap_i64) o.i64[dst] = v;
    ++dst;
  }
};
// A list location must lie inside its record's payload: every location the count passes write does
// (lo + len <= L). A word that does not -- stale or corrupt -- would send a gather walk through bytes
// outside the record (and, with a garbage length, on for billions of steps), so the record fails
// with TFRG_ST_INTERNAL (aux = the slot) and the list is not walked.
__device__ __forceinline__ bool loc_in_record(uint2 lc, int64_t L) {
  return (uint64_t)lc.x + lc.y <= (uint64_t)(L < 0 ? 0 : L);
}
__device__ void loc_fail(const DevOut& o, uint32_t r, uint32_t k, uint2 lc) {
  if (atomicExch(&o.status[r], (int)TFRG_ST_INTERNAL) == TFRG_OK) {
    o.aux[r] = k;
    atomicAdd(&o.info[kInfoErrors], 1u);
    atomicMax(&o.info[kInfoFirstError], ~r);
  }
#if defined(TFRG_DEBUG)
  printf("tfrg: record %u slot %u: list location (%u, %u) outside its record\n", r, k, lc.x, lc.y);
#else
  (void)lc;
#endif
}

template <bool COMPAT, class S>
__device__ void list_gather(S& s, const DevOut& o, int kind, int64_t lo, int64_t ll, uint64_t dst) {
  ColOut out{o, s.p0, dst};
  list_values<COMPAT>(s, kind, lo, ll, out);
}

// one int64 varint at `pos` of a validated packed chunk ending at `e` (fast path): <= 4 bytes from
// one word, longer ones byte by byte with the reference's compat semantics; false = bail
template <bool COMPAT>
__device__ __forceinline__ bool fast_list_gather(const FastSrc& s, const DevOut& o, uint32_t kind, uint32_t lo,
                                                 uint32_t ll, uint64_t dst) {
  uint32_t q = lo;
  const uint32_t le = lo + ll;
  while (q < le) {
    uint32_t fn, co, cl;
    if (!ffield(s, q, le, fn, co, cl) || fn != 1u) return false;
    if (kind == TFRG_KIND_BYTES) {
      if (dst < o.cap_b) {
        o.b_off[dst] = (uint32_t)(s.base + co);
        o.b_len[dst] = cl;
      }
      ++dst;
    } else if (kind == TFRG_KIND_FLOAT) {
      if (cl & 3u) return false;
      for (uint32_t i = 0; i < cl; i += 4) {
        if (dst < o.cap_f32) o.f32[dst] = lds_u32u(s.l, s.p + co + i);
        ++dst;
      }
    } else {
      uint32_t p = co;
      const uint32_t e = co + cl;
      if (dst + cl <= o.cap_i64) {  // at most cl values: no per-value capacity check, a running pointer
        int64_t* out = o.i64 + dst;
        while (p < e) {
          int64_t v;
          if (!fast_value<COMPAT>(s, p, e, v)) return false;
          *out++ = v;
        }
        dst = (uint64_t)(out - o.i64);
      } else {
        while (p < e) {
          int64_t v;
          if (!fast_value<COMPAT>(s, p, e, v)) return false;
          if (dst < o.cap_i64) o.i64[dst] = v;
          ++dst;
        }
      }
    }
  }
  return true;
}

// values of every out-of-line present slot of record r (inline single values are written by the
// caller's first pass)
template <bool COMPAT, class S>
__device__ __forceinline__ void gather_record(const DevBatch& B, const DevSchema& sc, const DevOut& o, uint32_t r,
                                              S& s, uint64_t placed) {
  for (uint32_t k = 0; k < sc.n_slots; ++k) {
    if (k < 64u && ((placed >> k) & 1ull)) continue;  // (count words of k_tpl_lane records unwritten)
    const size_t at = (size_t)k * B.n + r;
    const uint32_t c = o.count[at];
    if (!c || (c & kCountInline)) continue;
    const uint2 lc = o.loc[at];
    if (!loc_in_record(lc, s.L)) {
      loc_fail(o, r, k, lc);
      continue;
    }
    const uint64_t dst = o.slot_base[k] + o.rs[(size_t)k * (B.n + 1) + r];
    list_gather<COMPAT>(s, o, sc.slot_kind[k], (int64_t)lc.x, (int64_t)lc.y, dst);
  }
}

// Row-split scan, last level, fused with the lane-record gather. One workgroup per 256-record tile:
// per slot, the tile prefix (k_spine) + the in-tile exclusive scan of the counts give the row splits;
// single values kept inline by the count pass are written straight from the loc word, other lists of
// records <= lane_max are decoded from the wave's LDS stage. Records above lane_max belong to the
// wavefront gather kernels, which run next and read these row splits.
// kDT tiles per workgroup: kDT x kDG (count, loc) loads in flight per thread (4 for large batches,
// 1 when that would leave CUs idle)

template <bool COMPAT, uint32_t kDT>
__global__ __launch_bounds__(kLaneBlock) void k_down_gather(DevBatch B, DevSchema sc, DevOut o, uint32_t lane_max,
                                                            uint32_t n_tiles) {
  // slots per scan group (one barrier each): 2 beside 4 tiles per workgroup, 8 with one tile (small
  // batches and wide schemas: fewer barriers between the loads, same registers)
  constexpr uint32_t kDG = kDT == 1 ? 8u : 2u;
  __shared__ uint32_t s_w[2][kDT * kDG][4];  // wave totals, double-buffered across slot groups
  const uint32_t lane = threadIdx.x & 63u, wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t S = sc.n_slots;
  if (blockIdx.x == 0)
    for (uint32_t k = threadIdx.x; k < S; k += kLaneBlock) o.rs[(size_t)k * (B.n + 1) + B.n] = o.totals[k];
  // slots whose speculative placement by the lane kernel is final (DevSchema::spec): nothing to do.
  // Read once (the first 64 slots as a mask): the tile-sum stores below may alias irr for the
  // compiler, which would otherwise re-load spec / irr with their latency in every group.
  // (lane k: slot k, so the words of all of them are loaded at once)
  const uint64_t pmask = sc.spec ? (uint64_t)__ballot(lane < S && spec_placed(sc.spec, o, lane)) : 0ull;
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // (for k_tail_gather, which clears irr)
    o.info[kInfoPlacedLo] = (uint32_t)pmask;
    o.info[kInfoPlacedHi] = (uint32_t)(pmask >> 32);
  }
  auto placed = [&](uint32_t k) -> bool {
    return k < 64u ? ((pmask >> k) & 1ull) != 0ull : k < S && spec_placed(sc.spec, o, k);
  };
  // every slot placed: nothing to do (k_spine zeroed their tile sums; their look-back words were
  // never written)
  if (S <= 64u && pmask == (~0ull >> (64u - S))) return;
  uint32_t buf = 0;
  // a resident grid strides over the groups of kDT tiles (a launch of one workgroup per group spent
  // most of its time dispatching workgroups that only zero their tile sums when every slot is placed)
  const uint32_t n_groups = (n_tiles + kDT - 1) / kDT;
  for (uint32_t grp = blockIdx.x; grp < n_groups; grp += gridDim.x) {  // (workgroup-uniform)
    const uint32_t tile0 = grp * kDT;
    uint32_t r[kDT];
    bool valid[kDT];
  #pragma unroll
    for (uint32_t t = 0; t < kDT; ++t) {
      r[t] = ((tile0 + t) << kTileShift) + threadIdx.x;
      valid[t] = r[t] < B.n;
    }
    // row splits of every slot + inline single values. A non-zero count implies a decoded record
    // with the slot present (failed records and absent slots have count 0).
    uint32_t need = 0;  // bit t: record r[t] has an out-of-line list
    for (uint32_t k0 = 0; k0 < S; k0 += kDG) {
      bool sk[kDG];
      bool all = true;
  #pragma unroll
      for (uint32_t g = 0; g < kDG; ++g) {
        sk[g] = placed(k0 + g);
        all &= sk[g] || k0 + g >= S;
      }
      if (all) continue;  // (workgroup-uniform; buf toggles only with a barrier)
      uint32_t c[kDT][kDG], ex[kDT][kDG];
      uint2 lc[kDT][kDG];
  #pragma unroll
      for (uint32_t t = 0; t < kDT; ++t) {  // every load of the group issued before the barrier
  #pragma unroll
        for (uint32_t g = 0; g < kDG; ++g) {
          const uint32_t k = k0 + g < S ? k0 + g : k0;
          const bool in = valid[t] && k0 + g < S && !sk[g];
          c[t][g] = in ? o.count[(size_t)k * B.n + r[t]] : 0u;
          lc[t][g] = in ? o.loc[(size_t)k * B.n + r[t]] : make_uint2(0, 0);
        }
      }
  #pragma unroll
      for (uint32_t t = 0; t < kDT; ++t) {
  #pragma unroll
        for (uint32_t g = 0; g < kDG; ++g) {
          const uint32_t x = c[t][g] & ~kCountInline;
          // 0/1 counts (single values): the inclusive scan is a masked popcount of the ballot
          const uint32_t incl = __ballot(x > 1u) ? wave_incl_scan_u32(x, lane)
                                                 : (uint32_t)__popcll(__ballot(x != 0u) & (~0ull >> (63u - lane)));
          ex[t][g] = incl - x;
          if (lane == 63) s_w[buf][t * kDG + g][wib] = incl;
        }
      }
      __syncthreads();  // (the other buffer is rewritten only after the next group's barrier)
  #pragma unroll
      for (uint32_t g = 0; g < kDG; ++g) {
        const uint32_t k = k0 + g;
        if (k >= S) break;
        if (sk[g]) continue;
        const uint32_t kind = sc.slot_kind[k];
        const uint64_t sbase = o.slot_base[k];
  #pragma unroll
        for (uint32_t t = 0; t < kDT; ++t) {
          if (tile0 + t >= n_tiles) break;
          uint32_t pre = o.tsum[(size_t)k * o.tile_stride + tile0 + t];
          for (uint32_t w = 0; w < wib; ++w) pre += s_w[buf][t * kDG + g][w];
          const uint32_t rsv = pre + ex[t][g];
          if (valid[t]) o.rs[(size_t)k * (B.n + 1) + r[t]] = rsv;
          if (c[t][g] & kCountInline) put_inline(o, kind, lc[t][g], sbase + rsv);
          else if (c[t][g]) need |= 1u << t;
        }
      }
      buf ^= 1u;
    }
    // records with an out-of-line list: k_list_gather (kept out of this kernel so its register
    // budget stays that of the scan); larger records are skipped there (wavefront gathers)
  #pragma unroll
    for (uint32_t t = 0; t < kDT; ++t) {
      const bool nd = (need >> t) & 1u;
      const uint64_t nm = __ballot(nd);
      if (nm) {
        const int f = __builtin_ctzll(nm);
        uint32_t b0 = 0;
        if (lane == (uint32_t)f) b0 = atomicAdd(&o.info[kInfoNeed], (uint32_t)__popcll(nm));
        b0 = __shfl(b0, f, 64);
        if (nd) o.slow_list[b0 + (uint32_t)__popcll(nm & ((1ull << lane) - 1ull))] = r[t];
      }
    }
    // Leave the scan words zeroed for the next decode (no per-call memset): this group's tile
    // prefixes of every slot (+ the stride padding after the last tile), and the spine's look-back
    // words (workgroup 0; k_spine has finished).
    __syncthreads();
    const uint32_t t_end = tile0 + kDT < n_tiles ? tile0 + kDT : (tile0 < n_tiles ? o.tile_stride : tile0);
    const uint32_t span = t_end - tile0;
    for (uint32_t i = threadIdx.x; i < S * span; i += kLaneBlock)
      o.tsum[(size_t)(i / span) * o.tile_stride + tile0 + i % span] = 0u;
  }
  if (blockIdx.x == 0)
    for (uint32_t i = threadIdx.x; i < 2u * S * o.n_chunks; i += kLaneBlock) reinterpret_cast<uint32_t*>(o.spine_lb)[i] = 0u;
}

// Out-of-line lists of lane records (k_down_gather's list; lane order within a wave, so the records
// of a wave are usually one contiguous span): staged in LDS and decoded by their own lane.
template <bool COMPAT>
__device__ void role_list_gather(const DevBatch& B, const DevSchema& sc, const DevOut& o, uint32_t lane_max,
                                 uint8_t* stage, uint64_t placed) {
  const uint32_t lane = threadIdx.x & 63u, wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nneed = o.info[kInfoNeed];
  const uint32_t S = sc.n_slots;
  for (uint32_t base = blockIdx.x * kLaneBlock + wib * 64u; base < nneed; base += gridDim.x * kLaneBlock) {
    const uint32_t i = base + lane;
    bool need = i < nneed;
    const uint32_t r = need ? o.slow_list[i] : 0u;
    RecView v{};
    if (need) {
      v = rec_view(B, r);
      need = v.e - v.st <= lane_max;  // larger records belong to the wavefront gather kernels
    }
    uint64_t lo, hi;
    wave_span(need, v.st, v.e, lo, hi);
    const uint64_t lo16 = lo & ~15ull;
    const bool staged = hi > lo && hi - lo16 <= kStageBytes;
    if (staged) {
      stage_span(stage, B.bytes, lo16, hi, lane);
      wave_lds_sync();
    }
    if (need) {
      if (staged) {
        const FastSrc fs{stage, (uint32_t)(v.p0 - lo16), (uint32_t)v.L, v.p0};
        LdsSrc s;
        s.init(stage, lo16, v.p0, v.L);
        for (uint32_t k = 0; k < S; ++k) {
          if (k < 64u && ((placed >> k) & 1ull)) continue;  // (count words of k_tpl_lane records unwritten)
          const size_t at = (size_t)k * B.n + r;
          const uint32_t c = o.count[at];
          if (!c || (c & kCountInline)) continue;
          const uint2 lc = o.loc[at];
          if (!loc_in_record(lc, v.L)) {
            loc_fail(o, r, k, lc);
            continue;
          }
          const uint32_t kind = sc.slot_kind[k];
          const uint64_t dst = o.slot_base[k] + o.rs[(size_t)k * (B.n + 1) + r];
          if (!fast_list_gather<COMPAT>(fs, o, kind, lc.x, lc.y, dst))
            list_gather<COMPAT>(s, o, (int)kind, (int64_t)lc.x, (int64_t)lc.y, dst);
        }
      } else {
        Src s;
        s.init(B.bytes, v.p0, v.L);
        gather_record<COMPAT>(B, sc, o, r, s, placed);
      }
    }
    wave_lds_sync();
  }
}

// Huge records: one slot per lane, lists read from HBM.
template <bool COMPAT>
__device__ void role_wave_gather(const DevBatch& B, const DevSchema& sc, const DevOut& o, uint64_t placed) {
  const uint32_t lane = threadIdx.x & 63u, wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nhuge = o.info[kInfoHuge];
  for (uint32_t i = blockIdx.x * kWavesPerBlock + wib; i < nhuge; i += gridDim.x * kWavesPerBlock) {
    const uint32_t r = o.big_list[B.n - 1u - i];
    if (o.status[r] != TFRG_OK) continue;  // wave-uniform
    const RecView v = rec_view(B, r);
    for (uint32_t k = lane; k < sc.n_slots; k += 64) {
      if (k < 64u && ((placed >> k) & 1ull)) continue;  // (count words of k_tpl_lane records unwritten)
      const size_t at = (size_t)k * B.n + r;
      const uint32_t c = o.count[at];
      if (!c || (c & kCountInline)) continue;  // absent / empty, or written inline by k_down_gather
      const uint2 lc = o.loc[at];
      if (!loc_in_record(lc, v.L)) {
        loc_fail(o, r, k, lc);
        continue;
      }
      const uint64_t dst = o.slot_base[k] + o.rs[(size_t)k * (B.n + 1) + r];
      Src s;
      s.init(B.bytes, v.p0, v.L);
      list_gather<COMPAT>(s, o, (int)sc.slot_kind[k], (int64_t)lc.x, (int64_t)lc.y, dst);
    }
  }
}

__device__ __forceinline__ uint64_t readlane_u64(uint64_t x, int k) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)x, k);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(x >> 32), k);
  return ((uint64_t)hi << 32) | lo;
}

// Values of up to 64 slots of one staged record (one slot per lane). Canonical packed float lists
// are copied by the whole wave (lane j moves value j: contiguous stores), canonical packed int64
// lists are decoded by the whole wave (int64_balanced); bytes lists and anything non-canonical are
// decoded by their own lane.
// Per-lane form of hdr_0a: the list at [lo, lo+ll) is exactly one canonical chunk (tag 0x0a, length
// varint of <= 3 bytes) whose body is [bo, bo+bl).
__device__ __forceinline__ bool hdr_0a_v(const FastSrc& s, uint32_t lo, uint32_t ll, uint32_t& bo, uint32_t& bl) {
  const uint32_t w = lo + 2 <= s.L ? s.w4(lo) : 0u;
  const uint32_t b1 = (w >> 8) & 0xffu, b2 = (w >> 16) & 0xffu, b3 = w >> 24;
  const uint32_t h = b1 < 0x80u ? 2u : b2 < 0x80u ? 3u : 4u;
  const uint32_t len = (b1 & 0x7fu) | (h > 2u ? (b2 & 0x7fu) << 7 : 0u) | (h > 3u ? (b3 & 0x7fu) << 14 : 0u);
  bo = lo + h;
  bl = len;
  return (w & 0xffu) == 0x0au && (h < 4u || b3 < 0x80u) && bo + bl == lo + ll;
}

// Terminator bytes (< 0x80) among stage bytes [x0, x1) at stage offset `base`.
__device__ __forceinline__ uint32_t count_terms(const uint8_t* l, uint32_t base, uint32_t x0, uint32_t x1) {
  uint32_t n = 0;
  for (uint32_t q = x0; q < x1; q += 4) {
    uint32_t t = ~lds_u32u(l, base + q) & 0x80808080u;
    if (x1 - q < 4u) t &= bytes_mask(x1 - q);
    n += (uint32_t)__popc(t);
  }
  return n;
}

// The varint whose first byte is the low byte of w0 (w0, w1, w2: the 12 bytes from there),
// branch-free: per-word masks of the bytes up to the first terminator (t ^ (t - 1): all ones when
// the word has none; zero past the terminator's word) give its length (popcount), the 7-bit groups
// of each word are compacted under those masks and combined (COMPAT: the reference's int-width
// shifts, decoder.pyx:34-50, as in fast_value). Returns the length in bytes, 0 = more than 10.
template <bool COMPAT>
__device__ __forceinline__ uint32_t varint_w(uint32_t w0, uint32_t w1, uint32_t w2, int64_t& val) {
  const uint32_t t0 = ~w0 & 0x80808080u, t1 = ~w1 & 0x80808080u, t2 = ~w2 & 0x00008080u;
  const uint32_t m0 = t0 ^ (t0 - 1u);
  const uint32_t m1 = t0 ? 0u : t1 ^ (t1 - 1u);
  const uint32_t m2 = (t0 | t1) ? 0u : (t2 ^ (t2 - 1u)) & 0xffffu;
  const uint32_t nb = (uint32_t)(__popc(m0) + __popc(m1) + __popc(m2)) >> 3;
  const uint32_t x = vgroups(w0, m0), x1 = vgroups(w1, m1), x2 = vgroups(w2, m2);  // groups 0-3, 4-7, 8-9
  if (COMPAT) {
    const uint32_t lo32 = x | (x1 << 28) | ((x1 >> 7) << 3) | (x2 << 24);
    const bool neg = ((x1 >> 3) | (x2 >> 7)) & 1u;
    val = (int64_t)(((uint64_t)(neg ? 0xffffffffu : 0u) << 32) | lo32);
  } else {
    val = (int64_t)((uint64_t)x | ((uint64_t)x1 << 28) | ((uint64_t)x2 << 56));
  }
  return (t0 | t1 | t2) != 0u ? nb : 0u;
}

// the 12 stage bytes at offset `off` as three words (four aligned dwords: two ds_read2 from one address)
__device__ __forceinline__ void stage_w3(const uint8_t* l, uint32_t off, uint32_t& w0, uint32_t& w1, uint32_t& w2) {
  const uint32_t sh = off & 3u;
  const uint32_t* W = reinterpret_cast<const uint32_t*>(l) + (off >> 2);
  const uint32_t d0 = W[0], d1 = W[1], d2 = W[2], d3 = W[3];
  w0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
  w1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
  w2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
}

// One varint of 1..10 bytes at payload offset `pos` of a staged record. The caller guarantees a
// terminator before the end of the body (its last byte is one), so the bytes read past it never
// matter. false = more than 10 bytes (the exact path reports it).
template <bool COMPAT>
__device__ __forceinline__ bool varint_bf(const FastSrc& s, uint32_t& pos, int64_t& val) {
  uint32_t w0, w1, w2;
  stage_w3(s.l, s.p + pos, w0, w1, w2);
  const uint32_t nb = varint_w<COMPAT>(w0, w1, w2, val);
  pos += nb;
  return nb != 0u;
}

// Canonical packed int64 lists of one staged record, balanced over the whole wave. The bodies of
// the eligible slots (iv: one canonical chunk whose last byte is a terminator, so its value starts
// are exactly its c values), in slot order, form one virtual byte axis of T bytes cut into 64 equal
// ranges; lane j decodes every value that STARTS in its range [a, b). Its first value's index is
// the number of starts before a (wave scan of the per-lane start counts) minus the slot's value
// base. Per-slot parameters are fetched by lane shuffles in wave-uniform loops. A lane-per-list
// decode waits for the wave's longest list (C3: lists of U[0,64] values, half the lanes idle on
// float slots); this one gives every lane ~T/64 bytes. false = some value did not decode (or the
// start count disagrees with the counts): every eligible slot then takes the per-lane path, which
// rewrites its whole range (stores here never leave [dst, dst + c)).
template <bool COMPAT>
__device__ __forceinline__ bool int64_balanced(const FastSrc& fs, const DevOut& o, bool iv, uint32_t bo, uint32_t bl,
                                               uint32_t c, uint64_t dst, uint32_t lane) {
  const uint32_t len = iv ? bl : 0u, cnt = iv ? c : 0u;
  const uint32_t vend = wave_incl_scan_u32(len, lane);  // virtual end of slot k's body (lane k)
  const uint32_t T = __builtin_amdgcn_readlane(vend, 63);
  if (!T) return true;
  const uint32_t cend = wave_incl_scan_u32(cnt, lane);
  const uint32_t a = (uint32_t)(((uint64_t)lane * T) >> 6), b = (uint32_t)(((uint64_t)(lane + 1u) * T) >> 6);
  uint32_t k0 = 0;  // first slot whose body ends after a (vend is non-decreasing)
#pragma unroll
  for (uint32_t s = 32; s; s >>= 1)
    if ((uint32_t)__shfl((int)vend, (int)(k0 + s - 1u), 64) <= a) k0 += s;
  // pass 1: value starts in [a, b): position p of a body starts a value iff p == 0 or p-1 is a terminator
  uint32_t starts = 0, k = k0, x = a;
  while (__ballot(x < b)) {
    const uint32_t kk = k < 64u ? k : 63u;
    const uint32_t ve = (uint32_t)__shfl((int)vend, (int)kk, 64), vl = (uint32_t)__shfl((int)len, (int)kk, 64);
    const uint32_t ko = (uint32_t)__shfl((int)bo, (int)kk, 64);
    if (x < b && ve > x) {
      const uint32_t vb = ve - vl, pa = x - vb, pe = (b < ve ? b : ve) - vb;
      starts += (pa == 0u) + count_terms(fs.l, fs.p + ko, pa ? pa - 1u : 0u, pe - 1u);
      x = b < ve ? b : ve;
    }
    ++k;
  }
  const uint32_t incl = wave_incl_scan_u32(starts, lane);
  if (__builtin_amdgcn_readlane(incl, 63) != __builtin_amdgcn_readlane(cend, 63)) return false;
  // pass 2: decode the owned values
  uint32_t g = incl - starts;  // value starts before a
  bool bad = false;
  bool first = true;
  k = k0;
  x = a;
  while (__ballot(x < b)) {
    const uint32_t kk = k < 64u ? k : 63u;
    const uint32_t ve = (uint32_t)__shfl((int)vend, (int)kk, 64), vl = (uint32_t)__shfl((int)len, (int)kk, 64);
    const uint32_t ko = (uint32_t)__shfl((int)bo, (int)kk, 64);
    const uint32_t ce = (uint32_t)__shfl((int)cend, (int)kk, 64), cl = (uint32_t)__shfl((int)cnt, (int)kk, 64);
    const uint32_t dlo = (uint32_t)__shfl((int)(uint32_t)dst, (int)kk, 64);
    const uint32_t dhi = (uint32_t)__shfl((int)(uint32_t)(dst >> 32), (int)kk, 64);
    if (x < b && ve > x) {
      const uint32_t vb = ve - vl, pa = x - vb, pe = (b < ve ? b : ve) - vb;
      const uint64_t dk = ((uint64_t)dhi << 32) | dlo;
      uint32_t idx = first ? g - (ce - cl) : 0u;
      first = false;
      uint32_t pos = ko + pa;  // payload offset
      if (pa) {                // skip to the first start: after the first terminator at >= pa - 1
        const uint32_t q = ko + pa - 1u;
        const uint32_t t0 = ~fs.u32(q) & 0x80808080u, t1 = ~fs.u32(q + 4u) & 0x80808080u;
        const uint32_t t2 = ~fs.u32(q + 8u) & 0x80808080u;
        const uint32_t nt = t0 ? (__builtin_ctz(t0) >> 3) : t1 ? 4u + (__builtin_ctz(t1) >> 3)
                                                           : t2 ? 8u + (__builtin_ctz(t2) >> 3) : 12u;
        bad |= nt >= 12u;
        pos = q + nt + 1u;
      }
      const uint32_t pend = ko + pe;
      const uint32_t lim = dk + cl <= o.cap_i64 ? cl : (dk < o.cap_i64 ? (uint32_t)(o.cap_i64 - dk) : 0u);
      int64_t* out = o.i64 + dk;
      while (pos < pend) {  // (a failed varint still advances: the slot is redone per lane)
        int64_t v;
        bad |= !varint_bf<COMPAT>(fs, pos, v);
        if (idx < lim) out[idx] = v;
        ++idx;
      }
      x = b < ve ? b : ve;
    }
    ++k;
  }
  return !__ballot(bad);
}

// One varint at stage offset s whose length the caller has checked (1..10 bytes, its first byte
// < 0x80 is its last)
template <bool COMPAT>
__device__ __forceinline__ int64_t varint_term(const uint8_t* l, uint32_t s) {
  uint32_t w0, w1, w2;
  stage_w3(l, s, w0, w1, w2);
  int64_t v;
  (void)varint_w<COMPAT>(w0, w1, w2, v);
  return v;
}

// Canonical packed int64 lists of one staged record, value-parallel with COALESCED stores. In
// int64_balanced every lane decodes its own byte range, so one store instruction scatters 8-byte
// values over ~64 different lines (the gather's int64 part measured 1.12 of its 1.65 ms). Here
// pass A walks the stage span of the eligible bodies 256 bytes per step (lane j: aligned dword j),
// keeps the terminator bytes (< 0x80) inside a body and numbers them across the wave (three
// ballots + mbcnt), writing each one's stage offset (u16) and slot (u8) into a ring of kRingN in LDS:
// terminator g ends value g of the axis (the eligible slots in order). Pass B, as soon as 64 ends
// are pending, gives value gb + j to lane j: its end is ring[g], its start the slot's body start
// (first value) or ring[g - 1] + 1, the slot's parameters one ds_bpermute each; lanes j and j + 1
// then store neighbouring values of one slot. Requires the eligible bodies in increasing stage order
// with the slot index and 32-bit value positions (else -1: the caller takes int64_balanced). Every
// slot's last value must end on its body's last byte and the terminators must number exactly the
// counts (else 0: per-lane redo, which rewrites the whole range; stores here never leave
// [dst, dst + c)).
constexpr uint32_t kRingN = 324;  // 64 pending + 1 previous end + 256 of one pass-A step (+ pad)
// per wave in k_tail_gather: stage + ring (3 workgroups of 4 waves per CU, with LDS granularity)
constexpr uint32_t kWRegion = (kWStageStride + kRingN * 3u + 15u) & ~15u;  // (16-B aligned stages)

template <bool COMPAT>
__device__ __forceinline__ int int64_ring(const FastSrc& fs, const DevOut& o, bool iv, uint32_t bo, uint32_t bl,
                                          uint32_t c, uint64_t dst, uint32_t lane, uint16_t* ring) {
  const uint64_t m = __ballot(iv);
  if (!m) return 1;
  uint8_t* ring_k = reinterpret_cast<uint8_t*>(ring + kRingN);  // each entry's slot
  const uint32_t bs = fs.p + bo, be = bs + bl;  // stage offsets of the body
  const uint64_t lt = (1ull << lane) - 1ull;
  {  // physical order = slot order, and 32-bit value positions
    const uint64_t pm = m & lt;
    const int pl = pm ? 63 - __builtin_clzll(pm) : (int)lane;
    const uint32_t pbe = (uint32_t)__shfl((int)be, pl, 64);
    // (every value of the wave below 2^29 and inside the column: pass B's stores are the scalar
    // column base + a 32-bit byte offset, no per-value capacity test)
    if (__ballot(iv && ((pm && pbe > bs) || ((dst + c) >> 29) != 0u || dst + c > o.cap_i64))) return -1;
  }
  const uint32_t n = iv ? c : 0u;
  const uint32_t incl = wave_incl_scan_u32(n, lane);
  const uint32_t N = __builtin_amdgcn_readlane(incl, 63);
  const uint32_t pk_b = bs | (bl << 16), pk_c = (incl - n) | (n << 16), d32 = (uint32_t)dst;
  const uint32_t k_first = (uint32_t)__builtin_ctzll(m), k_last = 63u - (uint32_t)__builtin_clzll(m);
  const uint32_t Q0 = __builtin_amdgcn_readlane(bs, k_first) & ~3u, Qend = __builtin_amdgcn_readlane(be, k_last);
  const uint32_t* L32 = reinterpret_cast<const uint32_t*>(fs.l);
  uint32_t gtot = 0, rh = 0;  // terminators so far; ring slot of terminator gtot
  uint32_t gb = 0, rb = 0;    // values decoded so far; ring slot of value gb
  bool bad = false;
  auto pass_b = [&](uint32_t avail) {
    const bool act = lane < avail;
    uint32_t r = rb + lane;
    if (r >= kRingN) r -= kRingN;
    const uint32_t e = ring[r];
    const uint32_t ep = ring[r ? r - 1u : kRingN - 1u];
    const int k = (int)(ring_k[r] & 63u);
    const uint32_t pb = (uint32_t)__shfl((int)pk_b, k, 64), pc = (uint32_t)__shfl((int)pk_c, k, 64);
    const uint32_t pd = (uint32_t)__shfl((int)d32, k, 64);
    const uint32_t sbs = pb & 0xffffu, sbe = sbs + (pb >> 16), scn = pc >> 16;
    const uint32_t vi = gb + lane - (pc & 0xffffu);
    const uint32_t pe = e & 0xffffu;
    const uint32_t s = vi ? (ep & 0xffffu) + 1u : sbs;
    const uint32_t nb = pe + 1u - s;  // (wraps huge when pe < s)
    const bool ok = act && vi < scn && nb - 1u < 10u && (vi + 1u < scn || pe + 1u == sbe);
    bad |= act && !ok;
    const int64_t v = varint_term<COMPAT>(fs.l, ok ? s : 0u);
    const uint32_t at = pd + vi;  // (< 2^29)
    if (ok) *reinterpret_cast<int64_t*>(reinterpret_cast<uint8_t*>(o.i64) + (at << 3)) = v;
    gb += avail;
    rb += avail;
    if (rb >= kRingN) rb -= kRingN;
  };
  uint32_t wn = Q0 + 4u * lane < Qend ? L32[(Q0 >> 2) + lane] : 0u;  // (each step's dword read one step ahead)
  for (uint32_t Qw = Q0; Qw < Qend; Qw += 256u) {
    const uint32_t Q = Qw + 4u * lane;
    const uint32_t w = wn;
    wn = Q + 256u < Qend ? L32[(Q + 256u) >> 2] : 0u;
    // bytes [lo, hi) of this lane's dword inside an eligible body (bodies are >= 8 bytes apart: at
    // most one per dword) and its slot; the bodies overlapping the step from one ballot
    uint32_t bm = 0, ks = 0;
    for (uint64_t mw = __ballot(iv && bs < Qw + 256u && be > Qw); mw; mw &= mw - 1ull) {
      const uint32_t k = (uint32_t)__builtin_ctzll(mw);
      const uint32_t sbs = __builtin_amdgcn_readlane(bs, k), sbe = __builtin_amdgcn_readlane(be, k);
      const uint32_t lo = sbs > Q ? sbs - Q : 0u, hi0 = sbe > Q ? sbe - Q : 0u, hi = hi0 < 4u ? hi0 : 4u;
      if (hi > lo) {  // (1 <= hi <= 4, lo <= 3: both shifts below 32)
        bm = (0xffffffffu >> (32u - 8u * hi)) & (0xffffffffu << (8u * lo));
        ks = k;
      }
    }
    uint32_t t = ~w & 0x80808080u & bm;
    const uint32_t nt = (uint32_t)__popc(t);
    // this lane's first ring entry: terminators of the lanes below (three ballots of nt's bits)
    const uint64_t b0 = __ballot(nt & 1u), b1 = __ballot(nt & 2u), b2 = __ballot(nt & 4u);
    const uint32_t c0 = __builtin_amdgcn_mbcnt_hi((uint32_t)(b0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b0, rh));
    const uint32_t c1 = __builtin_amdgcn_mbcnt_hi((uint32_t)(b1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b1, 0u));
    const uint32_t c2 = __builtin_amdgcn_mbcnt_hi((uint32_t)(b2 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b2, 0u));
    const uint32_t at = c0 + 2u * c1 + 4u * c2;
    const uint32_t tot = (uint32_t)__popcll(b0) + 2u * (uint32_t)__popcll(b1) + 4u * (uint32_t)__popcll(b2);
    // its (up to 4) entries, unrolled (a loop ran to the wave's largest count with loop control)
#pragma unroll
    for (uint32_t i = 0; i < 4u; ++i) {
      if (!__ballot(i < nt)) break;  // (scalar)
      if (i < nt) {
        const uint32_t a0 = at + i, a = a0 >= kRingN ? a0 - kRingN : a0;
        ring[a] = (uint16_t)(Q + ((uint32_t)__builtin_ctz(t) >> 3));
        ring_k[a] = (uint8_t)ks;
        t &= t - 1u;
      }
    }
    gtot += tot;
    rh += tot;
    if (rh >= kRingN) rh -= kRingN;
    wave_lds_sync();
    while (gtot - gb >= 64u) pass_b(64u);
    wave_lds_sync();  // (pass B's reads before the next step's writes)
  }
  if (gtot > gb) pass_b(gtot - gb);
  wave_lds_sync();
  return (!__ballot(bad) && gtot == N) ? 1 : 0;
}

template <bool COMPAT>
__device__ __forceinline__ void stage_gather_group(const FastSrc& fs, const DevOut& o, bool present, uint32_t kind,
                                                   uint2 lc, uint32_t cnt, uint64_t dst, uint64_t lo16,
                                                   uint32_t lane, uint16_t* ring) {
  PHASE_MARK(g0);
  // every lane reads its own slot's chunk header up front: the wave loops below only readlane them
  uint32_t bo = 0, bl = 0;
  const bool packed = present && kind != TFRG_KIND_BYTES && hdr_0a_v(fs, lc.x, lc.y, bo, bl) &&
                      (kind != TFRG_KIND_FLOAT || !(bl & 3u));
  bool fail = present && kind != TFRG_KIND_BYTES && !packed;
  // canonical float lists: lane j moves value j (contiguous 4-byte stores), four lists per pass so
  // that four LDS reads are in flight before the stores
  // Per list, computed by its own lane (slot) first: the stage offset of its values, the last one's
  // offset, the values that fit the column and the column address; each list then takes one buffer
  // resource bounded at its fitting values, so a store past them is dropped by the hardware (no
  // per-value test, no exec-mask bookkeeping per list). The per-list work was scalar 64-bit
  // arithmetic (~30 SALU per list) and cost C3 as much as the copies.
  constexpr int kFG = 8;
  const bool isf = packed && kind == TFRG_KIND_FLOAT;
  uint64_t m = __ballot(isf);
  if (m) {
    // (lanes that are no float list hold zeros: a group past the last list re-reads lane 63, whose
    // stores are then either dropped (no values) or the same values again)
    const uint32_t fn_l = isf ? bl >> 2 : 0u, fb_l = fs.p + (isf ? bo : 0u), fo_l = fn_l ? 4u * (fn_l - 1u) : 0u;
    const uint64_t d_l = dst < o.cap_f32 ? dst : o.cap_f32;
    const uint32_t lim_l = o.cap_f32 - d_l < fn_l ? (uint32_t)(o.cap_f32 - d_l) : fn_l;
    const uint64_t a_l = reinterpret_cast<uint64_t>(o.f32 + d_l);
    const uint32_t j4 = 4u * lane;
    while (m) {
      uint32_t fb[kFG], fo[kFG];
      __amdgpu_buffer_rsrc_t rs[kFG];
      uint32_t nm = 0;
#pragma unroll
      for (int i = 0; i < kFG; ++i) {
        const int k = __builtin_ctzll(m | (1ull << 63));
        m &= m - 1ull;
        const uint32_t fn = __builtin_amdgcn_readlane(fn_l, k), lim = __builtin_amdgcn_readlane(lim_l, k);
        fb[i] = __builtin_amdgcn_readlane(fb_l, k);
        fo[i] = __builtin_amdgcn_readlane(fo_l, k);
        const uint64_t a = readlane_u64(a_l, k);  // (readlane returns int: a plain OR would sign-extend)
        rs[i] = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(a), (short)0, (int)(4u * lim), 0x00020000);
        nm = nm > fn ? nm : fn;
      }
      for (uint32_t j = 0; j < nm; j += 64) {  // (wave-uniform)
        const uint32_t off = 4u * j + j4;
        uint32_t x[kFG];
#pragma unroll
        for (int i = 0; i < kFG; ++i) x[i] = lds_u32u(fs.l, fb[i] + (off < fo[i] ? off : fo[i]));
#pragma unroll
        for (int i = 0; i < kFG; ++i) __builtin_amdgcn_raw_buffer_store_b32(x[i], rs[i], off, 0, 0);
      }
    }
  }
  PHASE_MARK(gf);
  PHASE_ADD(15, g0, gf);
  // canonical packed int64 lists: balanced over the whole wave
  const bool iv = packed && kind == TFRG_KIND_INT64 && bl > 0u && fs.l[fs.p + bo + bl - 1u] < 0x80u;
  fail |= packed && kind == TFRG_KIND_INT64 && !iv;
  int rr = int64_ring<COMPAT>(fs, o, iv, bo, bl, cnt, dst, lane, ring);
  if (rr < 0) rr = int64_balanced<COMPAT>(fs, o, iv, bo, bl, cnt, dst, lane) ? 1 : 0;
  if (!rr) fail |= iv;
  PHASE_MARK(g1);
  PHASE_ADD(11, gf, g1);
  if (present && (kind == TFRG_KIND_BYTES || fail)) {
    if (!fast_list_gather<COMPAT>(fs, o, kind, lc.x, lc.y, dst)) {
      LdsSrc s;
      s.init(fs.l, lo16, fs.base, fs.L);
      list_gather<COMPAT>(s, o, (int)kind, (int64_t)lc.x, (int64_t)lc.y, dst);
    }
  }
  PHASE_MARK(g2);
  PHASE_ADD(12, g1, g2);
}

// Medium records, one wave each, staged in LDS. The next record's bytes are loaded into registers
// while this one is gathered (48 VGPRs live across the gather).
template <bool COMPAT>
__device__ void role_stage_gather(const DevBatch& B, const DevSchema& sc, const DevOut& o, uint8_t* stage,
                                  uint16_t* ring, uint64_t placed) {
  const uint32_t lane = threadIdx.x & 63u, wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // Each XCD takes one contiguous eighth of the list (workgroups b and b + 8 share an XCD): the
  // slot metadata of neighbouring records shares 128-byte lines ([slot][n] columns), which its L2
  // then fetches once instead of once per XCD
  // (grids of fewer than 8 workgroups: one range)
  const uint32_t nall = o.info[kInfoBig];
  const uint32_t nx = gridDim.x >= 8u ? 8u : 1u;
  const uint32_t xcd = blockIdx.x % nx, nbx = (gridDim.x - xcd + nx - 1u) / nx;
  const uint32_t i0 = (uint32_t)((uint64_t)nall * xcd / nx), nbig = (uint32_t)((uint64_t)nall * (xcd + 1u) / nx);
  const uint32_t w0 = i0 + (blockIdx.x / nx) * kWavesPerBlock + wib;
  if (w0 >= nbig) return;  // wave-uniform: no records for this wave
  const uint32_t stride = nbx * kWavesPerBlock;
  uint32_t i = w0;
  RecPipe q;
  q.r1 = i < nbig ? o.big_list[i] : 0u;
  q.s1 = rec_start(B, q.r1);
  q.e1 = rec_end(B, q.r1);
  q.t1 = i < nbig ? o.status[q.r1] : -1;
  Pref pf = pref_load_v(B.bytes, q.s1 & ~15ull, q.t1 == TFRG_OK ? (q.e1 < B.nbytes ? q.e1 : B.nbytes) : 0ull, lane);
  q.r2 = i + stride < nbig ? o.big_list[i + stride] : 0u;
  q.s2v = rec_start(B, vgpr_launder(q.r2));
  q.e2v = rec_end(B, vgpr_launder(q.r2));
  q.t2v = o.status[vgpr_launder(q.r2)];
  q.r3v = o.big_list[vgpr_launder(i + 2 * stride < nbig ? i + 2 * stride : 0u)];
  // per-slot constants, and the slot metadata of the NEXT record loaded one record ahead (its
  // latency then hides behind this record's gather instead of opening every record)
  // (slots placed by k_tpl_lane: their count words are unwritten for its records)
  const bool sl = lane < sc.n_slots && !((placed >> lane) & 1ull);
  const uint32_t kind_l = sl ? (uint32_t)sc.slot_kind[lane] : 0u;
  const uint64_t sbase_l = sl ? o.slot_base[lane] : 0ull;
  uint32_t c_n = 0, rs_n = 0;
  uint2 lc_n = make_uint2(0, 0);
  auto meta_load = [&](uint32_t rr, bool okr) {
    c_n = 0;
    rs_n = 0;
    lc_n = make_uint2(0, 0);
    if (okr && sl) {
      const size_t at = (size_t)lane * B.n + rr;
      c_n = o.count[at];
      lc_n = o.loc[at];
      rs_n = o.rs[(size_t)lane * (B.n + 1) + rr];
    }
  };
  meta_load(q.r1, q.t1 == TFRG_OK);
  for (; i < nbig; i += stride) {
    PHASE_MARK(t0);
    const uint32_t r = q.r1;
    const bool ok = q.t1 == TFRG_OK;
    const RecView v = rec_view_se(B, q.s1, q.e1);
    const uint64_t lo16 = v.st & ~15ull;
    if (ok) pref_store(pf, stage, lo16, v.e, lane);
    wave_lds_sync();
    // slot metadata of this record (loaded during the previous one)
    const uint32_t c = c_n, kind = kind_l;
    const uint2 lc = lc_n;
    const uint64_t dst = sbase_l + rs_n;
    bool present = c && !(c & kCountInline);  // inline single values are k_down_gather's
    q.r1 = q.r2;
    q.s1 = rfl64(q.s2v);
    q.e1 = rfl64(q.e2v);
    q.t1 = i + stride < nbig ? (int32_t)rfl32((uint32_t)q.t2v) : -1;
    q.r2 = rfl32(q.r3v);
    q.r3v = o.big_list[vgpr_launder(i + 3 * stride < nbig ? i + 3 * stride : 0u)];
    pf = pref_load_v(B.bytes, q.s1 & ~15ull, q.t1 == TFRG_OK ? (q.e1 < B.nbytes ? q.e1 : B.nbytes) : 0ull, lane);
    q.s2v = rec_start(B, vgpr_launder(q.r2));
    q.e2v = rec_end(B, vgpr_launder(q.r2));
    q.t2v = o.status[vgpr_launder(q.r2)];
    meta_load(q.r1, q.t1 == TFRG_OK);
    if (!ok) continue;  // wave-uniform
    PHASE_MARK(t1);
    PHASE_ADD(9, t0, t1);
    if (present && !loc_in_record(lc, v.L)) {  // (lane = slot)
      loc_fail(o, r, lane, lc);
      present = false;
    }
    const FastSrc fs{stage, (uint32_t)(v.p0 - lo16), (uint32_t)v.L, v.p0};
    stage_gather_group<COMPAT>(fs, o, present, kind, lc, c, dst, lo16, lane, ring);
    for (uint32_t kb = 64; kb < sc.n_slots; kb += 64) {  // wide schemas: further groups of 64 slots
      const uint32_t k = kb + lane;
      bool pk = false;
      uint32_t kk = 0, ck = 0;
      uint2 lk = make_uint2(0, 0);
      uint64_t dk = 0;
      if (k < sc.n_slots) {
        const size_t at = (size_t)k * B.n + r;
        ck = o.count[at];
        pk = ck && !(ck & kCountInline);
        lk = o.loc[at];
        dk = o.slot_base[k] + o.rs[(size_t)k * (B.n + 1) + r];
        kk = sc.slot_kind[k];
        if (pk && !loc_in_record(lk, v.L)) {
          loc_fail(o, r, k, lk);
          pk = false;
        }
      }
      stage_gather_group<COMPAT>(fs, o, pk, kk, lk, ck, dk, lo16, lane, ring);
    }
    wave_lds_sync();
    PHASE_MARK(t2);
    PHASE_ADD(10, t1, t2);
  }
}

// The gathers after the row-split scan in ONE launch, each wave independent (no workgroup barrier):
// out-of-line lists of lane records (role list), records above lane_max staged in LDS (role stage),
// huge records from HBM (role wave). Every role uses the wave's stage region of kWStageStride bytes.
template <bool COMPAT>
__global__ __launch_bounds__(kWaveBlock) void k_tail_gather(DevBatch B, DevSchema sc, DevOut o, uint32_t lane_max) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const uint32_t wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* stage = reinterpret_cast<uint8_t*>(lds) + wib * kWRegion;
  uint16_t* ring = reinterpret_cast<uint16_t*>(stage + kWStageStride);  // (int64_ring)
  if (blockIdx.x == 0)  // (read by k_down_gather, which has finished: zero for the next decode)
    for (uint32_t k = threadIdx.x; k < sc.n_slots; k += kWaveBlock) o.irr[k] = 0u;
  // the slots whose speculative placement is final (k_down_gather's mask; irr is cleared above)
  const uint64_t placed = ((uint64_t)o.info[kInfoPlacedHi] << 32) | o.info[kInfoPlacedLo];
  role_list_gather<COMPAT>(B, sc, o, lane_max, stage, placed);
  role_stage_gather<COMPAT>(B, sc, o, stage, ring, placed);
  role_wave_gather<COMPAT>(B, sc, o, placed);
}

// Debug hook (tfrg_ctx: env TFRG_DEBUG_POISON_LOC at context creation): after the count passes,
// the list locations of up to 4 records are overwritten with a location far outside any record, as
// a stale or corrupt word would be; the gathers must then fail those records (TFRG_ST_INTERNAL).
__global__ void k_poison_loc(DevOut o, uint32_t n, uint32_t n_slots, uint4 recs) {
  const uint32_t rr[4] = {recs.x, recs.y, recs.z, recs.w};
  for (uint32_t k = threadIdx.x; k < n_slots; k += blockDim.x)
    for (int i = 0; i < 4; ++i)
      if (rr[i] < n) o.loc[(size_t)k * n + rr[i]] = make_uint2(0xfffff000u, 0x00ffffffu);
}

// ------------------------------------------------------------------------------------------------
// launcher
// ------------------------------------------------------------------------------------------------
constexpr int kLaneRep = 1;  // CRC table bank replication in the lane kernel (slice-by-8: 8 KiB per copy)

constexpr size_t kLaneLdsBudget = 64 * 1024; // lane kernels (occupancy): likewise

const char* const kStageNames[kNumStages] = {"k_tpl_lane",    "k_lane_count",  "k_body_count", "k_tail_count", "k_spine",
                                             "k_down_gather", "k_tail_gather", "k_bytes"};

static inline size_t r16(size_t x) { return (x + 15) & ~(size_t)15; }

template <bool COMPAT>
static hipError_t launch_all(const DevBatch& b, const DevSchema& sc, const DevOut& o, LaunchCfg& cfg,
                             const uint32_t* d_tab, const uint32_t* d_consts, hipStream_t st, hipEvent_t* ev) {
  auto mark = [&](int i) {
    if (ev) (void)hipEventRecord(ev[i], st);
  };
  const size_t S = sc.n_slots;
  const uint32_t n_tiles = (b.n + kTileRecs - 1) / kTileRecs;
  const size_t dict_lane = S * kLaneCountBlock * 4 + r16(S * kLaneCountBlock * 2);  // cnt u32 + ord u16 per lane
  const size_t tab_lds = 256ull * kLaneSlice * kLaneRep * 4;
  const size_t stage_lds = (size_t)kStageStride * (kLaneCountBlock / 64);
  const bool fast_ok = sc.n_keys <= kLdsMaxKeys && sc.ht_mask + 1 <= kLdsMaxHt;
  const size_t keys_lds = fast_ok ? (((size_t)sc.ht_mask + 4) / 4 * 4 + (size_t)sc.n_keys * kKrWords) * 4 : 0;
  // (MODE 0 only) spec words + their targets
  const size_t spec_lds = fast_ok && sc.spec ? ((S + 7) & ~(size_t)7) * 4 + S * kSpecTgtWords * 4 : 0;
  const size_t lane_lds = tab_lds + dict_lane + stage_lds + keys_lds + spec_lds;
  // speculative placement only with the per-lane LDS dict (MODE 0); the later kernels see the same
  DevSchema scx = sc;
  if (lane_lds > kLaneLdsBudget || !fast_ok) scx.spec = nullptr;
  const uint32_t wave_stage = cfg.wave_stage < kWStage ? cfg.wave_stage : kWStage;
  // record-shape templates first (k_tpl_lane, tfrg_tpl.hip): framed records with CRC verdicts, a
  // schema of <= kLeanMaxSlots slots; k_lane_count then takes only the records it left
  const bool lean = cfg.lean && sc.n_tpl && fast_ok && S <= kLeanMaxSlots && o.lmask && o.rlist &&
                    (sc.tpl_w == 16 || sc.tpl_w == 32 || sc.tpl_w == 64) &&
                    !(b.flags & (kFlagPayloadOnly | kFlagNoCrc)) && b.nbytes < 0xffffff00ull;
  // every record of the learning sample took a template and none is above lane_max: the passes after
  // k_tpl_lane (residual lane records, slow walks, large-record CRCs, gathers of placed slots) are
  // usually empty, and a full grid of workgroups that exit at once costs ~4 us per launch; they
  // run with small grids instead (any work they do find is still done: every one strides)
  const bool quiet = lean && cfg.tpl_full && !cfg.body_count;
  // every slot speculatively placed (DevSchema::spec, a target for each)
  bool all_spec = scx.spec && cfg.spec_h && S <= 64;
  for (size_t k = 0; all_spec && k < S; ++k) all_spec = cfg.spec_h[k] != 0u;
  // Optimistic: quiet with every slot placed (C1-shaped batches). A batch all of whose records take a
  // template is complete after k_tpl_lane; the passes after it would only launch. The last
  // workgroup of k_tpl_lane does their bookkeeping (tpl_quiet_finish), or flags the batch for a full
  // re-run by the host (tfrg_result_info) if a record took no template. Saves five dependent
  // launches (~4 us each) per batch.
  cfg.ran_optimistic = cfg.optimistic && quiet && all_spec && S > 0;
  // Optimistic without record shapes (C2: records above lane_max, every slot one inline value in the
  // learning sample, placed speculatively by k_lane_count MODE 0): k_lane_count, k_tail_count, and
  // the last workgroup of k_tail_count ends the decode (tail_quiet_finish) or flags it for a full
  // re-run. Not in strict mode (a CRC failure withdraws a record's columns).
  const bool quiet_big = cfg.optimistic && !lean && all_spec && S > 0 && lane_lds <= kLaneLdsBudget && fast_ok &&
                         cfg.body_count && !(b.flags & kFlagStrictCrc) && b.n > 0;
  cfg.ran_optimistic |= quiet_big;
  cfg.ran_quiet_big = quiet_big;
  // k_tail_count's LDS (role 1's per-lane dicts for kTailBlock threads, else its global-dict form;
  // role 2's tables and the finishing words)
  const size_t slow_tail = 2048ull * 4 + S * kTailBlock * 4 + r16(S * kTailBlock * 2);
  const bool tail_gord = slow_tail > kLaneLdsBudget;
  const size_t tail_lds = std::max<size_t>(tail_gord ? 2048ull * 4 : slow_tail, (kTailFinishWord + 4) * 4);
  // quiet_big: the records above lane_max walked beside the streaming CRC by k_tail_count's first
  // workgroups (role_big_walk) when its per-lane dicts fit the launch's LDS
  const size_t walk_lds = 256ull * kLaneSlice * 4 + S * kTailBlock * 4 + r16(S * kTailBlock * 2) + keys_lds + spec_lds;
  const bool walk_beside = quiet_big && cfg.walk_beside && walk_lds <= tail_lds;
  cfg.implicit = 0;
  DevOut ox = o;
  if (!lean) {
    ox.lmask = nullptr;
    ox.rlist = nullptr;
  }
  mark(kStageTplLane);
  if (lean) {
    LeanArgs a{};
    a.n_tpl = sc.n_tpl;
    a.img_words = sc.tpl_img_words;
    a.lane_max = cfg.lane_max;
    a.tsum = cfg.ran_optimistic ? nullptr : o.tsum;  // (placed slots: no scan; a re-run clears tsum)
    a.finish = cfg.ran_optimistic ? sc.slot_kind : nullptr;
    // (optimistic: status / verdict and constant order words are implicit, tfrg_info.implicit_cols)
    cfg.implicit = cfg.ran_optimistic ? TFRG_IMPLICIT_STATUS | (cfg.ord_const ? TFRG_IMPLICIT_ORDER : 0u) |
                                            (cfg.len_const ? TFRG_IMPLICIT_BYTES_LEN : 0u)
                                      : 0u;
    a.implicit = cfg.implicit;
    a.n_slots = (uint32_t)S;
    a.tile_stride = o.tile_stride;
    const uint64_t n = b.n;
    for (uint32_t k = 0; k < S; ++k) {
      LeanTgt& t = a.tg[k];
      t.ord = o.order + k * n;
      t.cnt = o.count + k * n;
      t.loc = o.loc + k * n;
      t.rs = o.rs + k * (n + 1);
      const uint32_t sw = scx.spec && cfg.spec_h ? cfg.spec_h[k] : 0u;
      if (sw) {  // as spec_target: column rows n * (rank - 1) + r, r below the capacity
        const uint32_t kind = sw & 3u;
        const uint64_t base = n * ((sw >> 2) - 1u);
        const uint64_t cap = kind == TFRG_KIND_INT64 ? o.cap_i64 : kind == TFRG_KIND_FLOAT ? o.cap_f32 : o.cap_b;
        t.lim = cap > base ? (uint32_t)std::min<uint64_t>(cap - base, n) : 0u;
        t.kind = kind;
        if (kind == TFRG_KIND_INT64) t.v1 = o.i64 + base;
        else if (kind == TFRG_KIND_FLOAT) t.v1 = o.f32 + base;
        else t.v1 = o.b_off + base;
        t.v2 = o.b_len + base;
      }
    }
    const hipError_t e = launch_tpl_lane(b, ox, a, sc.tpl_img, sc.tpl_w, d_tab, cfg.num_cus, st);
    if (e != hipSuccess) return e;
  }
  if (cfg.ran_optimistic && !quiet_big) {  // (k_tpl_lane's last workgroup finished the decode)
    for (int i = kStageLaneCount; i <= kStageMaterialize; ++i) mark(i);
    return hipGetLastError();
  }
  mark(kStageLaneCount);
  // one round of resident workgroups (a second, partial round would idle most CUs at the tail)
  auto resident_grid = [&](const void* fn, size_t lds, bool cap = true) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kLaneCountBlock, lds) != hipSuccess || per_cu < 1)
      per_cu = 1;
    const int g = per_cu * cfg.num_cus;
    int need = (int)(((int64_t)cfg.lane_grid * 256 + kLaneCountBlock - 1) / kLaneCountBlock);
    // (after a template pass that took its whole sample the residual pass is usually empty; it
    // strides over whatever groups it finds. Not for records above lane_max: k_tpl_lane leaves
    // every one of them, and walking them is this pass's work)
    if (quiet) need = std::min(need, 64);
    return g < need || !cap ? g : need;
  };
  if (lane_lds <= kLaneLdsBudget) {
    const void* fn = reinterpret_cast<const void*>(&k_lane_count<kLaneRep, COMPAT, 0>);
    hipLaunchKernelGGL((k_lane_count<kLaneRep, COMPAT, 0>), dim3(resident_grid(fn, lane_lds - tab_lds)),
                       dim3(kLaneCountBlock), lane_lds - tab_lds, st, b, scx, ox, d_tab, cfg.lane_max, wave_stage,
                       walk_beside ? 1u : 0u);
  } else if (S <= 64) {
    const size_t lds = stage_lds + keys_lds + (kLaneCountBlock / 64) * 64 * 4;  // (+ the static tables)
    const void* fn = reinterpret_cast<const void*>(&k_lane_count<kLaneRep, COMPAT, 1>);
    hipLaunchKernelGGL((k_lane_count<kLaneRep, COMPAT, 1>), dim3(resident_grid(fn, lds)), dim3(kLaneCountBlock), lds,
                       st, b, scx, ox, d_tab, cfg.lane_max, wave_stage, 0u);
  } else {
    const size_t lds = stage_lds + keys_lds;  // (+ the static tables)
    const void* fn = reinterpret_cast<const void*>(&k_lane_count<kLaneRep, COMPAT, 2>);
    hipLaunchKernelGGL((k_lane_count<kLaneRep, COMPAT, 2>), dim3(resident_grid(fn, lds)), dim3(kLaneCountBlock), lds,
                       st, b, scx, ox, d_tab, cfg.lane_max, wave_stage, 0u);
  }
  mark(kStageBodyCount);
  if (cfg.body_count && lane_lds > kLaneLdsBudget) {  // deferred bodies (lane modes 1 and 2 only)
    const uint32_t g = 8u * (uint32_t)cfg.num_cus;
    hipLaunchKernelGGL(k_body_count, dim3(g), dim3(kBodyBlock), 0, st, b, ox);
  }
  mark(kStageTailCount);
  // the exception paths before the scan: one launch, one round of resident workgroups (role 2 splits
  // the large payloads evenly over the waves; role 1 grid-strides over the slow list)
  {
    const bool gord = tail_gord;
    const size_t lds = tail_lds;
    const void* fn = gord ? reinterpret_cast<const void*>(&k_tail_count<COMPAT, true>)
                          : reinterpret_cast<const void*>(&k_tail_count<COMPAT, false>);
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kTailBlock, lds) != hipSuccess || per_cu < 1)
      per_cu = 1;
    // (a small batch: fewer workgroups -- both roles stride -- so that an empty launch, the usual case
    // of batches of small records, is not a full grid of dispatches)
    uint32_t g = std::min((uint32_t)(per_cu * cfg.num_cus), std::max(8u, (uint32_t)(b.nbytes >> 16) + b.n / 4096u));
    if (!cfg.body_count) g = std::min(g, 32u);  // (no record above lane_max: role 2 has nothing to stream)
    const uint32_t fin = quiet_big ? 1u : 0u;
    // the walking workgroups: one 64-record group per wave, at most 1/32 of the grid (the streaming
    // CRC is bound by its workgroups' issue rate: each one it loses costs it 1/g of its time, while a
    // walking wave takes several groups well within the CRC's time). Every workgroup of the grid is
    // resident, the walkers dispatched first.
    uint32_t wb = 0;
    if (walk_beside) {
      if (g < 2u) g = 2u;
      const uint32_t ng = (uint32_t)((b.n + 63) / 64);
      const uint32_t cap = cfg.walk_blocks ? cfg.walk_blocks : std::max(1u, g / 32u);
      wb = std::max(1u, std::min({(ng + kTailBlock / 64 - 1) / (kTailBlock / 64), cap, g - 1u}));
    }
    if (gord)
      hipLaunchKernelGGL((k_tail_count<COMPAT, true>), dim3(g), dim3(kTailBlock), lds, st, b, scx, ox, d_tab, d_consts,
                         cfg.lane_max, fin, wb);
    else
      hipLaunchKernelGGL((k_tail_count<COMPAT, false>), dim3(g), dim3(kTailBlock), lds, st, b, scx, ox, d_tab,
                         d_consts, cfg.lane_max, fin, wb);
  }
  if (quiet_big) {  // (k_tail_count's last workgroup finished the decode)
    for (int i = kStageSpine; i <= kStageMaterialize; ++i) mark(i);
    return hipGetLastError();
  }
  if (cfg.poison[0] != 0xffffffffu && S > 0)
    hipLaunchKernelGGL(k_poison_loc, dim3(1), dim3(64), 0, st, ox, b.n, (uint32_t)S,
                       make_uint4(cfg.poison[0], cfg.poison[1], cfg.poison[2], cfg.poison[3]));
  mark(kStageSpine);
  if (S > 0)
    hipLaunchKernelGGL(k_spine, dim3(o.n_chunks * (uint32_t)S), dim3(kSpineBlock), 0, st, ox, sc.slot_kind, (uint32_t)S, n_tiles,
                       scx.spec, b.n);
  mark(kStageDownGather);
  if (S > 0) {
    // (at most 8 resident 256-thread workgroups per CU; larger batches stride). Every slot with a
    // speculative target: usually all placed and nothing to do but the launch, one per CU (a failed
    // placement strides over the tiles)
    // (all placed: usually nothing to do but the launch; a small batch also strides with fewer)
    uint32_t resident = all_spec ? std::min((uint32_t)cfg.num_cus, std::max(8u, n_tiles / 4u)) : 8u * (uint32_t)cfg.num_cus;
    if (all_spec && quiet) resident = std::min(resident, 32u);
    if (n_tiles >= 16u * (uint32_t)cfg.num_cus) {
      const uint32_t ng = (n_tiles + 3) / 4;
      hipLaunchKernelGGL((k_down_gather<COMPAT, 4>), dim3(ng < resident ? ng : resident), dim3(kLaneBlock), 0, st, b,
                         scx, ox, cfg.lane_max, n_tiles);
    } else {
      hipLaunchKernelGGL((k_down_gather<COMPAT, 1>), dim3(n_tiles < resident ? n_tiles : resident), dim3(kLaneBlock),
                         0, st, b, scx, ox, cfg.lane_max, n_tiles);
    }
  }
  mark(kStageTailGather);
  bool all_spec_t = scx.spec && cfg.spec_h && S <= 64;
  for (size_t k = 0; all_spec_t && k < S; ++k) all_spec_t = cfg.spec_h[k] != 0u;
  if (S > 0) {  // the gathers after the scan: lane records' lists, staged and huge large records
    const size_t lds = (size_t)kWRegion * kWavesPerBlock;
    const void* fn = reinterpret_cast<const void*>(&k_tail_gather<COMPAT>);
    int per_cu = 0;  // one round of resident workgroups (3 per CU: a second round would run at 1/3)
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kWaveBlock, lds) != hipSuccess || per_cu < 1)
      per_cu = 1;
    int g = per_cu * cfg.num_cus < cfg.wave_grid ? per_cu * cfg.num_cus : cfg.wave_grid;
    // (a small batch: its roles stride over fewer waves; large records keep the full grid)
    g = (int)std::min<uint64_t>((uint64_t)g, std::max<uint64_t>(8u, std::max<uint64_t>(b.n / 1024u, b.nbytes >> 16)));
    if (quiet && all_spec_t) g = std::min(g, 32);
    hipLaunchKernelGGL((k_tail_gather<COMPAT>), dim3(g), dim3(kWaveBlock), lds, st, b, scx, ox, cfg.lane_max);
  }
  mark(kStageMaterialize);  // (the caller launches the optional materialize pass and marks the end)
  return hipGetLastError();
}

hipError_t launch_decode(const DevBatch& b, const DevSchema& sc, const DevOut& o, LaunchCfg& cfg,
                         const uint32_t* d_tab, const uint32_t* d_consts, hipStream_t st, hipEvent_t* ev) {
  if (b.flags & kFlagSpecVarint) return launch_all<false>(b, sc, o, cfg, d_tab, d_consts, st, ev);
  return launch_all<true>(b, sc, o, cfg, d_tab, d_consts, st, ev);
}

// Row splits of the finally placed slots (tfrg_info.placed_slots: the identity 0..n, never stored by
// the decode) written into the device columns, for tfrg_result_device's view; the placed mask is
// read from the decode's info words on the device (no host round trip).
__global__ __launch_bounds__(256) void k_fill_placed_rows(uint32_t* __restrict__ rs, const uint32_t* __restrict__ info,
                                                          uint32_t n_slots, uint32_t n) {
  const uint64_t placed = ((uint64_t)info[kInfoPlacedHi] << 32) | info[kInfoPlacedLo];
  const uint32_t k = blockIdx.y;
  if (k >= 64u || k >= n_slots || !((placed >> k) & 1ull)) return;
  uint32_t* row = rs + (size_t)k * (n + 1u);
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i <= n; i += gridDim.x * 256u) row[i] = i;
}

hipError_t launch_fill_placed_rows(uint32_t* rs, const uint32_t* info, uint32_t n_slots, uint32_t n, hipStream_t st) {
  const uint32_t slots = n_slots < 64u ? n_slots : 64u;
  if (!slots) return hipSuccess;
  const uint32_t blocks = (n + 1u + 255u) / 256u;
  hipLaunchKernelGGL(k_fill_placed_rows, dim3(blocks < 1024u ? blocks : 1024u, slots), dim3(256), 0, st, rs, info,
                     n_slots, n);
  return hipGetLastError();
}

// Streaming read (measurement only): each block reads a contiguous slab, U 16-byte loads in flight
// per lane (all issued before any is consumed), nontemporal (the data is not reused).
typedef uint32_t sr_u32x4 __attribute__((ext_vector_type(4)));
template <int U>
__global__ __launch_bounds__(256) void k_stream_read(const sr_u32x4* __restrict__ p, uint64_t n16, uint32_t* sink) {
  uint32_t acc = 0;
  const uint64_t per_block = (n16 + gridDim.x - 1) / gridDim.x;
  const uint64_t b0 = (uint64_t)blockIdx.x * per_block;
  const uint64_t b1 = b0 + per_block < n16 ? b0 + per_block : n16;
  uint64_t i = b0 + threadIdx.x;
  for (; i + (U - 1) * 256 < b1; i += U * 256) {
    sr_u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(p + i + u * 256);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (; i < b1; i += 256) {
    const sr_u32x4 a = p[i];
    acc ^= a.x ^ a.y ^ a.z ^ a.w;
  }
  if (acc == 0x9e3779b9u) atomicXor(sink, acc);  // practically never taken; keeps the loads live
}

// variant: 0 = 4 loads in flight, 16 blocks per CU; 1 = 8 loads, 8 blocks per CU; 2 = 8 loads, 16
// blocks per CU; 3 = 16 loads, 4 blocks per CU (bench.py reports the fastest)
hipError_t launch_stream_read(const void* d, uint64_t nbytes, uint32_t* sink, hipStream_t st, int variant) {
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const sr_u32x4* q = static_cast<const sr_u32x4*>(d);
  switch (variant) {
    case 0: hipLaunchKernelGGL(k_stream_read<4>, dim3(cus * 16), dim3(256), 0, st, q, nbytes / 16, sink); break;
    case 1: hipLaunchKernelGGL(k_stream_read<8>, dim3(cus * 8), dim3(256), 0, st, q, nbytes / 16, sink); break;
    case 2: hipLaunchKernelGGL(k_stream_read<8>, dim3(cus * 16), dim3(256), 0, st, q, nbytes / 16, sink); break;
    default: hipLaunchKernelGGL(k_stream_read<16>, dim3(cus * 4), dim3(256), 0, st, q, nbytes / 16, sink); break;
  }
  return hipGetLastError();
}

}  // namespace tfrg

#ifdef TFRG_PHASE_PROF
extern "C" int tfrg_debug_phase(unsigned long long* out, int n, int reset) {
  if (n > 32) n = 32;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(tfrg::g_phase), n * sizeof(unsigned long long)) != hipSuccess) return -2;
  if (reset) {
    unsigned long long z[32] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(tfrg::g_phase), z, sizeof(z)) != hipSuccess) return -2;
  }
  return n;
}
#endif
