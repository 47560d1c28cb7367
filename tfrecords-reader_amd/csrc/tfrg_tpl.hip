// tfrg_tpl.hip — k_tpl_lane: the record-shape template path of the lane-per-record decode (gfx950).
//
// Records of one file almost always share one structure: the same keys in the same order with the
// same header bytes; only list contents differ (tfrg_internal.h, "Record-shape template"). For such
// a record the reference's whole decode (decoder.pyx:107-300: Example -> Features -> map entries ->
// Feature -> list) yields the template's dict, and the TFRecord framing checks reduce to constants:
// the length field and its masked CRC-32C are template bytes, and the payload CRC-32C is
// K ^ lin(variable bits) with lin linear (crc32c.h). So a lane takes its record as a fixed set of
// words and does constant work, no walk:
//   * the last 4 W bytes of the record [end - 4 W, end) -> W VGPRs, W / 4 unaligned 16-byte buffer
//     loads straight from HBM (no LDS stage; out-of-range offsets read zeros);
//   * match: (word ^ Bm) & Mm == 0 over the window (two VALU per word, template words in SGPRs);
//   * CRC: one LDS lookup per variable payload byte in the position tables T_d (d = the byte's
//     distance from the payload end, slice-by-32 tables), XOR-combined; variable bits further than
//     32 bytes from the end first run a slice-by-4 chain whose state joins at distance 28..31;
//   * the dict into the columns, ONE store per column and 64-record group whatever template each
//     lane took: per slot, every template with hits in the group contributes its lanes' order,
//     count / loc or speculatively placed value (DevSchema::spec; the row split r implicit), taken
//     from the window registers at the template's (wave-uniform) position, and a select keeps each
//     lane's own; then the per-tile value counts.
// A wave owns a contiguous range of groups (whole tiles, or half a tile on small batches).
// A record no template takes (another shape, a framing or CRC mismatch) is left to k_lane_count:
// per 64-record group a miss mask (DevOut::lmask) and a list of the groups with misses
// (DevOut::rlist).
#include <hip/hip_runtime.h>
#include "tfrg_internal.h"
#include "crc32c.h"
#include "../../include/tfrg_status.h"

namespace tfrg {

namespace {

constexpr int kTplBlock = 512;        // 8 waves: the 32 KiB of tables are shared by 8 waves
constexpr uint32_t kTplTabs = 32;     // T_0 .. T_31
static_assert(4u * kTplTabs * 256u + 4u * kLiMaxWords + 512u <= 65536u, "lane image + CRC tables exceed LDS");
constexpr uint32_t kHitVerdict = TFRG_V_LEN_MATCH | TFRG_V_LEN_CRC | TFRG_V_DATA_CRC;

typedef __attribute__((address_space(4))) const uint32_t cu32;  // wave-uniform reads -> s_load

__device__ __forceinline__ uint32_t rfl(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

// ((x >> 8K) & 0xff) * 4 in one VALU (a shift with an SDWA byte select of its source)
template <int K>
__device__ __forceinline__ uint32_t bx4(uint32_t x) {
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

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// table T_d at byte address bx of the static table array (d a compile-time constant: the table base
// folds into the ds_read offset)
template <int D>
__device__ __forceinline__ uint32_t tl(const uint32_t* tab, uint32_t bx) {
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(tab) + D * 1024 + bx);
}

// linear CRC contribution of a word whose 4 bytes sit at distances D+3, D+2, D+1, D from the payload end
template <int D>
__device__ __forceinline__ uint32_t lin_word(const uint32_t* tab, uint32_t x) {
  return xor3(tl<D + 3>(tab, bx4<0>(x)), tl<D + 2>(tab, bx4<1>(x)), tl<D + 1>(tab, bx4<2>(x))) ^ tl<D>(tab, bx4<3>(x));
}

// 7-bit groups of the bytes of w selected by byte mask m, compacted (a varint of <= 4 bytes)
__device__ __forceinline__ uint32_t vgroups(uint32_t w, uint32_t m) {
  w &= m;
  return (w & 0x7fu) | ((w >> 1) & 0x3f80u) | ((w >> 2) & 0x1fc000u) | ((w >> 3) & 0xfe00000u);
}
__device__ __forceinline__ uint32_t bytes_mask(uint32_t nb) { return nb >= 4u ? 0xffffffffu : (1u << (nb << 3)) - 1u; }

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// record offsets of one lane (u32: the lean path runs on batches < 4 GiB); for kOffEnds, s is lane
// 0's start only (the previous record's end), the other lanes take theirs from lane - 1 (start_of)
struct LaneOff {
  uint32_t s, e;
};

__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) x += (uint32_t)__shfl_xor((int)x, m, 64);
  return x;
}

// The end of an optimistic decode (launch_all), by the last workgroup of k_tpl_lane: no 64-record
// group was listed -- every record took a template -- so every slot's placement is final and the
// passes after k_tpl_lane would have nothing to do but their bookkeeping, done here: the next
// decode's info words zeroed (k_lane_count), slot totals n, column bases and kind totals (k_spine's
// every-slot-placed path), the last row split of every slot and the placed mask (k_down_gather). A
// group listed (a record no template took, or one that failed): kInfoResid is not 0, and the host re-runs
// the decode with every pass (tfrg_result_info). Saves the five dependent launches after it.
// `listed`: the groups every workgroup listed, from the same atomic as the workgroup tickets (no
// fence: a release per workgroup would write back the XCD's L2 every time).
__device__ void tpl_quiet_finish(const DevOut& o, const uint8_t* slot_kind, uint32_t n_slots, uint32_t n,
                                 uint32_t listed) {
  if (threadIdx.x < kInfoCount) o.info_next[threadIdx.x] = 0u;
  if (listed != 0u) return;  // (uniform; the host sees kInfoResid and re-runs the decode)
  for (uint32_t k = threadIdx.x; k < n_slots; k += kTplBlock) {
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

template <int W, int OM>
__global__ __launch_bounds__(kTplBlock, W == 16 ? 6 : (W == 32 ? 4 : 2)) void k_tpl_lane(
    DevBatch B, DevOut o, LeanArgs A, const uint32_t* __restrict__ img, const uint32_t* __restrict__ tabs) {
  static_assert(W == 16 || W == 32 || W == 64, "window words");
  typedef uint32_t wvec __attribute__((ext_vector_type(W)));
  __shared__ __attribute__((aligned(16))) uint32_t tab[kTplTabs * 256];
  extern __shared__ __attribute__((aligned(16))) uint32_t limg[];  // the templates' lane image
  constexpr uint32_t kWaves = kTplBlock / 64;
  constexpr uint32_t kTw = kLiTw(W);
  const uint32_t lane = threadIdx.x & 63u, wib = rfl(threadIdx.x >> 6);
  cu32* gimg = (cu32*)img;  // (the image's wave-uniform words: scalar loads)
  const uint32_t crcw_u = gimg[3], chain_u = gimg[4];
  const uint8_t* lut = reinterpret_cast<const uint8_t*>(limg + kLiLut);
  // batches are < 0xffffff00 bytes (launch_tpl_lane): an offset of 0xffffff00 reads zeros
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(B.bytes), (short)0, (int)(uint32_t)B.nbytes, 0x00020000);
  const uint32_t nb = (uint32_t)B.nbytes;
  const uint32_t ngroups = (B.n + 63u) >> 6;
  static_assert(kTileShift == 8, "4 groups of 64 records per tile");
  // the wave's groups [gbeg, gend): whole tiles (gpw a multiple of 4, tile sums stored) or half a
  // tile (gpw 2: small batches on twice the waves, tile sums added atomically)
  const bool tail = blockIdx.x >= A.bsplit;
  const uint32_t gpw = tail ? 2u : A.gpw;
  const uint32_t gbeg0 = tail ? A.gsplit + ((blockIdx.x - A.bsplit) * kWaves + wib) * 2u : (blockIdx.x * kWaves + wib) * gpw;
  // (a wave past the batch runs no group: gend = gbeg; it still reaches the optimistic epilogue)
  const uint32_t gbeg = gbeg0 < ngroups ? gbeg0 : ngroups;
  const uint32_t gend = gbeg + gpw < ngroups ? gbeg + gpw : ngroups;
  const bool whole = (gpw & 3u) == 0u;

  auto offsets = [&](uint32_t g) -> LaneOff {
    LaneOff f{1u, 0u};  // (s > e: not in the batch)
    const uint32_t r = (g << 6) + lane;
    if (g < gend && r < B.n) {
      if constexpr (OM == kOffU64) {
        const uint64_t s = B.start[r], e = B.end[r];
        if (((s | e) >> 32) == 0) f = LaneOff{(uint32_t)s, (uint32_t)e};  // (else k_lane_count's record)
      } else if constexpr (OM == kOffU32) {
        f = LaneOff{B.start32[r], B.end32[r]};
      } else {
        f.e = B.end32[r];
        f.s = lane ? 0u : (r ? B.end32[r - 1] : B.first);
      }
    }
    return f;
  };
  auto start_of = [&](const LaneOff& f) -> uint32_t {
    if constexpr (OM == kOffEnds)  // wave_shr:1 -- lane l > 0 reads lane l - 1's end; lane 0 keeps its own
      return (uint32_t)__builtin_amdgcn_update_dpp((int)f.s, (int)f.e, 0x138, 0xf, 0xf, false);
    else
      return f.s;
  };
  auto in_batch = [&](uint32_t g, uint32_t s, uint32_t e) {
    return (g << 6) + lane < B.n && s <= e && e <= nb && e >= 16u;
  };
  auto window = [&](wvec& wn, const LaneOff& f) {
    const uint32_t e = f.e;
    const bool full = e >= 4u * W && e <= nb;
    const uint32_t voff = full ? e - 4u * W : 0xffffff00u;
#pragma unroll
    for (int q = 0; q < W / 4; ++q) {
      const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff + 16u * q, 0, 0));
      wn[4 * q] = v.x;
      wn[4 * q + 1] = v.y;
      wn[4 * q + 2] = v.z;
      wn[4 * q + 3] = v.w;
    }
  };
  // a record ending in the batch's first 4 W bytes (group 0 only): its window begins before the
  // batch; those bytes are outside the record (template mask 0), the rest is read byte by byte. (Its
  // own step, after the prologue: byte loads pending at a merge with the common path made the
  // compiler wait for every load in flight there.)
  auto head_fix = [&](wvec& wn, const LaneOff& f, uint32_t g) {
    if (g != 0u) return;  // (uniform)
    const uint32_t e = f.e;
    const bool full = e >= 4u * W && e <= nb;
    const bool head = in_batch(g, start_of(f), e) && !full;
    if (__ballot(head)) {
#pragma unroll
      for (int i = 0; i < W; ++i) {
        uint32_t x = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int64_t p = (int64_t)e - 4 * W + 4 * i + b;
          if (head && p >= 0) x |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rsrc, (uint32_t)p, 0, 0) << (8 * b);
        }
        if (head) wn[i] = x;
      }
    }
  };
  // window word q (wave-uniform): one indexed move (s_set_gpr_idx) for W <= 32; a compare chain for
  // W = 64, whose 64-register vector the indexed form would move through scratch
  auto wsel = [](const wvec& w, uint32_t q) -> uint32_t {
    if constexpr (W <= 32) {
      return w[q & (W - 1u)];
    } else {
      uint32_t a = 0;
#pragma unroll
      for (int i = 0; i < W; ++i)
        if (q == (uint32_t)i) a = w[i];
      return a;
    }
  };
  uint32_t acc = 0;  // lane k: slot k's value count over this tile's records so far
  uint32_t listed = 0;  // (wave-uniform) groups this wave listed for k_lane_count
  // one group: every lane matches the template its payload length selects (kLiLut; the next one of
  // the same length if that fails), then the dict into the columns, one store per column
  auto proc = [&](const wvec& w, uint32_t g, const LaneOff& f) {
    const uint32_t r = (g << 6) + lane;
    const bool valid = r < B.n;
    const uint32_t st = start_of(f), en = f.e;
    const bool inb = in_batch(g, st, en);
    const uint32_t rl = en - st;
    // (records above lane_max belong to the wavefront kernels)
    uint32_t cand = inb && rl >= 16u && rl - 16u <= kTplMaxL && rl <= A.lane_max ? (uint32_t)lut[rl - 16u] : 0xffu;
    uint32_t tsel = 0xffu;
    while (__ballot(cand != 0xffu)) {  // (usually one pass: lengths rarely share templates)
      const bool act = cand != 0xffu;
      const uint32_t* tp = limg + kLiTpl + (act ? cand : 0u) * kTw;
      const u32x4 meta = *reinterpret_cast<const u32x4*>(tp);  // L, K, next
      uint32_t diff = 0;
#pragma unroll
      for (int q = 0; q < W / 4; ++q) {
        const u32x4 bm = *reinterpret_cast<const u32x4*>(tp + 4 + 4 * q);
        const u32x4 mm = *reinterpret_cast<const u32x4*>(tp + 4 + W + 4 * q);
        diff |= ((w[4 * q] ^ bm.x) & mm.x) | ((w[4 * q + 1] ^ bm.y) & mm.y) | ((w[4 * q + 2] ^ bm.z) & mm.z) |
                ((w[4 * q + 3] ^ bm.w) & mm.w);
        // (one quarter of the template's words live at a time: hoisting all of them costs 32 VGPRs,
        // i.e. occupancy; other waves cover the LDS latency)
        if (q & 1) __builtin_amdgcn_sched_barrier(0);
      }
      // payload CRC-32C over the words where any template has variable bits (this lane's template
      // masks them, Cm): variable bits further than 32 bytes from the end through a slice-by-4 chain
      // (its state joins word W - 9, distances 28..31), the last 32 bytes by position tables
      const uint32_t* cm = tp + 4 + 2 * W;
      uint32_t c = 0;
      if (chain_u < (uint32_t)(W - 9)) {
#pragma unroll
        for (int i = 0; i < W - 9; ++i)
          if ((uint32_t)i >= chain_u) c = lin_word<0>(tab, c ^ (w[i] & cm[i]));
      }
      uint32_t lin = 0;
#define TFRG_LIN(j)                                                                                       \
  if (crcw_u & (1u << (j))) lin ^= lin_word<28 - 4 * (j)>(tab, (w[W - 9 + (j)] & cm[W - 9 + (j)]) ^ ((j) == 0 ? c : 0u));
      TFRG_LIN(0) TFRG_LIN(1) TFRG_LIN(2) TFRG_LIN(3) TFRG_LIN(4) TFRG_LIN(5) TFRG_LIN(6) TFRG_LIN(7)
#undef TFRG_LIN
      const bool ok = act && diff == 0u && crc_mask(lin ^ meta.y) == w[W - 1];
      tsel = ok ? cand : tsel;
      cand = act && !ok ? meta.z : 0xffu;
    }
    const bool hit = tsel != 0xffu;
    if (hit && !(A.implicit & TFRG_IMPLICIT_STATUS)) {  // (uniform test)
      o.status[r] = TFRG_OK;
      o.verdict[r] = (uint8_t)kHitVerdict;
    }
    if (__ballot(hit)) {
      const uint32_t* ts = limg + kLiTpl + (hit ? tsel : 0u) * kTw + 4 + 3 * W;  // the lane's slot table
      for (uint32_t k = 0; k < A.n_slots; ++k) {  // (wave-uniform)
        const uint32_t sq = gimg[kLiSlotQ + k];
        const u32x4 z = *reinterpret_cast<const u32x4*>(ts + 4u * k);
        const uint32_t mode = z.x & 0xffu, len = (z.x >> 8) & 0xffu, pos = z.y, cw = z.z;
        uint32_t lx = pos, ly = len;  // mode 0: a list's payload-relative location (absent: 0, 0)
        if (sq & kLiQValue) {  // (wave-uniform) one int64 varint / one float: the 4 bytes at window byte pos
          // (from the window registers -- a load here would wait out every store before it, vmcnt --
          // over the window words where some template has such a value)
          const uint32_t qw = pos >> 2;
          uint32_t a = 0, b = 0;
          for (uint32_t i = sq & 0xffu; i <= ((sq >> 8) & 0xffu); ++i) {  // (wave-uniform)
            const bool at = qw == i;
            a = at ? wsel(w, i) : a;
            b = at ? wsel(w, i + 1u) : b;
          }
          const uint32_t x = __builtin_amdgcn_alignbyte(b, a, pos & 3u);
          if (mode == 1u || mode == 2u) {
            lx = mode == 1u ? vgroups(x, bytes_mask(len)) : x;
            ly = 0;
          }
        }
        if (mode == 3u) lx = en + pos;  // one bytes element: its batch offset and length
        // (the tile sums: not kept by an optimistic decode, whose placed slots need no scan)
        const uint32_t tot = !A.tsum ? 0u
                             : (sq & kLiQSingle) ? (uint32_t)__popcll(__ballot(hit && cw != 0u))
                                                 : wave_sum(hit ? (cw & ~kCountInline) : 0u);
        const LeanTgt& T = A.tg[k];
        if (hit) {
          if (!(A.implicit & TFRG_IMPLICIT_ORDER)) T.ord[r] = (uint16_t)(z.x >> 16);
          if (T.kind) {  // speculative placement: value at column row r; the row split r is implicit
                         // (tfrg_info.placed_slots: a final placement's row splits are never stored)
            if (r < T.lim) {
              if (T.kind == TFRG_KIND_INT64) {
                reinterpret_cast<uint64_t*>(T.v1)[r] = lx;
              } else {
                reinterpret_cast<uint32_t*>(T.v1)[r] = lx;
                if (T.kind == TFRG_KIND_BYTES && !(A.implicit & TFRG_IMPLICIT_BYTES_LEN)) T.v2[r] = ly;
              }
            }
          } else {
            T.cnt[r] = cw;
            T.loc[r] = make_uint2(lx, ly);
          }
        }
        acc += lane == k ? tot : 0u;
      }
    }
    // records no template took: k_lane_count's
    const uint64_t mm = __ballot(valid && !hit);
    if (lane == 0) {
      o.lmask[g] = mm;
      if (mm) o.rlist[atomicAdd(&o.info[kInfoResid], 1u)] = g;
    }
    listed += mm ? 1u : 0u;
  };
  auto flush = [&](uint32_t g) {  // the tile sums of group g's tile: the first writer of tsum (zero
    // before the decode; k_lane_count's residual records add theirs with atomics after this kernel)
    if (lane < A.n_slots && acc && A.tsum) {
      if (whole)
        A.tsum[lane * A.tile_stride + (g >> 2)] = acc;
      else
        atomicAdd(&A.tsum[lane * A.tile_stride + (g >> 2)], acc);
    }
    acc = 0;
  };
  // one group per step (one window live: the per-lane template words need the registers); the next
  // group's offsets are requested before this group's stores. The wave's first offsets and window
  // are requested before the workgroup copies its CRC tables and lane image into LDS, so its first
  // HBM round trips overlap that copy (~3 % of a launch of 2,000 workgroups).
  // (the first round of the table and image copies, the first two groups' offsets: all in flight
  // together; then the first window, which needs the offsets)
  LaneOff fa = offsets(gbeg), f0 = offsets(gbeg + 1u);
  static_assert(kTplTabs * 256u % (4u * kTplBlock) == 0u, "table copy in whole 16-byte rounds");
  constexpr uint32_t kTabRounds = kTplTabs * 256u / (4u * kTplBlock);
  u32x4 tv[kTabRounds];
#pragma unroll
  for (uint32_t j = 0; j < kTabRounds; ++j) tv[j] = reinterpret_cast<const u32x4*>(tabs)[threadIdx.x + j * kTplBlock];
  const uint32_t iw0 = threadIdx.x < A.img_words ? img[threadIdx.x] : 0u;
  wvec wa;
  window(wa, fa);
#pragma unroll
  for (uint32_t j = 0; j < kTabRounds; ++j) reinterpret_cast<u32x4*>(tab)[threadIdx.x + j * kTplBlock] = tv[j];
  if (threadIdx.x < A.img_words) limg[threadIdx.x] = iw0;
  for (uint32_t i = threadIdx.x + kTplBlock; i < A.img_words; i += kTplBlock) limg[i] = img[i];
  __syncthreads();
  for (uint32_t g = gbeg; g < gend; ++g) {
    head_fix(wa, fa, g);
    proc(wa, g, fa);
    if (((g + 1u) & 3u) == 0u || g + 1u >= gend) flush(g);
    if (g + 1u < gend) {
      window(wa, f0);
      fa = f0;
      f0 = offsets(g + 2u);
    }
  }
  if (A.finish) {  // (uniform) optimistic decode: the last workgroup to finish ends it
    __shared__ uint32_t s_listed[kWaves];
    __shared__ uint32_t s_last, s_total;
    if (lane == 0) s_listed[wib] = listed;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t mine = 0;
      for (uint32_t i = 0; i < kWaves; ++i) mine += s_listed[i];
      const uint64_t old = atomicAdd(reinterpret_cast<unsigned long long*>(o.info + kInfoTplDone),
                                     ((unsigned long long)mine << 32) | 1ull);
      s_last = (uint32_t)old == gridDim.x - 1u;
      s_total = (uint32_t)(old >> 32) + mine;
    }
    __syncthreads();
    if (s_last) tpl_quiet_finish(o, A.finish, A.n_slots, B.n, s_total);
  }
}

}  // namespace

hipError_t launch_tpl_lane(const DevBatch& b, const DevOut& o, const LeanArgs& a, const uint32_t* img, uint32_t w,
                           const uint32_t* d_tab, int num_cus, hipStream_t st) {
  const uint32_t groups = (b.n + 63u) / 64u;
  const uint32_t tiles = (groups + 3u) / 4u;  // (one wave per 256-record tile)
  const uint32_t need = (tiles + kTplBlock / 64 - 1) / (kTplBlock / 64);
  // two tiles per wave (one for batches of fewer than 8 workgroups per CU, half a tile for batches of
  // fewer workgroups than CUs, a quarter -- one group -- below half as many: a latency-bound launch
  // of a few MiB, c1file 15.5 -> 12.2 us), no resident-grid stride: workgroups retire all through the launch,
  // so the end of the batch does not wait on the waves that drew an extra round of tiles (c4of8:
  // 0.414 ms against 0.430 ms for one round of resident workgroups; the 32 KiB table copy per
  // workgroup is L2 traffic)
  LeanArgs a2 = a;
  a2.gpw = need < (uint32_t)num_cus / 2u ? 1u : need < (uint32_t)num_cus ? 2u : need >= 8u * (uint32_t)num_cus ? 8u : 4u;
  // The dispatcher hands out workgroups in index order as slots free up, so the last ones decide
  // when the batch ends: the groups of about one round of resident workgroups (3 per CU) at the end
  // of a large batch go to workgroups of 2 groups per wave instead of gpw, and the last round idles
  // the CUs for a quarter of the time (TFRG_TPL_TAIL=0: off)
  static const bool split_on = [] {
    const char* e = getenv("TFRG_TPL_TAIL");
    return !e || atoi(e) != 0;
  }();
  constexpr uint32_t kW = kTplBlock / 64;
  uint32_t gsplit = groups, bsplit = 0xffffffffu;
  if (split_on && a2.gpw == 8u) {
    const uint32_t small = 3u * (uint32_t)num_cus * kW * 2u;  // groups of one round of 2-group workgroups
    if (groups > 4u * small) {
      const uint32_t big_blocks = (groups - small) / (kW * a2.gpw);
      gsplit = big_blocks * kW * a2.gpw;
      bsplit = big_blocks;
    }
  }
  a2.gsplit = gsplit;
  a2.bsplit = bsplit;
  const uint32_t blocks = bsplit != 0xffffffffu
                              ? bsplit + (groups - gsplit + kW * 2u - 1u) / (kW * 2u)
                              : ((groups + a2.gpw - 1u) / a2.gpw + kW - 1u) / kW;
  const dim3 grid(blocks ? blocks : 1u);
  const uint32_t* tabs = d_tab + kLeanTabOff;
  const size_t lds = (size_t)a.img_words * 4;  // (the lane image; the CRC tables are static)
#define TFRG_TPL_LAUNCH(WW, OO) hipLaunchKernelGGL((k_tpl_lane<WW, OO>), grid, dim3(kTplBlock), lds, st, b, o, a2, img, tabs)
#define TFRG_TPL_OM(WW)                                                        \
  switch (b.omode) {                                                           \
    case kOffU64: TFRG_TPL_LAUNCH(WW, kOffU64); break;                         \
    case kOffU32: TFRG_TPL_LAUNCH(WW, kOffU32); break;                         \
    default: TFRG_TPL_LAUNCH(WW, kOffEnds); break;                             \
  }
  switch (w) {
    case 16: TFRG_TPL_OM(16) break;
    case 32: TFRG_TPL_OM(32) break;
    case 64: TFRG_TPL_OM(64) break;
    default: return hipErrorInvalidValue;
  }
#undef TFRG_TPL_OM
#undef TFRG_TPL_LAUNCH
  return hipGetLastError();
}

}  // namespace tfrg
