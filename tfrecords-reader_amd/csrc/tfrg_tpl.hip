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
//   * the template's dict straight into the columns: order, count / loc, or the speculatively
//     placed value + row split (DevSchema::spec), and the per-tile value counts.
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

template <int W>
__global__ __launch_bounds__(kTplBlock, W == 16 ? 6 : (W == 32 ? 4 : 2)) void k_tpl_lane(
    DevBatch B, DevOut o, LeanArgs A, const uint32_t* __restrict__ tpl, const uint32_t* __restrict__ tabs) {
  static_assert(W == 16 || W == 32 || W == 64, "window words");
  __shared__ uint32_t tab[kTplTabs * 256];
  for (uint32_t i = threadIdx.x; i < kTplTabs * 256; i += kTplBlock) tab[i] = tabs[i];
  __syncthreads();
  constexpr uint32_t kWaves = kTplBlock / 64;
  const uint32_t lane = threadIdx.x & 63u, wib = rfl(threadIdx.x >> 6);
  // batches are < 0xffffff00 bytes (launch_tpl_lane): an offset of 0xffffff00 reads zeros
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(B.bytes), (short)0, (int)(uint32_t)B.nbytes, 0x00020000);
  const uint32_t ngroups = (B.n + 63u) >> 6;
  // A wave takes whole 256-record tiles (4 groups of 64), tile t0 + k nw: the per-slot tile sums
  // are then one plain store per tile (lane k: slot k), no atomics. kTileShift = 8 (asserted below).
  static_assert(kTileShift == 8, "4 groups of 64 records per tile");
  const uint32_t ntiles = (ngroups + 3u) >> 2;
  const uint32_t nw = gridDim.x * kWaves;
  // (A.half: wave w takes the groups 2w, 2w + 1, one step, and adds its tile sums atomically: a
  // batch too small to give every CU a workgroup runs on twice the waves)
  const uint32_t w0 = blockIdx.x * kWaves + wib;
  const uint32_t t0 = A.half ? w0 >> 1 : w0;
  if (t0 >= ntiles || (A.half && 4u * t0 + ((w0 & 1u) << 1) >= ngroups)) return;  // (wave-uniform; no barrier follows)
  // Two groups per step (g, g + 1 of the wave's tile), their windows loaded together: a step waits
  // once, for both windows and the previous step's column stores (gfx9 counts stores in vmcnt, in
  // issue order), so each wait covers 128 records. The offsets of the next step are requested
  // before this step's stores (they are then ready without waiting for those).
  auto offsets = [&](uint32_t gg, uint64_t& s, uint64_t& e) {
    s = 0;
    e = 0;
    if (gg < ngroups && (gg << 6) + lane < B.n) {
      s = B.start[(gg << 6) + lane];
      e = B.end[(gg << 6) + lane];
    }
  };
  auto in_batch = [&](uint32_t gg, uint64_t s, uint64_t e) {
    return gg < ngroups && (gg << 6) + lane < B.n && s <= e && e <= B.nbytes && e >= 16u;
  };
  auto window = [&](uint32_t (&wn)[W], bool inb, uint64_t e, uint32_t gg) {
    const bool full = inb && e >= 4u * W;
    const uint32_t voff = full ? (uint32_t)e - 4u * W : 0xffffff00u;
#pragma unroll
    for (int q = 0; q < W / 4; ++q) {
      const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff + 16u * q, 0, 0));
      wn[4 * q] = v.x;
      wn[4 * q + 1] = v.y;
      wn[4 * q + 2] = v.z;
      wn[4 * q + 3] = v.w;
    }
    // a record ending in the batch's first 4 W bytes (group 0 only): its window begins before the
    // batch; those bytes are outside the record (template mask 0), the rest is read byte by byte
    const bool head = inb && !full;
    if (gg == 0u && __ballot(head)) {
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
  uint32_t acc = 0;  // lane k: slot k's value count over this tile's records so far
  // one group: template match + CRC, the template's dict into the columns, the miss mask
  auto proc = [&](const uint32_t (&w)[W], uint32_t g, uint64_t st, uint64_t en) {
    const uint32_t r = (g << 6) + lane;
    const bool valid = r < B.n;
    const bool inb = in_batch(g, st, en);
    const uint32_t en32 = (uint32_t)en;
    const uint32_t rl = (uint32_t)(en - st);
    bool hit = false;
    for (uint32_t t = 0; t < A.n_tpl; ++t) {  // (wave-uniform)
      cu32* tp = (cu32*)tpl + t * kLtWords;
      const uint32_t L = tp[kLtL];
      if (L + 16u > A.lane_max) continue;  // (its records belong to the wavefront kernels)
      const bool cand = inb && !hit && rl == L + 16u;
      if (!__ballot(cand)) continue;
      uint32_t diff = 0;
#pragma unroll
      for (int i = 0; i < W - 1; ++i) diff |= (w[i] ^ tp[kLtWin + i]) & tp[kLtWin + W + i];
      // payload CRC-32C: variable bits further than 32 bytes from the end through a slice-by-4
      // chain (its state joins word W - 9, distances 28..31), the last 32 bytes by position tables
      uint32_t c = 0;
      const uint32_t chain = tp[kLtChain];
      if (chain < (uint32_t)(W - 9)) {
#pragma unroll
        for (int i = 0; i < W - 9; ++i)
          if ((uint32_t)i >= chain) c = lin_word<0>(tab, c ^ (w[i] & tp[kLtWin + 2 * W + i]));
      }
      const uint32_t crcw = tp[kLtCrcw];
      uint32_t lin = 0;
#define TFRG_LIN(j)                                                                              \
  if (crcw & (1u << (j))) lin ^= lin_word<28 - 4 * (j)>(tab, (w[W - 9 + (j)] & tp[kLtWin + 2 * W + W - 9 + (j)]) ^ \
                                                                  ((j) == 0 ? c : 0u));
      TFRG_LIN(0) TFRG_LIN(1) TFRG_LIN(2) TFRG_LIN(3) TFRG_LIN(4) TFRG_LIN(5) TFRG_LIN(6) TFRG_LIN(7)
#undef TFRG_LIN
      const bool ok = cand && diff == 0u && crc_mask(lin ^ tp[kLtK]) == w[W - 1];
      const uint64_t okm = __ballot(ok);
      hit |= ok;
      if (!okm) continue;
      // the template's dict, for the lanes that took it
      if (ok) {
        o.status[r] = TFRG_OK;
        o.verdict[r] = (uint8_t)kHitVerdict;
      }
      const uint32_t hits = (uint32_t)__popcll(okm);
      const uint32_t ne = tp[kLtNe];
      for (uint32_t e = 0; e < ne; ++e) {  // (wave-uniform)
        const uint32_t e0 = tp[kLtEnt + 4 * e], rank = tp[kLtEnt + 4 * e + 1], cw = tp[kLtEnt + 4 * e + 2],
                       pos = tp[kLtEnt + 4 * e + 3];
        const uint32_t slot = e0 & 0xffu, mode = (e0 >> 8) & 0xfu, len = e0 >> 16;
        const LeanTgt& T = A.tg[slot];
        uint32_t lx, ly = 0;
        if (mode == 1u || mode == 2u) {  // one int64 varint / one float: the 4 bytes at window byte pos
          // (from the window's registers: a load here would wait out every store before it, vmcnt)
          const uint32_t q = pos >> 2;
          uint32_t a = 0, b = 0;
#pragma unroll
          for (int i = 0; i < W; ++i)
            if (q == (uint32_t)i) {  // (wave-uniform)
              a = w[i];
              b = i + 1 < W ? w[i + 1] : 0u;
            }
          const uint32_t x = __builtin_amdgcn_alignbyte(b, a, pos & 3u);
          lx = mode == 1u ? vgroups(x, bytes_mask(len)) : x;
        } else if (mode == 3u) {  // one bytes element: its batch offset and length
          lx = en32 + pos;
          ly = len;
        } else {  // a list: its payload-relative location
          lx = pos;
          ly = len;
        }
        if (ok) {
          T.ord[r] = (uint16_t)rank;
          if (T.kind) {  // speculative placement: value at column row r; the row split r is implicit
                         // (tfrg_info.placed_slots: a final placement's row splits are never stored)
            if (r < T.lim) {
              if (T.kind == TFRG_KIND_INT64) {
                reinterpret_cast<uint64_t*>(T.v1)[r] = lx;
              } else {
                reinterpret_cast<uint32_t*>(T.v1)[r] = lx;
                if (T.kind == TFRG_KIND_BYTES) T.v2[r] = ly;
              }
            }
          } else {
            T.cnt[r] = cw;
            T.loc[r] = make_uint2(lx, ly);
          }
        }
        acc += lane == slot ? (cw & ~kCountInline) * hits : 0u;
      }
      for (uint32_t m = tp[kLtAbsent]; m; m &= m - 1u) {  // slots the shape lacks: order / count 0
        const LeanTgt& T = A.tg[__builtin_ctz(m)];
        if (ok) {
          T.ord[r] = 0;
          T.cnt[r] = 0;
        }
      }
    }
    // records no template took: k_lane_count's
    const uint64_t mm = __ballot(valid && !hit);
    if (lane == 0) {
      o.lmask[g] = mm;
      if (mm) o.rlist[atomicAdd(&o.info[kInfoResid], 1u)] = g;
    }
  };
  // the wave's steps: tile t0 + k nw, groups (4t, 4t+1), (4t+2, 4t+3)
  uint32_t t = t0, p = A.half ? (w0 & 1u) << 1 : 0u;
  uint64_t s0, e0, s1, e1;
  offsets(4u * t + p, s0, e0);
  offsets(4u * t + p + 1u, s1, e1);
  while (t < ntiles) {
    const uint32_t ga = 4u * t + p, gb = ga + 1u;
    uint32_t wa[W], wb[W];
    window(wa, in_batch(ga, s0, e0), e0, ga);
    window(wb, in_batch(gb, s1, e1), e1, gb);
    const uint64_t sa = s0, ea = e0, sb = s1, eb = e1;
    // the next step's offsets
    const uint32_t tn = p ? t + nw : t, pn = p ^ 2u;
    offsets(4u * tn + pn, s0, e0);
    offsets(4u * tn + pn + 1u, s1, e1);
    proc(wa, ga, sa, ea);
    if (gb < ngroups) proc(wb, gb, sb, eb);
    // the tile's sums: the first writer of tsum (zero before the decode; k_lane_count's residual
    // records add theirs with atomics after this kernel)
    if (A.half) {  // (wave-uniform) the other half of the tile is another wave's
      if (lane < A.n_slots && acc) atomicAdd(&A.tsum[lane * A.tile_stride + t], acc);
      break;
    }
    if (p || gb + 1u >= ngroups) {
      if (lane < A.n_slots && acc) A.tsum[lane * A.tile_stride + t] = acc;
      acc = 0;
    }
    if (gb + 1u >= ngroups) break;
    t = tn;
    p = pn;
  }
}

}  // namespace

hipError_t launch_tpl_lane(const DevBatch& b, const DevOut& o, const LeanArgs& a, const uint32_t* tpl, uint32_t w,
                           const uint32_t* d_tab, int num_cus, hipStream_t st) {
  const uint32_t groups = (b.n + 63u) / 64u;
  const uint32_t tiles = (groups + 3u) / 4u;  // (one wave per 256-record tile)
  const uint32_t need = (tiles + kTplBlock / 64 - 1) / (kTplBlock / 64);
  // two tiles per wave (one for batches of fewer than 8 workgroups per CU), no resident-grid
  // stride: workgroups retire all through the launch, so the end of the batch does not wait on
  // the waves that drew an extra round of tiles (c4of8: 0.414 ms against 0.430 ms for one round of
  // resident workgroups; the 32 KiB table copy per workgroup is L2 traffic)
  const uint32_t per_wave = need >= 8u * (uint32_t)num_cus ? 2u : 1u;
  LeanArgs a2 = a;
  a2.half = need < (uint32_t)num_cus ? 1u : 0u;  // (fewer workgroups than CUs: half a tile per wave)
  const dim3 grid(a2.half ? (tiles * 2u + kTplBlock / 64 - 1) / (kTplBlock / 64) : need ? (need + per_wave - 1u) / per_wave : 1u);
  const uint32_t* tabs = d_tab + kLeanTabOff;
  switch (w) {
    case 16: hipLaunchKernelGGL(k_tpl_lane<16>, grid, dim3(kTplBlock), 0, st, b, o, a2, tpl, tabs); break;
    case 32: hipLaunchKernelGGL(k_tpl_lane<32>, grid, dim3(kTplBlock), 0, st, b, o, a2, tpl, tabs); break;
    case 64: hipLaunchKernelGGL(k_tpl_lane<64>, grid, dim3(kTplBlock), 0, st, b, o, a2, tpl, tabs); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace tfrg
