// tfrg_bytes.hip — TFRG_FLAG_MATERIALIZE_BYTES: the bytes_list elements of a decoded batch gathered
// into one contiguous device byte column with u64 offsets (Arrow LargeBinary layout), instead of the
// default zero-copy (offset, length) views into the input. Replaces the reference's per-element
// `bytes(...)` copy (decoder.pyx:203-223, bytes_list_from_bytes) with two HBM-bound passes:
//   1. k_bytes_scan : exclusive scan of the element lengths (single pass, tickets + decoupled
//                     look-back), offsets[0..nb]; lists the elements longer than kBigElem.
//   2. k_bytes_copy : short elements copied cooperatively by waves over groups of 64 elements
//                     (lane j moves byte j of the group's concatenated output: coalesced stores),
//                     long ones one wave each with 16-byte aligned stores.
// The element count nb is device-resident (kind_totals[1], written by k_spine), so neither pass
// needs a host round trip.
#include <hip/hip_runtime.h>
#include "tfrg_internal.h"
#include "../../include/tfrg_status.h"

namespace tfrg {

constexpr int kBsBlock = 256;
constexpr int kBsItems = 16;
constexpr uint32_t kBsTile = kBsBlock * kBsItems;  // elements per scan tile
constexpr uint32_t kBigElem = 128;                 // longer elements: one wave each
constexpr uint64_t kLbFlagShift = 62;              // look-back word: flag (1 total, 2 prefix) << 62 | value

__device__ __forceinline__ uint64_t wave_incl_scan_u64(uint64_t v, uint32_t lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(v, d, 64);
    if (lane >= (uint32_t)d) v += y;
  }
  return v;
}

__global__ __launch_bounds__(kBsBlock) void k_bytes_scan(DevBytes d) {
  __shared__ uint32_t s_ticket;
  __shared__ uint64_t s_w[kBsBlock / 64];
  __shared__ uint64_t s_excl;
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  const uint64_t nb = d.kind_totals[TFRG_KIND_BYTES];
  if (nb > d.offsets_cap) return;  // k_spine flagged the overflow
  const uint64_t vmask = (1ull << kLbFlagShift) - 1ull;
  for (;;) {
    if (threadIdx.x == 0) s_ticket = atomicAdd(d.ticket, 1u);
    __syncthreads();
    const uint32_t tile = s_ticket;
    __syncthreads();
    const uint64_t i0 = (uint64_t)tile * kBsTile + (uint64_t)threadIdx.x * kBsItems;
    if ((uint64_t)tile * kBsTile > nb) break;  // workgroup-uniform (tiles cover offsets[0..nb])
    uint32_t v[kBsItems];
    uint64_t sum = 0;
    uint32_t nbig = 0;
#pragma unroll
    for (int j = 0; j < kBsItems; ++j) {
      const uint64_t i = i0 + j;
      v[j] = i < nb ? d.b_len[i] : 0u;
      sum += v[j];
      nbig += v[j] > kBigElem;
    }
    // long elements: listed for the wave-per-element copy (one atomic per wave)
    if (__ballot(nbig != 0)) {
      uint32_t pos = nbig;
#pragma unroll
      for (int s = 1; s < 64; s <<= 1) {
        const uint32_t y = __shfl_up(pos, s, 64);
        if (lane >= (uint32_t)s) pos += y;
      }
      uint32_t b0 = 0;
      if (lane == 63) b0 = atomicAdd(d.big_count, pos);
      b0 = __shfl(b0, 63, 64) + pos - nbig;
#pragma unroll
      for (int j = 0; j < kBsItems; ++j)
        if (v[j] > kBigElem) d.big_list[b0++] = (uint32_t)(i0 + j);
    }
    const uint64_t incl = wave_incl_scan_u64(sum, lane);
    if (lane == 63) s_w[wid] = incl;
    __syncthreads();
    uint64_t pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kBsBlock / 64; ++w) {
      const uint64_t x = s_w[w];
      pre += (uint32_t)w < wid ? x : 0ull;
      tot += x;
    }
    if (threadIdx.x == 0) {
      __hip_atomic_store(&d.lb[tile], ((tile ? 1ull : 2ull) << kLbFlagShift) | tot, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      uint64_t excl = 0;
      for (int64_t j = (int64_t)tile - 1; j >= 0;) {  // predecessors (ticket order: all started)
        const uint64_t w = __hip_atomic_load(&d.lb[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t flag = w >> kLbFlagShift;
        if (!flag) {
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        excl += w & vmask;
        if (flag == 2) break;
        --j;
      }
      if (tile) __hip_atomic_store(&d.lb[tile], (2ull << kLbFlagShift) | (excl + tot), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
      s_excl = excl;
    }
    __syncthreads();
    uint64_t run = s_excl + pre + incl - sum;
#pragma unroll
    for (int j = 0; j < kBsItems; ++j) {
      const uint64_t i = i0 + j;
      if (i <= nb) d.offsets[i] = run;
      run += v[j];
    }
  }
}

// 4 bytes at an arbitrary address inside the readable input (two aligned dwords + funnel shift)
__device__ __forceinline__ uint32_t ld_u32u(const uint8_t* p, uint64_t a, uint64_t lim) {
  const uint64_t a0 = a & ~3ull;
  const uint32_t w0 = *reinterpret_cast<const uint32_t*>(p + (a0 < lim ? a0 : lim));
  const uint32_t w1 = *reinterpret_cast<const uint32_t*>(p + (a0 + 4 < lim ? a0 + 4 : lim));
  return __builtin_amdgcn_alignbyte(w1, w0, (uint32_t)(a & 3u));
}

// one element copied by the whole wave: byte head up to a 16-byte aligned destination, 16-byte
// stores assembled from aligned source dwords, byte tail
__device__ __forceinline__ void copy_wave(uint8_t* out, uint64_t dst, const uint8_t* in, uint64_t src, uint64_t len,
                                          uint64_t lim, uint32_t lane) {
  uint64_t h = (16u - (uint32_t)(dst & 15u)) & 15u;
  if (h > len) h = len;
  if (lane < h) out[dst + lane] = in[src + lane];
  const uint64_t body = (len - h) >> 4;
  for (uint64_t c = lane; c < body; c += 64) {
    const uint64_t s = src + h + 16 * c;
    uint4 q;
    q.x = ld_u32u(in, s, lim);
    q.y = ld_u32u(in, s + 4, lim);
    q.z = ld_u32u(in, s + 8, lim);
    q.w = ld_u32u(in, s + 12, lim);
    *reinterpret_cast<uint4*>(out + dst + h + 16 * c) = q;
  }
  const uint64_t t0 = h + 16 * body;
  if (lane < len - t0) out[dst + t0 + lane] = in[src + t0 + lane];
}

__global__ __launch_bounds__(kBsBlock) void k_bytes_copy(DevBytes d) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nb = d.kind_totals[TFRG_KIND_BYTES];
  if (nb > d.offsets_cap) return;  // k_spine flagged the overflow
  const uint64_t total = d.offsets[nb];
  if (total > d.data_cap) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *d.overflow = 1u;
    return;
  }
  const uint64_t lim = d.in_readable - 4;
  const uint32_t wave = blockIdx.x * (kBsBlock / 64) + (threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * (kBsBlock / 64);
  // short elements: groups of 64, the group's output bytes spread over the lanes
  for (uint64_t g = wave; g * 64 < nb; g += nwaves) {
    const uint64_t e = g * 64 + lane;
    const bool in = e < nb;
    const uint32_t len = in ? d.b_len[e] : 0u;
    const uint32_t vl = len <= kBigElem ? len : 0u;
    const uint64_t src = in ? d.b_off[e] : 0u;
    const uint64_t dst = in ? d.offsets[e] : 0u;
    uint32_t vend = vl;  // inclusive scan of the short lengths: the group's virtual output axis
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
      const uint32_t y = __shfl_up(vend, s, 64);
      if (lane >= (uint32_t)s) vend += y;
    }
    const uint32_t T = __builtin_amdgcn_readlane(vend, 63);
    for (uint32_t p0 = 0; p0 < T; p0 += 64) {  // wave-uniform trip count: every lane shuffles
      const uint32_t p = p0 + lane;
      uint32_t k = 0;  // first lane whose virtual end is > p
#pragma unroll
      for (uint32_t s = 32; s; s >>= 1)
        if ((uint32_t)__shfl((int)vend, (int)(k + s - 1u), 64) <= p) k += s;
      k = k < 63u ? k : 63u;
      const uint32_t vb = (uint32_t)__shfl((int)vend, (int)k, 64) - (uint32_t)__shfl((int)vl, (int)k, 64);
      const uint64_t sk = __shfl(src, (int)k, 64), dk = __shfl(dst, (int)k, 64);
      if (p < T) d.data[dk + (p - vb)] = d.in[sk + (p - vb)];
    }
  }
  // long elements: one wave each
  const uint32_t nbig = *d.big_count;
  for (uint32_t i = wave; i < nbig; i += nwaves) {
    const uint32_t e = __builtin_amdgcn_readfirstlane(d.big_list[i]);
    copy_wave(d.data, d.offsets[e], d.in, d.b_off[e], d.b_len[e], lim, lane);
  }
}

hipError_t launch_materialize(const DevBytes& d, int num_cus, hipStream_t st) {
  hipLaunchKernelGGL(k_bytes_scan, dim3(num_cus * 2), dim3(kBsBlock), 0, st, d);
  hipLaunchKernelGGL(k_bytes_copy, dim3(num_cus * 8), dim3(kBsBlock), 0, st, d);
  return hipGetLastError();
}

uint64_t materialize_lb_words(uint64_t cap_b) { return (cap_b + 1 + kBsTile - 1) / kBsTile + 1; }

}  // namespace tfrg
