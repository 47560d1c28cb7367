// probe_lane.hip — memory-shape probe of the C1 lane path (measurement only, never the product).
//
// What does the HBM system give a kernel that moves exactly k_tpl_lane's bytes on C1-shaped
// records, with no decode work? Records of 58/59 bytes back to back; a lane takes one record:
// its offsets, its last 64 bytes as four unaligned 16-byte buffer loads, and (STORE) the 25 bytes
// a template hit writes: status u32, verdict u8, two order u16, an int64 value, a bytes view
// (u32 offset, u32 length). Variants: u64 (start, end) vs u32 end-only offsets; two groups of 64
// records per step (the product's shape) vs a software pipeline of one group per step whose next
// window is requested before this group's stores (gfx9's vmcnt counts loads and stores in issue
// order, so a wait for the next window then does not wait for this group's store acks).
//   hipcc -O3 --offload-arch=gfx950 tools/probe_lane.hip -o /tmp/probe_lane && /tmp/probe_lane
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct Cols {
  int32_t* status;
  uint8_t* verdict;
  uint16_t* ord0;
  uint16_t* ord1;
  uint64_t* v;
  uint32_t* boff;
  uint32_t* blen;
  uint32_t* sink;
};

enum : int { kU64 = 1, kStore = 2, kPipe = 4, kCheck = 8, kNoSV = 16, kNoOrd = 32, kStaged = 64, kTabLds = 128,
             kTab8 = 256, kGlds = 512, kTab16 = 1024, kNoLen = 2048 };
typedef __attribute__((address_space(1))) void gvoid;
typedef __attribute__((address_space(3))) void lvoid;

template <int MODE>
__global__ __launch_bounds__(512, 6) void k_probe(const uint8_t* bytes, uint32_t nbytes, const uint64_t* st64,
                                                  const uint64_t* en64, const uint32_t* en32, uint32_t n, Cols c,
                                                  uint32_t tiles_per_wave) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(bytes), (short)0,
                                                                       (int)nbytes, 0x00020000);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = blockIdx.x * 8u + (threadIdx.x >> 6);
  const uint32_t ngroups = (n + 63u) >> 6;
  uint32_t g0 = wave * 4u * tiles_per_wave, g1 = g0 + 4u * tiles_per_wave;
  if (g1 > ngroups) g1 = ngroups;
  if (g0 >= g1) return;
  uint32_t acc = 0;
  auto ends = [&](uint32_t g, uint32_t& s, uint32_t& e) {
    const uint32_t r = (g << 6) + lane;
    if (r >= n) {
      s = e = 0;
      return;
    }
    if (MODE & kU64) {
      s = (uint32_t)st64[r];
      e = (uint32_t)en64[r];
    } else {
      e = en32[r];
      // start = the previous record's end: lane - 1's, lane 0 loads it
      uint32_t p = __builtin_amdgcn_mov_dpp(e, 0x138, 0xf, 0xf, false);  // wave_shr:1
      if (lane == 0) p = r ? en32[r - 1] : 0u;
      s = p;
      if ((MODE & kCheck) && s != (uint32_t)st64[r]) atomicAdd(c.sink + 1, 1u);
    }
  };
  __shared__ __attribute__((aligned(16))) uint32_t stage[8][1024 + 32];  // 4 KiB + slack per wave
  // kTabLds: 32 KiB more LDS per workgroup (k_tpl_lane's CRC position tables): 2 workgroups per CU
  constexpr uint32_t kPad = (MODE & kTabLds) ? ((MODE & kTab8) ? 2048u : (MODE & kTab16) ? 4096u : 8192u) : 1u;
  __shared__ uint32_t tabpad[kPad];
  if (MODE & kTabLds) {
    for (uint32_t i = threadIdx.x; i < kPad; i += 512u) tabpad[i] = i;
    __syncthreads();
  }
  uint32_t* st_w = stage[threadIdx.x >> 6];
  auto window = [&](uint32_t e, uint32_t (&w)[16]) {
    if (MODE & kStaged) {
      // the wave's 64 records are one span: coalesced 16-byte loads of it into LDS, then each lane
      // reads its window from LDS (aligned dwords + alignbyte)
      const uint32_t e_last = __builtin_amdgcn_readlane(e, 63), e_first = __builtin_amdgcn_readfirstlane(e);
      const uint32_t lo = (e_first >= 64u ? e_first - 64u : 0u) & ~15u;
      const uint32_t hi = e_last;
      for (uint32_t k = 0; k < 4u; ++k) {
        const uint32_t off = lo + 16u * (lane + 64u * k);
        if (off < hi) {
          const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
          *reinterpret_cast<u32x4*>(st_w + 4u * (lane + 64u * k)) = v;
        }
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // (lgkmcnt(0): the wave's LDS writes done)
      __builtin_amdgcn_wave_barrier();
      const uint32_t b0 = e >= 64u ? e - 64u - lo : 0u;
      const uint32_t q0 = b0 >> 2, sh = b0 & 3u;
      uint32_t prev = st_w[q0];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const uint32_t nx = st_w[q0 + i + 1];
        w[i] = __builtin_amdgcn_alignbyte(nx, prev, sh);
        prev = nx;
      }
      __builtin_amdgcn_wave_barrier();
      return;
    }
    const uint32_t voff = e >= 64u ? e - 64u : 0xffffff00u;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff + 16u * q, 0, 0));
      w[4 * q] = v.x;
      w[4 * q + 1] = v.y;
      w[4 * q + 2] = v.z;
      w[4 * q + 3] = v.w;
    }
  };
  auto proc = [&](uint32_t g, uint32_t s, uint32_t e, const uint32_t (&w)[16]) {
    const uint32_t r = (g << 6) + lane;
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) x ^= w[i] * (uint32_t)(2 * i + 1);
    if (MODE & kTabLds) x ^= tabpad[x & (kPad - 1u)];
    acc += x;
    if (MODE & kStore) {
      if (r < n) {
        if (!(MODE & kNoSV)) {
          c.status[r] = (int32_t)((x & 1u) & (e - s == 0u));  // 0 in practice
          c.verdict[r] = 7;
        }
        if (!(MODE & kNoOrd)) {
          c.ord0[r] = 1;
          c.ord1[r] = 2;
        }
        c.v[r] = w[10] & 0x7fu;
        c.boff[r] = e - 16u;
        if (!(MODE & kNoLen)) c.blen[r] = 12u;
      }
    }
  };
  if (MODE & kGlds) {
    // round 6: each wave's next window loaded straight into its LDS buffer (global_load_lds, lane-
    // linear: lane l's 16-byte piece q at q * 1 KiB + 16 l) while this group is processed from VGPRs
    auto issue = [&](uint32_t e) {
      const uint32_t voff = e >= 64u ? e - 64u : 0u;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        __builtin_amdgcn_global_load_lds((gvoid*)(bytes + voff + 16u * q), (lvoid*)(st_w + 256u * q), 16, 0, 0);
    };
    uint32_t sa, ea, sb = 0, eb = 0;
    ends(g0, sa, ea);
    issue(ea);
    if (g0 + 1u < g1) ends(g0 + 1u, sb, eb);
    for (uint32_t g = g0; g < g1; ++g) {
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
      asm volatile("" ::: "memory");
      uint32_t w[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(st_w + 256u * q + 4u * lane);
        w[4 * q] = v.x;
        w[4 * q + 1] = v.y;
        w[4 * q + 2] = v.z;
        w[4 * q + 3] = v.w;
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the buffer is read before it is refilled
      asm volatile("" ::: "memory");
      const uint32_t s_ = sa, e_ = ea;
      if (g + 1u < g1) {
        issue(eb);
        sa = sb;
        ea = eb;
        if (g + 2u < g1) ends(g + 2u, sb, eb);
      }
      proc(g, s_, e_, w);
    }
  } else if (MODE & kPipe) {
    uint32_t sa, ea, sb, eb;
    uint32_t wa[16];
    ends(g0, sa, ea);
    window(ea, wa);
    for (uint32_t g = g0; g < g1; ++g) {
      uint32_t wb[16];
      const bool more = g + 1u < g1;
      if (more) {
        ends(g + 1u, sb, eb);
        window(eb, wb);
      }
      proc(g, sa, ea, wa);
      if (!more) break;
#pragma unroll
      for (int i = 0; i < 16; ++i) wa[i] = wb[i];
      sa = sb;
      ea = eb;
    }
  } else {
    uint32_t s0, e0, s1, e1;
    ends(g0, s0, e0);
    ends(g0 + 1u, s1, e1);
    for (uint32_t g = g0; g < g1; g += 2) {
      uint32_t wa[16], wb[16];
      window(e0, wa);
      window(e1, wb);
      const uint32_t sa = s0, ea = e0, sb = s1, eb = e1;
      if (g + 2u < g1) {
        ends(g + 2u, s0, e0);
        ends(g + 3u, s1, e1);
      }
      proc(g, sa, ea, wa);
      if (g + 1u < g1) proc(g + 1u, sb, eb, wb);
    }
  }
  if (acc == 0x12345678u) c.sink[0] = acc;
}

template <int MODE>
float run(const uint8_t* b, uint32_t nb, const uint64_t* s64, const uint64_t* e64, const uint32_t* e32, uint32_t n,
          Cols c, uint32_t tpw, int reps) {
  const uint32_t groups = (n + 63) / 64, tiles = (groups + 3) / 4;
  const uint32_t waves = (tiles + tpw - 1) / tpw;
  const dim3 grid((waves + 7) / 8);
  hipEvent_t a, z;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&z));
  for (int i = 0; i < 3; ++i) k_probe<MODE><<<grid, 512>>>(b, nb, s64, e64, e32, n, c, tpw);
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) k_probe<MODE><<<grid, 512>>>(b, nb, s64, e64, e32, n, c, tpw);
  CK(hipEventRecord(z));
  CK(hipEventSynchronize(z));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, z));
  return ms / reps;
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 16777216u;
  std::vector<uint32_t> e32(n);
  std::vector<uint64_t> s64(n), e64(n);
  uint64_t pos = 0;
  uint32_t seed = 12345;
  for (uint32_t i = 0; i < n; ++i) {
    seed = seed * 1664525u + 1013904223u;
    const uint32_t len = (seed >> 28) < 2 ? 58 : 59;  // ~13 % one-byte labels
    s64[i] = pos;
    pos += len;
    e64[i] = pos;
    e32[i] = (uint32_t)pos;
  }
  const uint32_t nb = (uint32_t)pos;
  uint8_t* d_b;
  CK(hipMalloc(&d_b, nb + 64));
  CK(hipMemset(d_b, 0x5a, nb + 64));
  uint64_t *d_s64, *d_e64;
  uint32_t* d_e32;
  CK(hipMalloc(&d_s64, 8ull * n));
  CK(hipMalloc(&d_e64, 8ull * n));
  CK(hipMalloc(&d_e32, 4ull * n));
  CK(hipMemcpy(d_s64, s64.data(), 8ull * n, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_e64, e64.data(), 8ull * n, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_e32, e32.data(), 4ull * n, hipMemcpyHostToDevice));
  Cols c;
  CK(hipMalloc(&c.status, 4ull * n));
  CK(hipMalloc(&c.verdict, 1ull * n));
  CK(hipMalloc(&c.ord0, 2ull * n));
  CK(hipMalloc(&c.ord1, 2ull * n));
  CK(hipMalloc(&c.v, 8ull * n));
  CK(hipMalloc(&c.boff, 4ull * n));
  CK(hipMalloc(&c.blen, 4ull * n));
  CK(hipMalloc(&c.sink, 64));
  const int reps = 20;
  CK(hipMemset(c.sink, 0, 64));
  run<kCheck>(d_b, nb, d_s64, d_e64, d_e32, n, c, 2, 1);
  uint32_t bad[2] = {0, 0};
  CK(hipMemcpy(bad, c.sink, 8, hipMemcpyDeviceToHost));
  printf("{\"dpp_wave_shr_check_mismatches\": %u}\n", bad[1]);
  printf("{\"records\": %u, \"bytes\": %u}\n", n, nb);
  auto rep_ = [&](const char* name, int mode, uint32_t tpw, float ms) {
    const double rd = (double)nb + (mode & kU64 ? 16.0 : 4.0) * n;
    const double wr = mode & kStore ? (25.0 - (mode & kNoSV ? 5.0 : 0.0) - (mode & kNoOrd ? 4.0 : 0.0) -
                                       (mode & kNoLen ? 4.0 : 0.0)) * n : 0.0;
    printf("{\"variant\": \"%s\", \"tiles_per_wave\": %u, \"ms\": %.4f, \"alg_TBps\": %.3f, \"frac\": %.4f, "
           "\"framed_GiBps\": %.1f}\n",
           name, tpw, ms, (rd + wr) / ms / 1e9, (rd + wr) / ms / 1e9 / 8.0, nb / (ms / 1e3) / 1073741824.0);
    fflush(stdout);
  };
  for (int rep = 0; rep < 2; ++rep)
    for (uint32_t tpw : {1u, 2u}) {
      constexpr int V = kStore | kNoSV | kNoOrd | kNoLen;
      rep_("v12_lane", V, tpw, run<V>(d_b, nb, d_s64, d_e64, d_e32, n, c, tpw, reps));
      rep_("v12_lane_tab", V | kTabLds, tpw, run<V | kTabLds>(d_b, nb, d_s64, d_e64, d_e32, n, c, tpw, reps));
      rep_("v12_glds_tab16", V | kGlds | kTabLds | kTab16, tpw,
           run<V | kGlds | kTabLds | kTab16>(d_b, nb, d_s64, d_e64, d_e32, n, c, tpw, reps));
      rep_("v12_glds", V | kGlds, tpw, run<V | kGlds>(d_b, nb, d_s64, d_e64, d_e32, n, c, tpw, reps));
      rep_("read_glds", kGlds, tpw, run<kGlds>(d_b, nb, d_s64, d_e64, d_e32, n, c, tpw, reps));
      rep_("read_lane", 0, tpw, run<0>(d_b, nb, d_s64, d_e64, d_e32, n, c, tpw, reps));
    }
  for (int rep = 0; rep < 0; ++rep)
    for (uint32_t tpw : {1u}) {
      rep_("rw_u32_tab", kStore | kTabLds, tpw, run<kStore | kTabLds>(d_b, nb, d_s64, d_e64, d_e32, n, c, tpw, reps));
      rep_("rw_u32_staged_tab8", kStore | kStaged | kTabLds | kTab8, tpw,
           run<kStore | kStaged | kTabLds | kTab8>(d_b, nb, d_s64, d_e64, d_e32, n, c, tpw, reps));
      rep_("rw_u32_values_only_staged_tab8", kStore | kNoSV | kNoOrd | kStaged | kTabLds | kTab8, tpw,
           run<kStore | kNoSV | kNoOrd | kStaged | kTabLds | kTab8>(d_b, nb, d_s64, d_e64, d_e32, n, c, tpw, reps));
      rep_("rw_u32_noord_staged_tab8", kStore | kNoOrd | kStaged | kTabLds | kTab8, tpw,
           run<kStore | kNoOrd | kStaged | kTabLds | kTab8>(d_b, nb, d_s64, d_e64, d_e32, n, c, tpw, reps));
    }
  return 0;
}
