#!/usr/bin/env python3
"""Measurement-only builds of libtfrg (never the product library): the kernel sources copied to a
temporary directory, patched, built into tfr_reader/libtfrg_<name>.so (load with TFRG_LIB=...), for
paired A/Bs on the GPU box (tools/ab.sh). Patches are (file, old, new) string replacements; a
variant whose patch no longer applies is an error.  usage: variants.py name [name ...]"""
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
CS = REPO / "tfrecords-reader_amd" / "csrc"

VARIANTS = {
    # k_tpl_lane printing every record it leaves to k_lane_count (debug)
    "dbgtpl": [("tfrg_tpl.hip", "#include <hip/hip_runtime.h>", "#define TFRG_DEBUG_TPL 1\n#include <hip/hip_runtime.h>")],
    # k_tpl_lane: one tile (4 groups) per wave on large batches instead of two
    "t1": [("tfrg_tpl.hip", "a2.gpw = need < (uint32_t)num_cus ? 2u : need >= 8u * (uint32_t)num_cus ? 8u : 4u;",
            "a2.gpw = need < (uint32_t)num_cus ? 2u : 4u;"),
           ("tfrg_tpl.hip", "if (split_on && a2.gpw == 8u) {", "if (split_on && a2.gpw >= 4u) {")],
    # k_tpl_lane: two groups per step (both windows loaded together) at 5 waves/SIMD (96 VGPRs)
    "g2lb5": [("tfrg_tpl.hip", "#define TFRG_TPL_GROUPS_PER_STEP 1", "#define TFRG_TPL_GROUPS_PER_STEP 2"),
              ("tfrg_tpl.hip", "__launch_bounds__(kTplBlock, W == 16 ? 6 : (W == 32 ? 4 : 2))",
               "__launch_bounds__(kTplBlock, W == 16 ? 5 : (W == 32 ? 4 : 2))")],
    "t1g2lb5": [("tfrg_tpl.hip", "a2.gpw = need < (uint32_t)num_cus ? 2u : need >= 8u * (uint32_t)num_cus ? 8u : 4u;",
                 "a2.gpw = need < (uint32_t)num_cus ? 2u : 4u;"),
                ("tfrg_tpl.hip", "if (split_on && a2.gpw == 8u) {", "if (split_on && a2.gpw >= 4u) {"),
                ("tfrg_tpl.hip", "#define TFRG_TPL_GROUPS_PER_STEP 1", "#define TFRG_TPL_GROUPS_PER_STEP 2"),
                ("tfrg_tpl.hip", "__launch_bounds__(kTplBlock, W == 16 ? 6 : (W == 32 ? 4 : 2))",
                 "__launch_bounds__(kTplBlock, W == 16 ? 5 : (W == 32 ? 4 : 2))")],
    # k_tpl_lane at 8 waves/SIMD (64 VGPRs)
    "lb8v3": [("tfrg_tpl.hip", "__launch_bounds__(kTplBlock, W == 16 ? 6 : (W == 32 ? 4 : 2))",
               "__launch_bounds__(kTplBlock, W == 16 ? 8 : (W == 32 ? 4 : 2))")],
    # k_tail_count in 1024-thread workgroups, one per CU (the streaming CRC's 70 KiB of LDS tables
    # loaded 256 times instead of 512; the same 16 waves per CU)
    "tail1024": [("tfrg_kernels.hip", "constexpr uint32_t kTailBlock = 512;", "constexpr uint32_t kTailBlock = 1024;"),
                 ("tfrg_kernels.hip", "__global__ __launch_bounds__(kTailBlock, 2) void k_tail_count",
                  "__global__ __launch_bounds__(kTailBlock, 4) void k_tail_count")],
    # k_tpl_lane without its column stores (read side alone; wrong results)
    "nostore": [("tfrg_tpl.hip", "      if (ok) {\n        o.status[r] = TFRG_OK;",
                 "      if (ok && A.n_tpl > 99) {\n        o.status[r] = TFRG_OK;"),
                ("tfrg_tpl.hip", "        if (ok) {\n          T.ord[r] = (uint16_t)rank;",
                 "        if (ok && A.n_tpl > 99) {\n          T.ord[r] = (uint16_t)rank;")],
    # k_tpl_lane window loads with the streaming (slc) cache policy
    "ntload": [("tfrg_tpl.hip", "__builtin_amdgcn_raw_buffer_load_b128(rsrc, voff + 16u * q, 0, 0)",
                "__builtin_amdgcn_raw_buffer_load_b128(rsrc, voff + 16u * q, 0, 2)")],
    # k_tpl_lane with every valid lane taking template 0 (wrong results; all stores kept)
    "fakehit": [("tfrg_tpl.hip", "      const bool ok = cand && diff == 0u && crc_mask(lin ^ tp[kLtK]) == w[W - 1];",
                 "      const bool ok = t == 0u && (diff | lin | 1u) != 0u && (g << 6) + lane < B.n;")],
    # the same with the window loads made coalesced (lane j: 16 bytes at j * 16 of a 4 KiB span)
    "fakehit_coal": [("tfrg_tpl.hip", "      const bool ok = cand && diff == 0u && crc_mask(lin ^ tp[kLtK]) == w[W - 1];",
                      "      const bool ok = t == 0u && (diff | lin | 1u) != 0u && (g << 6) + lane < B.n;"),
                     ("tfrg_tpl.hip", "    const uint32_t voff = full ? (uint32_t)e - 4u * W : 0xffffff00u;",
                      "    const uint32_t voff = full ? ((gg * 3712u) & ~15u) + 16u * lane - 48u * lane / 16u * 0u : 0xffffff00u;"),
                     ("tfrg_tpl.hip", "raw_buffer_load_b128(rsrc, voff + 16u * q, 0, 0)",
                      "raw_buffer_load_b128(rsrc, voff + 1024u * q, 0, 0)")],
    # k_tail_count without role 1 (the exact walker): the streaming CRC's registers alone (timing only)
    "crc_only": [("tfrg_kernels.hip", "  role_slow_count<1, COMPAT, GORD, kTailBlock>(B, sc, o, crc_tab, lane_max);\n", "")],
    # k_tpl_lane with four / three tiles per wave on large batches (fewer workgroups, table copies)
    "tpw4": [("tfrg_tpl.hip", "const uint32_t per_wave = need >= 8u * (uint32_t)num_cus ? 2u : 1u;",
              "const uint32_t per_wave = need >= 16u * (uint32_t)num_cus ? 4u : need >= 8u * (uint32_t)num_cus ? 2u : 1u;")],
    "tpw3": [("tfrg_tpl.hip", "const uint32_t per_wave = need >= 8u * (uint32_t)num_cus ? 2u : 1u;",
              "const uint32_t per_wave = need >= 12u * (uint32_t)num_cus ? 3u : need >= 8u * (uint32_t)num_cus ? 2u : 1u;")],
    # k_tpl_lane with a whole tile (four groups) per step (no half-tile mode: large batches only)
    "g4": [("tfrg_tpl.hip", "  uint32_t t = t0, p = A.half ? (w0 & 1u) << 1 : 0u;\n  uint64_t s0, e0, s1, e1;\n  offsets(4u * t + p, s0, e0);\n  offsets(4u * t + p + 1u, s1, e1);\n  while (t < ntiles) {\n    const uint32_t ga = 4u * t + p, gb = ga + 1u;\n    uint32_t wa[W], wb[W];\n    window(wa, in_batch(ga, s0, e0), e0, ga);\n    window(wb, in_batch(gb, s1, e1), e1, gb);\n    const uint64_t sa = s0, ea = e0, sb = s1, eb = e1;\n    // the next step's offsets\n    const uint32_t tn = p ? t + nw : t, pn = p ^ 2u;\n    offsets(4u * tn + pn, s0, e0);\n    offsets(4u * tn + pn + 1u, s1, e1);\n    proc(wa, ga, sa, ea);\n    if (gb < ngroups) proc(wb, gb, sb, eb);", '  uint32_t t = t0, p = 0u;\n  uint64_t s0, e0, s1, e1, s2, e2, s3, e3;\n  offsets(4u * t, s0, e0);\n  offsets(4u * t + 1u, s1, e1);\n  offsets(4u * t + 2u, s2, e2);\n  offsets(4u * t + 3u, s3, e3);\n  while (t < ntiles) {\n    const uint32_t ga = 4u * t, gb = ga + 1u;\n    uint32_t wa[W], wb[W], wc[W], wd[W];\n    window(wa, in_batch(ga, s0, e0), e0, ga);\n    window(wb, in_batch(gb, s1, e1), e1, gb);\n    window(wc, in_batch(ga + 2u, s2, e2), e2, ga + 2u);\n    window(wd, in_batch(ga + 3u, s3, e3), e3, ga + 3u);\n    const uint64_t sa = s0, ea = e0, sb = s1, eb = e1, sc = s2, ec = e2, sd = s3, ed = e3;\n    const uint32_t tn = t + nw, pn = 2u;\n    offsets(4u * tn, s0, e0);\n    offsets(4u * tn + 1u, s1, e1);\n    offsets(4u * tn + 2u, s2, e2);\n    offsets(4u * tn + 3u, s3, e3);\n    proc(wa, ga, sa, ea);\n    if (gb < ngroups) proc(wb, gb, sb, eb);\n    if (ga + 2u < ngroups) proc(wc, ga + 2u, sc, ec);\n    if (ga + 3u < ngroups) proc(wd, ga + 3u, sd, ed);\n    p = 2u;\n    const uint32_t gbb = ga + 3u;\n    if (gbb + 1u >= ngroups) { if (lane < A.n_slots && acc) A.tsum[lane * A.tile_stride + t] = acc; break; }\n    if (lane < A.n_slots && acc) A.tsum[lane * A.tile_stride + t] = acc;\n    acc = 0;\n    t = tn;\n    continue;')],
    # k_tpl_lane at 8 waves/SIMD (64 VGPRs: 4 workgroups per CU instead of 3; spills a few registers)
    "lb8": [("tfrg_tpl.hip", "__launch_bounds__(kTplBlock, W == 16 ? 6 : (W == 32 ? 4 : 2))",
             "__launch_bounds__(kTplBlock, W == 16 ? 8 : (W == 32 ? 4 : 2))")],
    # k_tail_gather without the float copies / the packed int64 decode / int64_ring's pass B
    # (VALU attribution by PMC; wrong results)
    "g_nofloat": [("tfrg_kernels.hip", "  uint64_t m = __ballot(isf);", "  uint64_t m = 0;")],
    "g_noint64": [("tfrg_kernels.hip", "  int rr = int64_ring<COMPAT>(fs, o, iv, bo, bl, cnt, dst, lane, ring);", "  int rr = 1;")],
    "g_nopassb": [("tfrg_kernels.hip", "    while (gtot - gb >= 64u) pass_b(64u);\n", "    gb = gtot;\n"),
                  ("tfrg_kernels.hip", "  if (gtot > gb) pass_b(gtot - gb);", "  gb = gtot;")],
    # k_tpl_lane without the row-split stores of placed slots (identity rows; wrong row splits)
    "nors": [("tfrg_tpl.hip", "            T.rs[r] = r;\n", "")],
    # the same without the key-order stores too (wrong row splits and key order)
    "nors_noord": [("tfrg_tpl.hip", "            T.rs[r] = r;\n", ""),
                   ("tfrg_tpl.hip", "          T.ord[r] = (uint16_t)rank;\n", "")],
    # int64_ring pass A: a body's byte mask in a dword from saturating subtractions
    "c3bm": [("tfrg_kernels.hip",
              "      const uint32_t lo = sbs > Q ? sbs - Q : 0u, hi0 = sbe > Q ? sbe - Q : 0u, hi = hi0 < 4u ? hi0 : 4u;\n"
              "      if (hi > lo) {  // (1 <= hi <= 4, lo <= 3: both shifts below 32)\n"
              "        bm = (0xffffffffu >> (32u - 8u * hi)) & (0xffffffffu << (8u * lo));\n",
              "      const uint32_t lo = __builtin_elementwise_sub_sat(sbs, Q), hi0 = __builtin_elementwise_sub_sat(sbe, Q), hi = hi0 < 4u ? hi0 : 4u;\n"
              "      if (hi > lo) {\n"
              "        bm = ~(0xfffffffeu << (8u * hi - 1u)) & (0xffffffffu << (8u * lo));\n")],
    # k_spine without its every-slot-placed fast path (the per-slot fast path and last-workgroup pass)
    "noallp": [("tfrg_kernels.hip", "  const bool allp = spec && n_slots <= (uint32_t)kSpineBlock &&",
                "  const bool allp = false && spec && n_slots <= (uint32_t)kSpineBlock &&")],
    # k_down_gather's placed-slot mask by one thread per workgroup, slot after slot
    "serialpm": [("tfrg_kernels.hip",
                  "  const uint64_t pmask = sc.spec ? (uint64_t)__ballot(lane < S && spec_placed(sc.spec, o, lane)) : 0ull;\n",
                  "  uint64_t pmask = 0;\n  if (sc.spec)\n    for (uint32_t k = 0; k < S && k < 64u; ++k) pmask |= (uint64_t)spec_placed(sc.spec, o, k) << k;\n"
                  "  pmask = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(pmask >> 32)) << 32) | __builtin_amdgcn_readfirstlane((uint32_t)pmask);\n")],
    # k_tpl_lane without the status / verdict stores (wrong results)
    "nostatus": [("tfrg_tpl.hip", "        o.status[r] = TFRG_OK;\n        o.verdict[r] = (uint8_t)kHitVerdict;\n", "")],
    # k_tpl_lane ablations (round 6; timing only, wrong results): no payload CRC / no template
    # match / no slot extraction and column stores / none of the three
    "abl_nocrc": [('tfrg_tpl.hip', '      if (chain_u < (uint32_t)(W - 9)) {', '      if (false) {'), ('tfrg_tpl.hip', '      TFRG_LIN(0) TFRG_LIN(1) TFRG_LIN(2) TFRG_LIN(3) TFRG_LIN(4) TFRG_LIN(5) TFRG_LIN(6) TFRG_LIN(7)\n', ''), ('tfrg_tpl.hip', '      const bool ok = act && diff == 0u && crc_mask(lin ^ meta.y) == w[W - 1];', '      const bool ok = act && diff == 0u && (lin | meta.y | w[W - 1] | c | 1u) != 0u;')],
    "abl_nomatch": [('tfrg_tpl.hip', '        diff |= ((w[4 * q] ^ bm.x) & mm.x) | ((w[4 * q + 1] ^ bm.y) & mm.y) | ((w[4 * q + 2] ^ bm.z) & mm.z) |\n                ((w[4 * q + 3] ^ bm.w) & mm.w);', '        diff |= 0u * (bm.x & mm.x);')],
    "abl_noslot": [('tfrg_tpl.hip', '    if (__ballot(hit)) {\n      const uint32_t* ts', '    if (__ballot(hit) && A.n_slots == 12345u) {\n      const uint32_t* ts')],
    "abl_none": [('tfrg_tpl.hip', '      if (chain_u < (uint32_t)(W - 9)) {', '      if (false) {'), ('tfrg_tpl.hip', '      TFRG_LIN(0) TFRG_LIN(1) TFRG_LIN(2) TFRG_LIN(3) TFRG_LIN(4) TFRG_LIN(5) TFRG_LIN(6) TFRG_LIN(7)\n', ''), ('tfrg_tpl.hip', '      const bool ok = act && diff == 0u && crc_mask(lin ^ meta.y) == w[W - 1];', '      const bool ok = act && diff == 0u && (lin | meta.y | w[W - 1] | c | 1u) != 0u;'), ('tfrg_tpl.hip', '        diff |= ((w[4 * q] ^ bm.x) & mm.x) | ((w[4 * q + 1] ^ bm.y) & mm.y) | ((w[4 * q + 2] ^ bm.z) & mm.z) |\n                ((w[4 * q + 3] ^ bm.w) & mm.w);', '        diff |= 0u * (bm.x & mm.x);'), ('tfrg_tpl.hip', '    if (__ballot(hit)) {\n      const uint32_t* ts', '    if (__ballot(hit) && A.n_slots == 12345u) {\n      const uint32_t* ts')],
    # k_tpl_lane: 16 / 32 groups per wave on large batches (fewer workgroups, fewer table copies)
    "gpw16": [('tfrg_tpl.hip', 'a2.gpw = need < (uint32_t)num_cus / 2u ? 1u : need < (uint32_t)num_cus ? 2u : need >= 8u * (uint32_t)num_cus ? 8u : 4u;', 'a2.gpw = need < (uint32_t)num_cus / 2u ? 1u : need < (uint32_t)num_cus ? 2u : need >= 16u * (uint32_t)num_cus ? 16u : need >= 8u * (uint32_t)num_cus ? 8u : 4u;'), ('tfrg_tpl.hip', 'if (split_on && a2.gpw == 8u) {', 'if (split_on && a2.gpw >= 8u) {')],
    "gpw32": [('tfrg_tpl.hip', 'a2.gpw = need < (uint32_t)num_cus / 2u ? 1u : need < (uint32_t)num_cus ? 2u : need >= 8u * (uint32_t)num_cus ? 8u : 4u;', 'a2.gpw = need < (uint32_t)num_cus / 2u ? 1u : need < (uint32_t)num_cus ? 2u : need >= 32u * (uint32_t)num_cus ? 32u : need >= 8u * (uint32_t)num_cus ? 8u : 4u;'), ('tfrg_tpl.hip', 'if (split_on && a2.gpw == 8u) {', 'if (split_on && a2.gpw >= 8u) {')],
    # k_tpl_lane on large batches: {3, 6} workgroups per CU in all, each wave one contiguous run of
    # groups (a table copy per resident workgroup, not per 64 groups)
    "persist3": [('tfrg_tpl.hip', 'a2.gpw = need < (uint32_t)num_cus / 2u ? 1u : need < (uint32_t)num_cus ? 2u : need >= 8u * (uint32_t)num_cus ? 8u : 4u;', 'a2.gpw = need < (uint32_t)num_cus / 2u ? 1u : need < (uint32_t)num_cus ? 2u : need >= 8u * (uint32_t)num_cus ? ((groups + 3u * (uint32_t)num_cus * 8u - 1u) / (3u * (uint32_t)num_cus * 8u) + 3u) & ~3u : 4u;'), ('tfrg_tpl.hip', 'if (split_on && a2.gpw == 8u) {', 'if (split_on && a2.gpw == 0xfffu) {')],
    "persist6": [('tfrg_tpl.hip', 'a2.gpw = need < (uint32_t)num_cus / 2u ? 1u : need < (uint32_t)num_cus ? 2u : need >= 8u * (uint32_t)num_cus ? 8u : 4u;', 'a2.gpw = need < (uint32_t)num_cus / 2u ? 1u : need < (uint32_t)num_cus ? 2u : need >= 8u * (uint32_t)num_cus ? ((groups + 6u * (uint32_t)num_cus * 8u - 1u) / (6u * (uint32_t)num_cus * 8u) + 3u) & ~3u : 4u;'), ('tfrg_tpl.hip', 'if (split_on && a2.gpw == 8u) {', 'if (split_on && a2.gpw == 0xfffu) {')],
    # k_tpl_lane at 7 waves/SIMD (72 VGPRs)
    "lb7": [("tfrg_tpl.hip", "__launch_bounds__(kTplBlock, W == 16 ? 6 : (W == 32 ? 4 : 2))",
             "__launch_bounds__(kTplBlock, W == 16 ? 7 : (W == 32 ? 4 : 2))")],
    # the streaming CRC's per-record flush (timing only, wrong verdicts): none of it / without the
    # x^(8192 jlo) shift of split slices
    "flush_none": [("tfrg_kernels.hip", "                                       uint32_t n_slots, uint32_t lane) {\n  const uint64_t bas = rl64(w.base, k);",
                    "                                       uint32_t n_slots, uint32_t lane) {\n  if (n_slots != 0xfffffffeu) return;\n  const uint64_t bas = rl64(w.base, k);")],
    "flush_nojlo": [("tfrg_kernels.hip", "  if (jlo) {  // x x^(8192 jlo)", "  if (jlo && n_slots == 0xfffffffeu) {  // x x^(8192 jlo)")],
    # k_tail_count: the streaming CRC (role 2) before the exact walker (role 1), so its prologue does
    # not wait for role 1's slow-list count
    "role2first": [("tfrg_kernels.hip", """  role_slow_count<1, COMPAT, GORD, kTailBlock>(B, sc, o, crc_tab, lane_max);
  __syncthreads();  // (the LDS tables are reloaded by role 2)
  role_crc_stream<kTailBlock>(B, o, crc_tab, consts, sc.n_slots);
  if (finish) {""", """  role_crc_stream<kTailBlock>(B, o, crc_tab, consts, sc.n_slots);
  __syncthreads();  // (the LDS tables are reloaded by role 1)
  role_slow_count<1, COMPAT, GORD, kTailBlock>(B, sc, o, crc_tab, lane_max);
  if (finish) {""")],
}


VARIANTS["noboff"] = [("tfrg_tpl.hip", "                reinterpret_cast<uint32_t*>(T.v1)[r] = lx;\n                if (T.kind == TFRG_KIND_BYTES",
                        "                if (T.kind != TFRG_KIND_BYTES) reinterpret_cast<uint32_t*>(T.v1)[r] = lx;\n                if (T.kind == TFRG_KIND_BYTES")]  # (measurement only: the bytes offsets not stored)


# (measurement only) the streaming CRC's loads and group structure without its arithmetic: what the
# role-2 load pattern achieves on its own (wrong verdicts)
VARIANTS["crc_loadonly"] = [("tfrg_kernels.hip", """  auto process = [&](const Grp& g) {
""", """  auto process = [&](const Grp& g) {
    if (n_slots != 0xfffffffeu) {
#pragma unroll
      for (int d = 0; d < kCrcDepth; ++d) S ^= g.wd[d].x ^ g.wd[d].y ^ g.wd[d].z ^ g.wd[d].w;
      return;
    }
""")]


# (measurement) streaming-CRC groups that never cross a record (a record's last group is partial;
# its unused loads repeat the group's last chunk instead of reading ahead)
VARIANTS["crc_align"] = [("tfrg_kernels.hip", """    if (!g.n) return;
    const uint64_t rl = Rs + g.n - 1u;
    const uint32_t k0 = (uint32_t)__popcll(__ballot(w.base <= Rs)) - 1u;
    const uint32_t kl = (uint32_t)__popcll(__ballot(w.base <= rl)) - 1u;""", """    if (!g.n) return;
    const uint32_t k0 = (uint32_t)__popcll(__ballot(w.base <= Rs)) - 1u;
    {
      const uint64_t re = rl64(w.base, k0 + 1u);
      if (Rs + g.n > re) g.n = (uint32_t)(re - Rs);
    }
    const uint64_t rl = Rs + g.n - 1u;
    const uint32_t kl = k0;"""),
    ("tfrg_kernels.hip", """        g.wd[d] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(brs, vo + 1024u * d, 0, 0));""",
     """        g.wd[d] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(brs, vo + 1024u * ((uint32_t)d < g.n ? (uint32_t)d : g.n - 1u), 0, 0));""")]


def build(name: str) -> Path:
    with tempfile.TemporaryDirectory() as td:
        d = Path(td) / "pkg" / "csrc"  # (the sources include ../../include)
        shutil.copytree(CS, d, ignore=shutil.ignore_patterns("build*"))
        (Path(td) / "include").symlink_to(REPO / "include")
        for f, old, new in VARIANTS[name]:
            src = (d / f).read_text()
            assert src.count(old) == 1, (name, f, old[:60])
            (d / f).write_text(src.replace(old, new))
        out = REPO / "tfrecords-reader_amd" / "tfr_reader" / f"libtfrg_{name}.so"
        subprocess.run(["make", "-j8", f"OUT={out}", f"PYMOD={Path(td) / 'unused.so'}", f"{out}"], cwd=d, check=True,
                       stdout=subprocess.DEVNULL)
    return out


if __name__ == "__main__":
    for n in sys.argv[1:]:
        print(build(n))
