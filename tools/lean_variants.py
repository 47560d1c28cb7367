#!/usr/bin/env python3
"""Measurement-only variants of k_tpl_lane (never the product library): patched copies of
csrc/tfrg_tpl.hip built into tfr_reader/libtfrg_<name>.so (load with TFRG_LIB=...).
usage: lean_variants.py name [name ...]"""
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
CS = REPO / "tfrecords-reader_amd" / "csrc"
SRC = (CS / "tfrg_tpl.hip").read_text()

VARIANTS = {
    # no column stores (read side alone; wrong results)
    "nostore": [("      if (ok) {\n        o.status[r] = TFRG_OK;", "      if (ok && A.n_tpl > 99) {\n        o.status[r] = TFRG_OK;"),
                ("        if (ok) {\n          T.ord[r] = (uint16_t)rank;", "        if (ok && A.n_tpl > 99) {\n          T.ord[r] = (uint16_t)rank;")],
    # dword-aligned window loads (+1 dword) and a per-lane byte funnel shift
    "align4": [("""    uint32_t w[W];
#pragma unroll
    for (int q = 0; q < W / 4; ++q) {
      const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff + 16u * q, 0, 0));
      w[4 * q] = v.x;
      w[4 * q + 1] = v.y;
      w[4 * q + 2] = v.z;
      w[4 * q + 3] = v.w;
    }""", """    uint32_t w[W + 1];
    const uint32_t va = voff & ~3u, sh = voff & 3u;
#pragma unroll
    for (int q = 0; q < W / 4; ++q) {
      const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, va + 16u * q, 0, 0));
      w[4 * q] = v.x;
      w[4 * q + 1] = v.y;
      w[4 * q + 2] = v.z;
      w[4 * q + 3] = v.w;
    }
    w[W] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, va + 4u * W, 0, 0);
#pragma unroll
    for (int i = 0; i < W; ++i) w[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);""")],
}


def build(name: str) -> Path:
    src = SRC
    for old, new in VARIANTS[name]:
        assert src.count(old) == 1, (name, old[:60])
        src = src.replace(old, new)
    d = Path("/tmp/lean_var")
    d.mkdir(exist_ok=True)
    f = d / f"tfrg_tpl_{name}.hip"
    f.write_text(src)
    obj = d / f"tfrg_tpl_{name}.o"
    inc = f"-I{CS}"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", inc, "-c", str(f),
                    "-o", str(obj)], check=True, cwd=CS)
    objs = [str(CS / "build" / o) for o in ("tfrg_kernels.o", "tfrg_bytes.o", "tfrg_capi.o", "tfrg_stream.o",
                                             "tfrg_host.o", "tfrg_cpu.o")]
    out = REPO / "tfrecords-reader_amd" / "tfr_reader" / f"libtfrg_{name}.so"
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-o", str(out), str(obj), *objs,
                    "-lz", "-lpthread"], check=True)
    return out


if __name__ == "__main__":
    for n in sys.argv[1:]:
        print(build(n))
