"""Generate the committed golden fixtures from the REFERENCE itself (build container only).

Runs kmkolasinski/tfrecords-reader's own Cython decoder/indexer (built from /root/reference by
oracle/build_ref.sh into oracle/_ref/) and its protobuf schema (tfr_example_pb2, upb) to record
input/output vectors. The reference never travels: only the data written here is committed.

Outputs (tests/golden/):
  cases.jsonl        one payload per line: hex bytes + the reference's decode outcome
                     (dict in key order / exception type + message / crash) and, where upb
                     parses it, the protobuf-spec outcome.
  files/<name>.tfrecord + files/<name>.json
                     TFRecord files written with the reference test recipes (tests/utils.py:
                     24-105) plus C0/C2/C3-shaped minis and framing edge cases; the JSON holds
                     the reference indexer pointers (indexer.pyx:212-252), the reference .idx
                     bytes (indexer.pyx:260-285), per-record decode outcomes and the CRC-32C
                     verdicts computed by a bitwise spec implementation (the reference has none).

Usage:  oracle/build_ref.sh && python tests/golden/gen_golden.py
"""

from __future__ import annotations

import base64
import importlib.util
import json
import os
import random
import signal
import struct
import subprocess
import sys
import tempfile
from pathlib import Path

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
REF = Path(os.environ.get("REF", "/root/reference"))
REF_BUILD = REPO / "oracle" / "_ref"
FILES = HERE / "files"


def _load(name: str, path: Path):
    spec = importlib.util.spec_from_file_location(name, str(path))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def load_reference():
    suffix = [p for p in REF_BUILD.glob("decoder*.so")]
    if not suffix:
        raise SystemExit("run oracle/build_ref.sh first")
    dec = _load("tfr_reader.cython.decoder", suffix[0])
    idx = _load("tfr_reader.cython.indexer", next(REF_BUILD.glob("indexer*.so")))
    pb2 = _load("tfr_example_pb2", REF / "src/tfr_reader/example/tfr_example_pb2.py")
    return dec, idx, pb2


# ----------------------------------------------------------------------------------------------
# minimal independent protobuf writer for hand-built (also malformed) payloads
# ----------------------------------------------------------------------------------------------
def enc(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def ld(fn: int, payload: bytes) -> bytes:
    return enc((fn << 3) | 2) + enc(len(payload)) + payload


def entry(key: bytes, feat: bytes) -> bytes:
    return ld(1, ld(1, key) + ld(2, feat))


def example(*entries: bytes) -> bytes:
    return ld(1, b"".join(entries))


def i64(*vals: int) -> bytes:
    return ld(3, ld(1, b"".join(enc(v) for v in vals)))


def f32(*vals: float) -> bytes:
    return ld(2, ld(1, b"".join(struct.pack("<f", v) for v in vals)))


def byt(*vals: bytes) -> bytes:
    return ld(1, b"".join(ld(1, v) for v in vals))


# ----------------------------------------------------------------------------------------------
# running the reference decoder in a crash-tolerant child process
# ----------------------------------------------------------------------------------------------
CHILD = r"""
import sys, json, importlib.util, signal, struct
def load(name, path):
    spec = importlib.util.spec_from_file_location(name, path); m = importlib.util.module_from_spec(spec)
    sys.modules[name] = m; spec.loader.exec_module(m); return m
dec = load("tfr_reader.cython.decoder", sys.argv[1])
def fbits(x):
    return struct.unpack("<I", struct.pack("<f", x))[0]
def alarm(*_): raise TimeoutError("hang")
signal.signal(signal.SIGALRM, alarm)
for line in sys.stdin:
    raw = bytes.fromhex(line.strip())
    signal.alarm(2)
    try:
        ex = dec.example_from_bytes(raw)
        feats = ex.features
        if feats is None:
            out = {"exc": "AttributeError", "msg": "'NoneType' object has no attribute 'feature'"}
        else:
            d = []
            for k, f in feats.feature.items():
                kind = f.WhichOneof("kind")
                v = getattr(f, kind).value
                if kind == "float_list": v = [fbits(x) for x in v]
                elif kind == "bytes_list": v = [b.hex() for b in v]
                else: v = list(v)
                d.append([k.encode("utf-8").hex(), kind, v])
            out = {"ok": d}
    except TimeoutError:
        out = {"hang": True}
    except BaseException as e:
        out = {"exc": type(e).__name__, "msg": str(e)}
    signal.alarm(0)
    sys.stdout.write(json.dumps(out) + "\n"); sys.stdout.flush()
"""


def run_reference(payloads: list[bytes]) -> list[dict]:
    """Decode every payload with the reference; a segfault marks that case and the rest re-run."""
    so = str(next(REF_BUILD.glob("decoder*.so")))
    results: list[dict] = []
    i = 0
    while i < len(payloads):
        proc = subprocess.run(
            [sys.executable, "-c", CHILD, so],
            input="\n".join(p.hex() for p in payloads[i:]) + "\n",
            capture_output=True,
            text=True,
            timeout=600,
        )
        got = [json.loads(x) for x in proc.stdout.splitlines() if x.strip()]
        results.extend(got)
        i += len(got)
        if proc.returncode != 0 and i < len(payloads):
            results.append({"crash": -proc.returncode if proc.returncode < 0 else proc.returncode})
            i += 1
    return results


def run_upb(pb2, payloads: list[bytes]) -> list[dict | None]:
    out: list[dict | None] = []
    for raw in payloads:
        try:
            ex = pb2.Example()
            ex.ParseFromString(raw)
        except Exception:  # noqa: BLE001
            out.append(None)
            continue
        d = []
        for k in ex.features.feature:
            f = ex.features.feature[k]
            kind = f.WhichOneof("kind")
            if kind is None:
                out_k = None
                break
            v = getattr(f, kind).value
            if kind == "float_list":
                v = [struct.unpack("<I", struct.pack("<f", x))[0] for x in v]
            elif kind == "bytes_list":
                v = [b.hex() for b in v]
            else:
                v = list(v)
            d.append([k.encode("utf-8").hex(), kind, v])
        else:
            out_k = d
        out.append({"ok": out_k} if out_k is not None else None)
    return out


# ----------------------------------------------------------------------------------------------
# case catalogue
# ----------------------------------------------------------------------------------------------
def edge_cases() -> list[tuple[str, bytes]]:
    k = b"k"
    C = [
        ("empty example", b""),
        ("empty features", ld(1, b"")),
        ("feature no kind", ld(1, ld(1, ld(1, k) + ld(2, b"")))),
        ("map entry key only", ld(1, ld(1, ld(1, k)))),
        ("map entry empty", ld(1, ld(1, b""))),
        ("empty key", example(entry(b"", i64()))),
        ("empty int64 list", example(entry(k, i64()))),
        ("empty float list", example(entry(k, f32()))),
        ("empty bytes list", example(entry(k, byt()))),
        ("non-packed int64 wire0", example(entry(k, ld(3, enc(1 << 3 | 0) + enc(5))))),
        ("non-packed floats wire5", example(entry(k, ld(2, enc(1 << 3 | 5) + b"\x00\x00\x80\x3f" + enc(1 << 3 | 5) + b"\x00\x00\x00\x40")))),
        ("packed float len 6", example(entry(k, ld(2, ld(1, b"\x00\x00\x80\x3f\x01\x02"))))),
        ("packed float len 3", example(entry(k, ld(2, ld(1, b"\x01\x02\x03"))))),
        ("mixed float chunks", example(entry(k, ld(2, ld(1, struct.pack("<2f", 1.5, -2.0)) + enc(1 << 3 | 5) + struct.pack("<f", 3.25) + ld(1, struct.pack("<f", 7.0)))))),
        ("two packed chunks int64", example(entry(k, ld(3, ld(1, enc(1) + enc(2)) + ld(1, enc(3)))))),
        ("dup keys last wins", example(entry(k, i64(1)), entry(k, i64(2)))),
        ("dup keys kind change", example(entry(b"a", i64(1)), entry(b"b", f32(2.0)), entry(b"a", byt(b"x")))),
        ("two kinds in feature", example(entry(k, ld(3, ld(1, enc(1))) + ld(1, ld(1, b"zz"))))),
        ("value before key", ld(1, ld(1, ld(2, i64(1)) + ld(1, k)))),
        ("entry fields swapped numbers", ld(1, ld(1, ld(2, b"key2") + ld(1, i64(9))))),
        ("entry three fields", ld(1, ld(1, ld(1, k) + ld(2, i64(4)) + ld(3, b"junk")))),
        ("entry fixed32 key", ld(1, ld(1, enc(1 << 3 | 5) + b"abcd" + ld(2, i64(5))))),
        ("entry fixed64 value", ld(1, ld(1, ld(1, k) + enc(2 << 3 | 1) + b"\x1a\x02\x0a\x00\x00\x00\x00\x00"))),
        ("unknown top field fixed64", enc(2 << 3 | 1) + b"\x01" * 8 + example(entry(k, i64(7)))),
        ("unknown top field varint", enc(2 << 3 | 0) + enc(5) + ld(1, b"")),
        ("unknown top field fixed32", enc(3 << 3 | 5) + b"\x01\x02\x03\x04" + example(entry(k, i64(7)))),
        ("unknown top field len", ld(7, b"hello") + example(entry(k, i64(7)))),
        ("truncated", example(entry(k, i64(7)))[:-1]),
        ("truncated fixed64", enc(2 << 3 | 1) + b"\x01" * 7),
        ("truncated fixed32", enc(2 << 3 | 5) + b"\x01" * 3),
        ("bad utf8 key", example(entry(b"\xff", i64()))),
        ("bad utf8 key surrogate", example(entry(b"\xed\xa0\x80", i64()))),
        ("bad utf8 key overlong", example(entry(b"\xc0\xaf", i64()))),
        ("bad utf8 key truncated", example(entry(b"ab\xe2\x82", i64()))),
        ("utf8 key multibyte", example(entry("κλειδί-🔑".encode(), i64(3)))),
        ("feature field 4", example(entry(k, ld(4, b"")))),
        ("feature field 0", example(entry(k, ld(0, b"")))),
        ("bytes_list empty value", example(entry(k, byt(b"", b"ab")))),
        ("bytes_list other fields", example(entry(k, ld(1, ld(2, b"zz") + ld(1, b"a") + enc(3 << 3 | 5) + b"1234")))),
        ("bytes_list wrong wire", example(entry(k, ld(1, enc(1 << 3 | 5) + b"abcd")))),
        ("float_list wrong wire", example(entry(k, ld(2, enc(1 << 3 | 1) + b"abcdefgh")))),
        ("int64_list wrong wire 5", example(entry(k, ld(3, enc(1 << 3 | 5) + b"abcd")))),
        ("int64_list wrong wire 1", example(entry(k, ld(3, enc(1 << 3 | 1) + b"abcdefgh")))),
        ("int64_list other field", example(entry(k, ld(3, ld(2, b"zz") + ld(1, enc(5)))))),
        ("varint 11 bytes", example(entry(k, ld(3, ld(1, b"\xff" * 10 + b"\x01"))))),
        ("varint 10 bytes", example(entry(k, ld(3, ld(1, b"\xff" * 9 + b"\x01"))))),
        ("tag varint 11 bytes", b"\x80" * 10 + b"\x01"),
        ("features field 2 unknown", ld(1, ld(2, b"x") + entry(k, i64(3)))),
        ("int64 packed overrun", example(entry(k, ld(3, ld(1, b"\x81"))))),
        ("int64 packed overrun tail", example(entry(k, ld(3, ld(1, enc(300) + b"\xff")))) + ld(9, b"\x05")),
        ("int64 packed overrun into next entry", example(entry(b"a", ld(3, ld(1, b"\x96"))), entry(b"b", i64(1)))),
        ("features twice", ld(1, entry(b"a", i64())) + ld(1, entry(b"b", i64()))),
        ("features twice first bad", ld(1, entry(b"a", ld(9, b""))) + ld(1, entry(b"b", i64()))),
        ("features wire 5", enc(1 << 3 | 5) + b"abcd"),
        ("feature map wire 5", ld(1, enc(1 << 3 | 5) + b"abcd")),
        ("wire type 3 group", ld(1, enc(1 << 3 | 3))),
        ("wire type 4", ld(1, enc(1 << 3 | 4))),
        ("wire type 6", enc(1 << 3 | 6)),
        ("wire type 7", enc(5 << 3 | 7)),
        ("outer error wins over inner", ld(1, entry(b"a", ld(9, b"")) + enc(2 << 3 | 3))),
        ("inner error order", ld(1, entry(b"a", ld(9, b"")) + entry(b"\xff", i64()))),
        ("tag overrun at end", example(entry(k, i64(1))) + b"\x8a"),
        ("nested tag overrun", ld(1, ld(1, ld(1, k) + ld(2, i64(1))) + b"\x80")),
        ("int64 values ref range", example(entry(k, i64(0, 1, 127, 128, 2**31 - 1, -1, -8, 300)))),
        ("int64 values out of range", example(entry(k, i64(2**31, 2**32, 2**35, 2**62, -9, -(2**31), -(2**63), 2**63 - 1)))),
        ("floats special", example(entry(k, ld(2, ld(1, b"".join(struct.pack("<I", x) for x in [0, 0x80000000, 0x7F800000, 0xFF800000, 0x7FC00000, 0x7FC12345, 0x00000001, 0x807FFFFF, 0x3F800000])))))),
        ("float snan", example(entry(k, ld(2, ld(1, struct.pack("<I", 0x7FA00000)))))),
        ("many keys", example(*[entry(f"key{j}".encode(), i64(j)) for j in range(100)])),
        ("large bytes", example(entry(b"img", byt(bytes(range(256)) * 40)), entry(b"label", i64(42)))),
        ("length varint 5 bytes", ld(1, b"") + enc(1 << 3 | 2) + b"\x80\x80\x80\x80\x00"),
        ("negative length", ld(1, entry(k, i64(1))) + enc(3 << 3 | 2) + b"\xff\xff\xff\xff\x0f"),
    ]
    return C


def random_example(rng: random.Random) -> bytes:
    ents = []
    for j in range(rng.randint(0, 6)):
        key = rng.choice([b"label", b"id", b"image", b"f", f"k{j}".encode(), b"x" * rng.randint(1, 20)])
        kind = rng.randint(1, 3)
        n = rng.choice([0, 1, 1, 2, 3, 8])
        if kind == 1:
            feat = byt(*[bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 12))) for _ in range(n)])
        elif kind == 2:
            feat = f32(*[rng.uniform(-10, 10) for _ in range(n)])
        else:
            feat = i64(*[rng.choice([rng.randint(0, 127), rng.randint(0, 2**31 - 1), rng.randint(-8, -1), rng.randint(-(2**63), 2**63 - 1)]) for _ in range(n)])
        ents.append(entry(key, feat))
    return example(*ents)


def mutate(rng: random.Random, raw: bytes) -> bytes:
    b = bytearray(raw)
    for _ in range(rng.randint(1, 3)):
        op = rng.randint(0, 4)
        if op == 0 and b:
            b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
        elif op == 1 and b:
            b[rng.randrange(len(b))] = rng.choice([0x00, 0x80, 0xFF, 0x7F, 0x08, 0x0A, 0x12, 0x1A, 0x0D, 0x15, 0x09])
        elif op == 2 and b:
            del b[rng.randrange(len(b))]
        elif op == 3:
            b.insert(rng.randrange(len(b) + 1), rng.getrandbits(8))
        elif op == 4 and b:
            b = b[: rng.randrange(len(b))]
    return bytes(b)


# ----------------------------------------------------------------------------------------------
# files
# ----------------------------------------------------------------------------------------------
def crc32c_bitwise(data: bytes) -> int:
    c = 0xFFFFFFFF
    for x in data:
        c ^= x
        for _ in range(8):
            c = (c >> 1) ^ (0x82F63B78 & -(c & 1))
    return c ^ 0xFFFFFFFF


def masked(data: bytes) -> int:
    c = crc32c_bitwise(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def frame(payloads: list[bytes], spec_crc: bool) -> bytes:
    out = bytearray()
    for p in payloads:
        lb = len(p).to_bytes(8, "little")
        out += lb
        out += struct.pack("<I", masked(lb)) if spec_crc else b"\x00\x00\x00\x00"
        out += p
        out += struct.pack("<I", masked(p)) if spec_crc else b"\x00\x00\x00\x00"
    return bytes(out)


def ref_file_payloads(pb2) -> dict[str, list[bytes]]:
    """The reference test recipes (tests/utils.py:9-105), serialized with upb exactly as there."""
    dummy = []
    for i in range(1, 11):
        ex = pb2.Example(features=pb2.Features(feature={
            "bytes_feature": pb2.Feature(bytes_list=pb2.BytesList(value=[f"A{i}".encode()])),
            "float_feature": pb2.Feature(float_list=pb2.FloatList(value=[1.1 * i, 2.2 * i, 3.3 * i])),
            "int64_feature": pb2.Feature(int64_list=pb2.Int64List(value=[10 * i, 20 * i, 30 * i])),
        }))
        dummy.append(ex.SerializeToString())
    demo = []
    names = ["cat", "dog"]
    for i in range(40):
        name = names[i % 2]
        ex = pb2.Example(features=pb2.Features(feature={
            "name": pb2.Feature(bytes_list=pb2.BytesList(value=[name.encode()])),
            "label": pb2.Feature(int64_list=pb2.Int64List(value=[1 if name == "cat" else 0])),
            "image_id": pb2.Feature(bytes_list=pb2.BytesList(value=[f"image-id-{i}".encode()])),
        }))
        demo.append(ex.SerializeToString())
    import numpy as np  # noqa: PLC0415

    rng = np.random.default_rng(7)
    img = rng.integers(0, 255, (10, 10, 3), dtype=np.uint8).tobytes()
    pixels = [pb2.Example(features=pb2.Features(feature={
        "image": pb2.Feature(bytes_list=pb2.BytesList(value=[img])),
    })).SerializeToString()]
    return {"dummy": dummy, "demo": demo, "pixels": pixels}


def c0_payloads(n: int) -> list[bytes]:
    """C0/C1 shape: label = i % 1000, id = f'img-{i:08d}'."""
    return [example(entry(b"label", i64(i % 1000)), entry(b"id", byt(f"img-{i:08d}".encode()))) for i in range(n)]


def c2_payloads(n: int, seed: int = 2) -> list[bytes]:
    """C2 shape (D4), image sizes scaled down 16x to keep the fixture small."""
    import numpy as np  # noqa: PLC0415

    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        size = int(np.clip(rng.lognormal(np.log(40960), 0.5), 4096, 524288)) // 16
        img = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
        out.append(example(entry(b"image", byt(img)), entry(b"label", i64(int(rng.integers(0, 102)))),
                           entry(b"file_name", byt(f"image_{i:05d}.jpg".encode()))))
    return out


def c3_payloads(n: int, seed: int = 3) -> list[bytes]:
    """C3 shape (D5): 32 int64_list i{j} + 32 float_list f{j}, lengths U[0,64]."""
    import numpy as np  # noqa: PLC0415

    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        ents = []
        for j in range(32):
            m = int(rng.integers(0, 65))
            bits = rng.integers(1, 32, m)
            vals = [int(rng.integers(0, 1 << int(b))) for b in bits]
            vals = [v if rng.random() >= 0.05 else int(rng.integers(-8, 0)) for v in vals]
            ents.append(entry(f"i{j}".encode(), i64(*vals)))
        for j in range(32):
            m = int(rng.integers(0, 65))
            ents.append(entry(f"f{j}".encode(), f32(*rng.standard_normal(m).astype(np.float32).tolist())))
        out.append(example(*ents))
    return out


def file_record(idx_mod, dec_results, path: Path, spec_crc_expected: bool | None):
    r = idx_mod.TFRecordFileReader(str(path), save_index=True)
    pointers = [[p["start"], p["end"], p["example_size"]] for p in r.get_pointers()]
    r.close()
    del r
    idx_bytes = Path(str(path) + ".idx").read_bytes()
    os.unlink(str(path) + ".idx")
    data = path.read_bytes()
    crc = []
    for s, e, _ in pointers:
        if e > len(data) or e - s < 16:
            crc.append(None)
            continue
        lb, lcrc = data[s:s + 8], struct.unpack("<I", data[s + 8:s + 12])[0]
        pl, dcrc = data[s + 12:e - 4], struct.unpack("<I", data[e - 4:e])[0]
        crc.append([int(masked(lb) == lcrc), int(masked(pl) == dcrc)])
    return {"pointers": pointers, "idx_hex": idx_bytes.hex(), "crc": crc}


def main() -> None:
    dec, idx, pb2 = load_reference()
    rng = random.Random(1234)
    FILES.mkdir(parents=True, exist_ok=True)

    # -------- payload cases
    cases: list[tuple[str, bytes]] = edge_cases()
    for name, pls in ref_file_payloads(pb2).items():
        cases += [(f"{name}[{i}]", p) for i, p in enumerate(pls)]
    cases += [(f"c0[{i}]", p) for i, p in enumerate(c0_payloads(200)[::13])]
    cases += [(f"c3[{i}]", p) for i, p in enumerate(c3_payloads(4))]
    seeds = [p for _, p in cases if 0 < len(p) < 3000]
    for i in range(200):
        cases.append((f"random[{i}]", random_example(rng)))
    for i in range(1500):
        base = rng.choice(seeds + [random_example(rng) for _ in range(2)])
        cases.append((f"fuzz[{i}]", mutate(rng, base)))

    payloads = [p for _, p in cases]
    ref = run_reference(payloads)
    upb = run_upb(pb2, payloads)
    assert len(ref) == len(payloads)
    with open(HERE / "cases.jsonl", "w") as f:
        for (name, p), r, u in zip(cases, ref, upb):
            f.write(json.dumps({"name": name, "payload": p.hex(), "ref": r, "upb": u}) + "\n")
    kinds = {}
    for r in ref:
        k = next(iter(r))
        kinds[k] = kinds.get(k, 0) + 1
    print("cases:", len(cases), kinds)

    # -------- files
    specs = {
        "dummy": (ref_file_payloads(pb2)["dummy"], False),
        "demo": (ref_file_payloads(pb2)["demo"], False),
        "c0_mini": (c0_payloads(1024), False),
        "c0_mini_crc": (c0_payloads(1024), True),
        "c2_mini_crc": (c2_payloads(12), True),
        "c3_mini_crc": (c3_payloads(24), True),
    }
    for name, (pls, spec_crc) in specs.items():
        path = FILES / f"{name}.tfrecord"
        data = frame(pls, spec_crc)
        if name == "c0_mini_crc":  # corrupt a few records: CRC negatives (decode must still succeed)
            b = bytearray(data)
            off = 0
            for i, p in enumerate(pls):
                if i % 97 == 5:
                    b[off + 12 + 3] ^= 0x01  # payload byte flip -> data CRC mismatch
                if i % 101 == 7:
                    b[off + 9] ^= 0x40      # length CRC byte flip
                off += len(p) + 16
            data = bytes(b)
        path.write_bytes(data)
        meta = file_record(idx, None, path, spec_crc)
        r = idx.TFRecordFileReader(str(path), save_index=False)
        raws = [r.get_example(i) for i in range(len(r))]
        r.close()
        meta["records"] = run_reference(raws)
        (FILES / f"{name}.json").write_text(json.dumps(meta))
        print("file", name, len(meta["pointers"]), "records", len(data), "bytes")

    # framing edge files (indexer.pyx:225-249): trailing < 8 bytes, zero-length record,
    # declared length past EOF, empty file
    good = frame(c0_payloads(3), True)
    edges = {
        "edge_trailing": good + b"\x01\x02\x03\x04\x05",
        "edge_zero_len": frame([b"", c0_payloads(1)[0], b""], True),
        "edge_overrun": good + (1000).to_bytes(8, "little") + b"\x00" * 4 + b"\x0a\x00",
        "edge_empty": b"",
        "edge_len_only": good + (5).to_bytes(8, "little"),
    }
    for name, data in edges.items():
        path = FILES / f"{name}.tfrecord"
        path.write_bytes(data)
        meta = file_record(idx, None, path, True)
        # get_example on every pointer: overrunning records raise IOError in the reference
        r = idx.TFRecordFileReader(str(path), save_index=False)
        got = []
        for i in range(len(r)):
            try:
                got.append({"raw": r.get_example(i).hex()})
            except BaseException as e:  # noqa: BLE001
                got.append({"exc": type(e).__name__, "msg": str(e)})
        r.close()
        meta["get_example"] = got
        (FILES / f"{name}.json").write_text(json.dumps(meta))
        print("edge", name, meta["pointers"])


if __name__ == "__main__":
    main()
