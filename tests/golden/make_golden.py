#!/usr/bin/env python3
"""Regenerate tests/golden/*.json from the REFERENCE CRC32C.

Run in the build container (needs /root/reference; oracle/Makefile compiles
kv/src/util/crc32c.cc from its own sources into oracle/_ref/):

    make -C oracle && python tests/golden/make_golden.py

What is written (data only -- inputs and expected outputs):
  kats.json   known-answer tests restated from the reference's own tests:
              RFC 3720 B.4 (rocksdb/util/crc32c_test.cc:66-100,
              leveldb/util/crc32c_test.cc:13-49), the 27 folly 3-way vectors on
              the FNV-filled 4 MiB buffer (rocksdb/util/crc32c_test.cc:21-64,
              fill rule :145-176; stored as the buffer RULE plus expected values),
              leveldb's "TestCRCBuffer" (leveldb/util/crc32c.cc:269-271), the
              Extend and Mask tests (:123-138), and the SURVEY 8c anchors.
              Every expected value is recomputed here by the compiled reference
              and must equal the literal the reference test asserts.
  spans.json  seeded random spans over a splitmix64 buffer (rule in the file):
              lengths around every boundary the kernels have (0..80, 16-byte
              and 4 KiB edges, the 64 KiB segment edge), offsets 0..31 and
              SST-like unaligned packing, zero and non-zero init_crc; expected
              crc and Mask(crc) from the reference.
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from tests.golden.common import splitmix64_bytes  # noqa: E402

REF = os.path.join(REPO, "oracle", "_ref", "libref_crc32c.so")
ORACLE = os.path.join(REPO, "oracle", "_build", "liboracle.so")

FOLLY_BUFFER_SIZE = 512 * 1024 * 8
FOLLY = [  # (offset, length, ~crc) rocksdb/util/crc32c_test.cc:30-63
    (0, 0, 0xFFFFFFFF), (8, 1, 1543413366), (8, 2, 523493126), (8, 3, 1560427360),
    (8, 4, 3422504776), (8, 5, 447841138), (8, 6, 3910050499), (8, 7, 3346241981),
    (9, 1, 3855826643), (10, 2, 560880875), (11, 3, 1479707779), (12, 4, 2237687071),
    (13, 5, 4063855784), (14, 6, 2553454047), (15, 7, 1349220140), (8, 8, 627613930),
    (8, 9, 2105929409), (8, 10, 2447068514), (8, 11, 863807079), (8, 12, 292050879),
    (8, 13, 1411837737), (8, 14, 2614515001), (8, 15, 3579076296), (8, 16, 2897079161),
    (8, 17, 675168386), (0, FOLLY_BUFFER_SIZE, 2096790750), (1, FOLLY_BUFFER_SIZE // 2, 3854797577),
]
ISCSI_PDU = [0x01, 0xc0, 0x00, 0x00] + [0] * 12 + [0x14, 0, 0, 0, 0, 0, 0x04, 0, 0, 0, 0, 0x14,
                                                     0, 0, 0, 0x18, 0x28] + [0] * 7 + [0x02] + [0] * 7


def _ref():
    lib = ctypes.CDLL(REF)
    lib.ref_crc32c_extend.restype = ctypes.c_uint32
    lib.ref_crc32c_extend.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
    lib.ref_mask.restype = ctypes.c_uint32
    lib.ref_mask.argtypes = [ctypes.c_uint32]
    return lib


def _oracle():
    lib = ctypes.CDLL(ORACLE)
    lib.oracle_fill_folly_buffer.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    return lib


def ref_extend(lib, init, arr: np.ndarray, off=0, n=None) -> int:
    n = arr.size - off if n is None else n
    return int(lib.ref_crc32c_extend(init, arr.ctypes.data + off, n))


def make_kats(ref, orc) -> dict:
    def b(x):
        return np.frombuffer(bytes(x), dtype=np.uint8).copy()

    rfc = [
        ("zeros32", [0] * 32, 0x8a9136aa),
        ("ones32", [0xff] * 32, 0x62a8ab43),
        ("ascending32", list(range(32)), 0x46dd794e),
        ("descending32", [31 - i for i in range(32)], 0x113fdb5c),
        ("iscsi_read_pdu48", ISCSI_PDU, 0xd9963a56),
        ("leveldb_TestCRCBuffer", list(b"TestCRCBuffer"), 0xdcbc59fa),
    ]
    out = {"rfc": []}
    for name, data, lit in rfc:
        got = ref_extend(ref, 0, b(data))
        assert got == lit, (name, hex(got), hex(lit))
        out["rfc"].append({"name": name, "data_hex": bytes(data).hex(), "crc": lit})

    buf = np.zeros(FOLLY_BUFFER_SIZE, dtype=np.uint8)
    orc.oracle_fill_folly_buffer(buf.ctypes.data, buf.size)
    folly = []
    for off, n, notcrc in FOLLY:
        want = (~notcrc) & 0xFFFFFFFF
        got = ref_extend(ref, 0, buf, off, n)
        assert got == want, (off, n, hex(got), hex(want))
        half = n // 2
        stitched = int(ref.ref_crc32c_extend(ref_extend(ref, 0, buf, off, half),
                                             buf.ctypes.data + off + half, n - half))
        assert stitched == want
        folly.append({"offset": off, "length": n, "crc": want})
    out["folly"] = {"buffer_size": FOLLY_BUFFER_SIZE,
                    "rule": "rocksdb/util/crc32c_test.cc:145-176 (oracle_fill_folly_buffer)",
                    "vectors": folly}

    hello = ref_extend(ref, 0, b(b"hello "))
    out["extend"] = {"hello_": hello, "hello_world": ref_extend(ref, 0, b(b"hello world")),
                     "extend_hello_world": int(ref.ref_crc32c_extend(hello, b"world", 5))}
    assert out["extend"]["hello_world"] == out["extend"]["extend_hello_world"]
    foo = ref_extend(ref, 0, b(b"foo"))
    out["mask"] = {"foo_crc": foo, "foo_mask": int(ref.ref_mask(foo)),
                   "foo_mask_mask": int(ref.ref_mask(ref.ref_mask(foo)))}

    # SURVEY 8c anchors: 4 KiB blocks and the type-byte Extend of WriteRawBlock
    pat = (np.arange(65536) & 0xFF).astype(np.uint8)
    anchors = {
        "zeros4096": ref_extend(ref, 0, np.zeros(4096, np.uint8)),
        "ones4096": ref_extend(ref, 0, np.full(4096, 0xFF, np.uint8)),
    }
    for n in (512, 1024, 2048, 4096, 8192, 16384, 32768, 65536):
        anchors[f"iota{n}"] = ref_extend(ref, 0, pat, 0, n)
    blk = np.concatenate([pat[:4096], np.zeros(1, np.uint8)])
    anchors["iota4096_type0"] = ref_extend(ref, 0, blk)
    anchors["iota4096_type0_mask"] = int(ref.ref_mask(anchors["iota4096_type0"]))
    assert anchors["zeros4096"] == 0x98f94189 and anchors["ones4096"] == 0x25c1fe13
    assert anchors["iota4096"] == 0x9c71fe32 and anchors["iota4096_type0"] == 0x83391be9
    assert anchors["iota4096_type0_mask"] == 0xda55f14a
    out["anchors"] = anchors
    return out


def make_spans(ref) -> dict:
    seed, size = 0x5EED_C0DE, 1 << 20
    buf = splitmix64_bytes(seed, size)
    rng = np.random.default_rng(20260415)
    lens = list(range(0, 81))
    for edge in (128, 255, 256, 257, 511, 512, 513, 1008, 1023, 1024, 1025, 2047, 2048, 2049,
                 4080, 4095, 4096, 4097, 4100, 4111, 4112, 4113, 4224, 4225, 8191, 8192, 8193,
                 16383, 16384, 16385, 32767, 32768, 32769, 65519, 65535, 65536, 65537,
                 65551, 65552, 65553, 131071, 131072, 131073, 200000):
        lens.append(edge)
    lens += [int(x) for x in rng.integers(81, 70000, size=300)]
    spans = []
    for n in lens:
        for off in (0, 1, 3, 4, 7, 8, 13, 15, 16, 17, 31):
            if off + n > size:
                continue
            if n > 4096 and off not in (0, 1, 15, 16):
                continue
            init = 0 if (n + off) % 3 else int(rng.integers(0, 2**32))
            spans.append((off, n, init))
    # SST-like packing: blocks of ~4 KiB + 1 type byte at prev + n + 5
    cur = 3
    while len(spans) < 2600:
        n = int(rng.integers(4097, 4226))
        if cur + n > size:
            break
        spans.append((cur, n, 0))
        cur += n + 4
    rows = []
    for off, n, init in spans:
        crc = ref_extend(ref, init, buf, off, n)
        rows.append([off, n, init, crc, int(ref.ref_mask(crc))])
    return {"buffer": {"rule": "splitmix64", "seed": seed, "size": size},
            "columns": ["offset", "length", "init_crc", "crc", "masked"],
            "rows": rows}


def main() -> None:
    ref, orc = _ref(), _oracle()
    with open(os.path.join(HERE, "kats.json"), "w") as f:
        json.dump(make_kats(ref, orc), f, indent=1)
    with open(os.path.join(HERE, "spans.json"), "w") as f:
        json.dump(make_spans(ref), f, separators=(",", ":"))
    print("wrote kats.json, spans.json")


if __name__ == "__main__":
    main()
