#!/usr/bin/env python3
"""Extract the reference's own known-answer vectors into data fixtures.

Run HERE (the build container), where the reference is mounted read-only at
/root/reference.  It reads the reference's *_test.go files as text, pulls out
the literal test vectors (inputs and expected outputs only) and writes them as
JSON under tests/golden/.  No reference source text is copied: only the byte
strings / integer arrays the tests assert on.

Fixtures written:
  bitpack32.json   unpack8int32Tests  bitpacking32_test.go:25-654  (width, bytes, [8]int32)
  bitpack64.json   unpack8int64Tests  bitpacking64_test.go:25-1744 (width, bytes, [8]int64)
  crash_files.json fuzz-crash regression files (whole parquet files as bytes):
                   chunk_reader_test.go:5-21, deltabp_decoder_test.go:5-149,152-296,
                   type_dict_test.go:30-173, type_bytearray_test.go:5-26,
                   page_v1_test.go:5-512, schema_test.go:140-216,219-363
                   expected outcome: an error or a clean end, never a crash.
  dremel.json      TestTwitterBlog data_store_test.go:346-389 level vectors.
"""
import json
import os
import re
import sys

REF = os.environ.get("PQ_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


def parse_int_list(s):
    return [int(x, 0) for x in re.split(r"\s*,\s*", s.strip().rstrip(",")) if x]


def extract_bitpack(fname, var, nbits):
    text = open(os.path.join(REF, fname)).read()
    start = text.index("var %s" % var)
    body = text[start:]
    pat = re.compile(
        r"\{\s*(\d+)\s*,\s*\[\]byte\{([^}]*)\}\s*,\s*\[8\]int%d\{([^}]*)\}\s*,?\s*\}" % nbits, re.S)
    out = []
    for m in pat.finditer(body):
        w = int(m.group(1))
        data = parse_int_list(m.group(2)) if m.group(2).strip() else []
        vals = parse_int_list(m.group(3))
        assert len(vals) == 8 and len(data) == w, (w, data, vals)
        out.append({"width": w, "data": bytes(data).hex(), "values": vals})
    return out


_ESC = {"a": 7, "b": 8, "f": 12, "n": 10, "r": 13, "t": 9, "v": 11, "\\": 92, '"': 34, "'": 39}


def go_string_bytes(lit):
    """Decode one Go interpreted string literal body (without quotes) to bytes."""
    out = bytearray()
    i = 0
    while i < len(lit):
        c = lit[i]
        if c != "\\":
            out += c.encode("utf-8")
            i += 1
            continue
        n = lit[i + 1]
        if n == "x":
            out.append(int(lit[i + 2:i + 4], 16))
            i += 4
        elif n in "01234567":
            out.append(int(lit[i + 1:i + 4], 8))
            i += 4
        elif n == "u":
            out += chr(int(lit[i + 2:i + 6], 16)).encode("utf-8")
            i += 6
        elif n == "U":
            out += chr(int(lit[i + 2:i + 10], 16)).encode("utf-8")
            i += 10
        else:
            out.append(_ESC[n])
            i += 2
    return bytes(out)


def extract_crash(fname, test):
    text = open(os.path.join(REF, fname)).read()
    start = text.index("func %s(" % test)
    seg = text[start:]
    seg = seg[seg.index("[]byte(") + len("[]byte("):]
    end = seg.index("readAllData")
    seg = seg[:end]
    lits = re.findall(r'"((?:[^"\\]|\\.)*)"', seg, re.S)
    return b"".join(go_string_bytes(l) for l in lits)


CRASH = [
    ("chunk_reader_test.go", "TestFuzzCrashReadRowGroup"),
    ("deltabp_decoder_test.go", "TestFuzzCrashDeltaBitPackDecoder64DivByZero"),
    ("deltabp_decoder_test.go", "TestFuzzCrashDeltaBitPackDecoder64LenOutOfRange"),
    ("type_dict_test.go", "TestFuzzCrashDictDecoderDecodeValues"),
    ("type_bytearray_test.go", "TestFuzzCrashByteArrayPlainDecoderNext"),
    ("page_v1_test.go", "TestDataPageReaderV1InitCrash"),
    ("schema_test.go", "TestFuzzCrashReadGroupSchema2"),
    ("schema_test.go", "TestFuzzCrashReadGroupSchema"),
]


def main():
    if not os.path.isdir(REF):
        print("reference not mounted at %s; fixtures are already committed" % REF)
        return 0
    b32 = extract_bitpack("bitpacking32_test.go", "unpack8int32Tests", 32)
    b64 = extract_bitpack("bitpacking64_test.go", "unpack8int64Tests", 64)
    json.dump({"source": "bitpacking32_test.go:25-654 unpack8int32Tests", "vectors": b32},
              open(os.path.join(OUT, "bitpack32.json"), "w"), indent=0)
    json.dump({"source": "bitpacking64_test.go:25-1744 unpack8int64Tests", "vectors": b64},
              open(os.path.join(OUT, "bitpack64.json"), "w"), indent=0)
    crash = []
    for f, t in CRASH:
        data = extract_crash(f, t)
        assert data.startswith(b"PAR1"), (f, t, data[:8])
        crash.append({"source": "%s %s" % (f, t), "expect": "error-or-clean-end", "data": data.hex()})
    json.dump({"files": crash}, open(os.path.join(OUT, "crash_files.json"), "w"), indent=0)
    dremel = {
        "source": "data_store_test.go:346-389 TestTwitterBlog",
        "max_def": 2, "max_rep": 2,
        "rep_levels": [0, 2, 2, 1, 2, 2, 2, 0, 1, 2],
        "def_levels": [2] * 10,
        "values": list(range(1, 11)),
        "rows": [[[1, 2, 3], [4, 5, 6, 7]], [[8], [9, 10]]],
    }
    json.dump(dremel, open(os.path.join(OUT, "dremel.json"), "w"), indent=1)
    print("bitpack32: %d vectors, bitpack64: %d vectors, crash files: %d" % (len(b32), len(b64), len(crash)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
