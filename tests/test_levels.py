"""K3 level decode (k_page_levels) against the oracle on hand-built hybrid
streams with run-level control: RLE runs from 1 value to far past one batch
(1-byte and multi-byte headers, redundant varint bytes), bit-packed runs from
one group to hundreds (payload crossing the LDS window), every level width
1..8, pages whose value count ends inside a run, streams that end early
(EOF), trailing bytes, and rep + def streams on the same page.  Semantics are
hybridDecoder.next (hybrid_decoder.go:82-166); the oracle is pinned by the
reference's bit-unpack KATs and Dremel vectors (tests/test_oracle.py)."""
import numpy as np
import pytest

import parity as P
import pqtest_util as U
from pqgpu import abi


def uvarint(v, pad=0):
    o = bytearray()
    while v >= 0x80:
        o.append(v & 0x7F | 0x80)
        v >>= 7
    if pad:  # redundant continuation bytes (binary.ReadUvarint accepts them)
        o.append(v | 0x80)
        o += b"\x80" * (pad - 1)
        o.append(0)
    else:
        o.append(v)
    return bytes(o)


def bitpack(vals, w):
    out = bytearray((len(vals) * w + 7) // 8)
    bit = 0
    for v in vals:
        for k in range(w):
            if (int(v) >> k) & 1:
                out[(bit + k) >> 3] |= 1 << ((bit + k) & 7)
        bit += w
    return bytes(out)


def stream(rng, n, maxl, short=False):
    """Random hybrid stream of at least n values (fewer if short) -> (bytes, values)."""
    w = max(1, int(maxl).bit_length())
    rb = (w + 7) // 8
    out, vals = bytearray(), []
    target = int(n * rng.uniform(0.3, 0.9)) if short else n + int(rng.integers(0, 40))
    while len(vals) < target:
        r = rng.random()
        if r < 0.45:
            cnt = int(rng.integers(1, 20)) if rng.random() < 0.8 else int(rng.integers(20, 6000))
            v = int(rng.integers(0, maxl + 1))
            out += uvarint(cnt << 1, pad=int(rng.integers(1, 4)) if rng.random() < 0.05 else 0)
            out += v.to_bytes(rb, "little")
            vals += [v] * cnt
        else:
            g = int(rng.integers(1, 8)) if rng.random() < 0.8 else int(rng.integers(8, 400))
            vs = rng.integers(0, maxl + 1, 8 * g)
            out += uvarint(g << 1 | 1) + bitpack(vs, w)
            vals += [int(x) for x in vs]
    if rng.random() < 0.2:
        out += bytes(rng.integers(0, 256, int(rng.integers(1, 30)), dtype=np.uint8))  # trailing bytes
    return bytes(out), vals


def chunk(rng, pages, maxd, maxr, short_frac=0.0):
    parts = []
    for _ in range(pages):
        n = int(rng.integers(1, 30000))
        defs, _ = stream(rng, n, maxd, short=rng.random() < short_frac)
        rep = stream(rng, n, maxr)[0] if maxr else None
        vals = rng.integers(-2**31, 2**31 - 1, n, dtype=np.int64).astype("<i4").tobytes()
        parts.append(U.v1_page(vals, n, 0, rep=rep, defs=defs))
    return b"".join(parts)


@pytest.fixture(scope="module")
def dec():
    import pqgpu
    d = pqgpu.GpuDecoder(0)
    yield d
    d.close()


def test_stream_generator_roundtrip():
    """The generator's streams decode to its values through the oracle's bit unpack."""
    from oracle import pyoracle as O  # noqa: F401  (oracle pinned in test_oracle.py)
    rng = np.random.default_rng(3)
    s, vals = stream(rng, 5000, 3)
    assert len(vals) >= 5000 and len(s) > 10


@pytest.mark.gpu
@pytest.mark.parametrize("maxd", [1, 2, 3, 5, 7, 15, 100, 255])
def test_def_levels_random_streams(dec, maxd):
    rng = np.random.default_rng(maxd)
    for _ in range(3):
        P.compare_chunk_bytes(chunk(rng, 12, maxd, 0), dec, ptype=abi.INT32, max_def=maxd)


@pytest.mark.gpu
@pytest.mark.parametrize("maxd,maxr", [(1, 1), (3, 2), (7, 7)])
def test_rep_and_def_streams(dec, maxd, maxr):
    rng = np.random.default_rng(100 + maxd)
    for _ in range(3):
        P.compare_chunk_bytes(chunk(rng, 10, maxd, maxr), dec, ptype=abi.INT32, max_def=maxd, max_rep=maxr)


@pytest.mark.gpu
def test_short_streams_fail_like_the_oracle(dec):
    rng = np.random.default_rng(77)
    for maxd in (1, 4, 200):
        for _ in range(4):
            P.compare_chunk_bytes(chunk(rng, 6, maxd, 0, short_frac=0.5), dec, ptype=abi.INT32, max_def=maxd)


@pytest.mark.gpu
def test_level_stream_mutations(dec):
    """Byte flips inside level streams: status and bytes agree with the oracle."""
    rng = np.random.default_rng(78)
    for maxd in (1, 3):
        base = chunk(rng, 4, maxd, 0)
        for _ in range(40):
            b = bytearray(base)
            for _ in range(int(rng.integers(1, 4))):
                b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
            P.compare_chunk_bytes(bytes(b), dec, ptype=abi.INT32, max_def=maxd)


def short_chain_page(rng, nruns, how):
    """A 1-bit level stream of `nruns` runs (the writer's shape: bit-packed
    runs of up to 63 groups, RLE runs), for the whole-page decoder's serial
    chain walk (<= 64 runs) and the exit table past it."""
    out, vals = bytearray(), []
    for _ in range(nruns):
        if rng.random() < 0.7:
            g = int(rng.integers(1, 64))
            vs = (rng.random(8 * g) < 0.9).astype(np.int64)
            out += uvarint(g << 1 | 1) + bitpack(vs, 1)
            vals += [int(x) for x in vs]
        else:
            cnt = int(rng.integers(1, 700))
            v = int(rng.integers(0, 2))
            out += uvarint(cnt << 1) + bytes([v])
            vals += [v] * cnt
    n = len(vals)
    if how == "inside":  # the count ends inside the last run
        n = max(1, n - int(rng.integers(1, 8)))
    elif how == "short":  # the stream ends before the count (EOF)
        n = n + int(rng.integers(1, 50))
    elif how == "bad_after":  # a bad RLE value after the count: never read
        out += uvarint(8 << 1) + bytes([2])
    elif how == "bad_before":  # a bad RLE value before the count
        out = out[:0] + uvarint(8 << 1) + bytes([2]) + out
        n = n + 8
    elif how == "trailing":
        out += bytes(rng.integers(0, 256, 17, dtype=np.uint8))
    vals_b = rng.integers(-2**31, 2**31 - 1, n, dtype=np.int64).astype("<i4").tobytes()
    return U.v1_page(vals_b, n, 0, defs=bytes(out))


@pytest.mark.gpu
@pytest.mark.parametrize("nruns", [1, 2, 40, 63, 64, 65, 90])
@pytest.mark.parametrize("how", ["exact", "inside", "short", "bad_after", "bad_before", "trailing"])
def test_one_bit_short_chains(dec, nruns, how):
    rng = np.random.default_rng(1000 * nruns + len(how))
    pages = b"".join(short_chain_page(rng, nruns, how) for _ in range(6))
    P.compare_chunk_bytes(pages, dec, ptype=abi.INT32, max_def=1)
