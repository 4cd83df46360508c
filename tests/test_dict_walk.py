"""Dictionary index streams of 4-byte dictionary pages (run tables from
k_hybrid_walk + k_dict4 / k_dict4_big), with either level decoder, against
the oracle: hand-built dictionary chunks whose RLE_DICTIONARY pages
carry index streams with run-level control at every bit width 1..32 -- RLE
runs of 1 value to far past one batch, bit-packed runs of one group to
hundreds (payload crossing the ring window), redundant varint header bytes
(the serial header path), pages that end inside a run, streams that end early
(EOF), out-of-range keys (dict: invalid index), RLE values wider than the bit
width, empty runs, and random byte mutations.  Semantics: hybridDecoder.next
(hybrid_decoder.go:82-166) under dictDecoder.decodeValues (type_dict.go:39-59);
the oracle is pinned by the reference's bit-unpack KATs (tests/test_oracle.py)."""
import numpy as np
import pytest

import parity as P
import pqtest_util as U
from pqgpu import abi
from test_levels import bitpack, uvarint


def index_stream(rng, nkeys, w, dcount, bad_frac=0.0, short=False, odd=0.0):
    """Random hybrid stream of >= nkeys keys of width w (fewer if `short`);
    keys < dcount except a `bad_frac` of runs; `odd`: probability of an empty
    run or an RLE value wider than w at a run boundary."""
    rb = (w + 7) // 8
    top = (1 << w) - 1
    out, n = bytearray(), 0
    target = int(nkeys * rng.uniform(0.2, 0.95)) if short else nkeys + int(rng.integers(0, 40))

    def key():
        if rng.random() < bad_frac:
            return int(rng.integers(dcount, top + 1)) if dcount <= top else int(rng.integers(0, top + 1))
        return int(rng.integers(0, min(dcount, top + 1)))

    while n < target:
        if odd and rng.random() < odd:
            if w % 8 and rng.random() < 0.5:  # a value of w + 1 bits still fits the rb value bytes
                out += uvarint(int(rng.integers(1, 9)) << 1) + (top + 1 + int(rng.integers(0, 3))).to_bytes(rb, "little")
            else:
                out += uvarint(int(rng.integers(0, 2)))  # empty RLE / empty bit-packed run
            continue
        r = rng.random()
        if r < 0.5:
            cnt = int(rng.integers(1, 24)) if rng.random() < 0.85 else int(rng.integers(24, 5000))
            out += uvarint(cnt << 1, pad=int(rng.integers(1, 6)) if rng.random() < 0.03 else 0)
            out += key().to_bytes(rb, "little")
            n += cnt
        else:
            g = int(rng.integers(1, 6)) if rng.random() < 0.8 else int(rng.integers(6, 300))
            ks = [key() for _ in range(8 * g)]
            out += uvarint(g << 1 | 1, pad=int(rng.integers(1, 6)) if rng.random() < 0.03 else 0) + bitpack(ks, w)
            n += 8 * g
    if short and rng.random() < 0.5 and len(out) > 4:
        out = out[:-int(rng.integers(1, 4))]  # cut inside the last run
    if rng.random() < 0.2:
        out += bytes(rng.integers(0, 256, int(rng.integers(1, 30)), dtype=np.uint8))  # trailing bytes
    return bytes(out)


def dict_chunk(rng, pages, w, dcount, nullable=True, bad_frac=0.0, short_frac=0.0, odd=0.0, max_page=30000):
    ents = rng.integers(-2**31, 2**31 - 1, dcount, dtype=np.int64).astype("<i4").tobytes()
    parts = [U.page_header_dict(len(ents), len(ents), dcount) + ents]
    for _ in range(pages):
        n = int(rng.integers(1, max_page))
        defs = None
        nn = n
        if nullable:
            d = (rng.random(n) >= rng.uniform(0.0, 0.4)).astype(np.int64)
            nn = int(d.sum())
            defs = uvarint(((n + 7) // 8) << 1 | 1) + bitpack(d, 1)
        idx = bytes([w]) + index_stream(rng, nn, w, dcount, bad_frac, rng.random() < short_frac, odd)
        parts.append(U.v1_page(idx, n, 8, defs=defs))
    return b"".join(parts)


# the decode paths (pqg_runtime.hip, read when the context is created): the
# default one (run tables from the lane walker + k_dict4, 1-bit levels by the
# whole-page decoder, pqg_lev1.h) and the same with the batch level decoder
# alone (PQG_LEV1=0: the fallback of pages the whole-page decoder does not take)
PATHS = {"default": {}, "batch_levels": {"PQG_LEV1": "0"}}


@pytest.fixture(scope="module", params=list(PATHS))
def dec(request):
    import os
    import pqgpu
    env = PATHS[request.param]
    old = {k: os.environ.get(k) for k in ("PQG_LEV1",)}
    os.environ.update(env)
    try:
        d = pqgpu.GpuDecoder(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    yield d
    d.close()


def test_index_stream_generator():
    """CPU: the generator's streams parse as hybrid streams of the asked width."""
    rng = np.random.default_rng(5)
    s = index_stream(rng, 3000, 13, 5000)
    assert len(s) > 10
    c = dict_chunk(rng, 3, 7, 100)
    assert c[:1] == b"\x15"


@pytest.mark.gpu
@pytest.mark.parametrize("w", [1, 2, 3, 5, 8, 9, 12, 13, 16, 17, 20, 24, 25, 31, 32])
def test_dict_walk_widths(dec, w):
    rng = np.random.default_rng(900 + w)
    for dcount in (1 << min(w, 12), min(1 << w, 70000) if w < 32 else 70000):
        chunk = dict_chunk(rng, 8, w, dcount)
        P.compare_chunk_bytes(chunk, dec, ptype=abi.INT32, max_def=1)


@pytest.mark.gpu
@pytest.mark.parametrize("w", [1, 4, 11, 20, 32])
def test_dict_walk_required_pages(dec, w):
    rng = np.random.default_rng(950 + w)
    chunk = dict_chunk(rng, 10, w, 1 << min(w, 10), nullable=False)
    P.compare_chunk_bytes(chunk, dec, ptype=abi.INT32)


@pytest.mark.gpu
@pytest.mark.parametrize("w", [2, 9, 16, 32])
def test_dict_walk_bad_keys(dec, w):
    """Out-of-range keys (w = 32: keys with bit 31 set are negative int32 in Go)."""
    rng = np.random.default_rng(960 + w)
    for _ in range(6):
        dcount = int(rng.integers(1, 1 << min(w, 11)))
        chunk = dict_chunk(rng, 3, w, dcount, bad_frac=0.002)
        P.compare_chunk_bytes(chunk, dec, ptype=abi.INT32, max_def=1)


@pytest.mark.gpu
@pytest.mark.parametrize("w", [1, 3, 8, 15, 24, 32])
def test_dict_walk_short_and_odd_streams(dec, w):
    """Streams that end early, empty runs, RLE values wider than w."""
    rng = np.random.default_rng(970 + w)
    for k in range(6):
        chunk = dict_chunk(rng, 3, w, 1 << min(w, 12), short_frac=0.6, odd=(0.0, 0.0005, 0.01)[k % 3])
        P.compare_chunk_bytes(chunk, dec, ptype=abi.INT32, max_def=1)


@pytest.mark.gpu
def test_dict_walk_mutations(dec):
    """Byte flips inside index streams and level streams of dictionary pages."""
    rng = np.random.default_rng(980)
    for w in (3, 12, 20):
        base = dict_chunk(rng, 4, w, 1 << min(w, 10), max_page=6000)
        for _ in range(30):
            b = bytearray(base)
            for _ in range(int(rng.integers(1, 4))):
                b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
            P.compare_chunk_bytes(bytes(b), dec, ptype=abi.INT32, max_def=1)


@pytest.mark.gpu
def test_dict_walk_float_and_flba4(dec):
    """The other 4-byte dictionary columns: FLOAT and FIXED_LEN_BYTE_ARRAY(4)."""
    rng = np.random.default_rng(990)
    chunk = dict_chunk(rng, 5, 10, 1000)
    P.compare_chunk_bytes(chunk, dec, ptype=abi.FLOAT, max_def=1)
    P.compare_chunk_bytes(chunk, dec, ptype=abi.FIXED_LEN_BYTE_ARRAY, type_length=4, max_def=1)
