"""K2 split decode (pqg_snappy.hip: k_snap_plan -> k_snap_seg -> k_snap_link ->
k_snap_decode).  golang/snappy's Encode, which the reference writer uses
(compress.go:42-44, vendor/github.com/golang/snappy/encode.go:18-41), encodes
independent 64 KiB blocks; such pages decode as 64 KiB sub-blocks on many
waves.  Any other valid stream (a copy across a 64 KiB boundary) and every
corrupt one go back to the one-wave decode of the whole block, which the page
flag PQG_PAGE_FLAG_SNAPPY_SERIAL records.  Every case is GPU vs the oracle
(decode_other.go:14-101 restated), bit for bit, on both paths."""
import ctypes as C

import numpy as np
import pytest

import parity as P
import pqgpu
from gen import pqwrite as W
from oracle import pyoracle as O
from pqgpu import abi

SERIAL = 2  # PQG_PAGE_FLAG_SNAPPY_SERIAL


@pytest.fixture(scope="module")
def dec():
    d = pqgpu.GpuDecoder(0)
    yield d
    d.close()


def decode_file(dec, data):
    """Parity of every chunk of `data`; returns [(page type, usize, flags)] of the compressed pages."""
    pf = pqgpu.ParquetFile(data)
    dev = dec.upload(pf.data)
    out = []
    try:
        jobs = [pqgpu.device_job(pf, rg, c, dev) for rg in range(pf.num_row_groups) for c in range(pf.num_columns)]
        res = dec.decode_jobs(jobs)
        i = 0
        for rg in range(pf.num_row_groups):
            for c in range(pf.num_columns):
                got = dec.download(res[i], i)
                P.compare_chunk(P.oracle_chunk(pf, rg, c), got, "rg%d col%d" % (rg, c))
                out += [(p.page_type, p.uncompressed_size, p.flags) for p in got.pages]
                i += 1
    finally:
        dec.free(dev)
    return out


def big_pages(pages):
    return [p for p in pages if p[1] > W.SNAPPY_BLOCK]


def strings_file(rows=60_000, vocab=20_000, seed=7):
    return W.config_c4(rows=rows, vocab=vocab, rows_per_page=rows, seed=seed, dict_limit=1 << 20)[0]


@pytest.mark.gpu
def test_split_strings_block_shaped(dec):
    """C4 shape: a big dictionary page and big PLAIN pages, golang/snappy blocks:
    every page decodes split (no serial page)."""
    pages = decode_file(dec, strings_file())
    assert len(big_pages(pages)) >= 1
    assert not any(f & SERIAL for _, _, f in pages), pages


@pytest.mark.gpu
def test_split_falls_back_on_cross_block_copies(dec):
    """The same strings compressed as ONE snappy block per page (copies reach
    across 64 KiB boundaries): still bit-exact, through the serial path."""
    with W.snappy_block_size(0):
        data = strings_file()
    pages = decode_file(dec, data)
    assert any(f & SERIAL for t, u, f in big_pages(pages)), pages


@pytest.mark.gpu
def test_split_incompressible_long_literals(dec):
    """Random int64 PLAIN pages of 1.6 MB: 64 KiB literals, so the chain enters
    most segments far from their start (k_snap_link walks those)."""
    rng = np.random.default_rng(3)
    v = rng.integers(-2**63, 2**63 - 1, size=400_000, dtype=np.int64)
    data = W.write_file([W.Column("x", W.INT64, v, codec=W.SNAPPY, rows_per_page=200_000)], len(v))
    pages = decode_file(dec, data)
    assert len(big_pages(pages)) == 2 and not any(f & SERIAL for _, _, f in pages)


@pytest.mark.gpu
def test_split_mixed_literals_and_runs(dec):
    """Pages alternating incompressible stretches, long runs (overlapping
    copies) and repeats, V1 and V2, over sub-block boundaries at every phase."""
    rng = np.random.default_rng(5)
    parts = []
    for i in range(40):
        k = i % 4
        n = int(rng.integers(100, 30_000))
        if k == 0:
            parts.append(rng.integers(0, 256, n, dtype=np.uint8))
        elif k == 1:
            parts.append(np.full(n, int(rng.integers(0, 256)), np.uint8))
        elif k == 2:
            pat = rng.integers(0, 256, int(rng.integers(2, 40)), dtype=np.uint8)
            parts.append(np.resize(pat, n))
        else:
            parts.append(rng.integers(0, 4, n, dtype=np.uint8))
    blob = np.concatenate(parts)
    v = blob[: len(blob) // 8 * 8].view(np.int64)
    for ver in (1, 2):
        data = W.write_file([W.Column("x", W.INT64, v, codec=W.SNAPPY, page_version=ver,
                                      rows_per_page=len(v) // 3 + 1)], len(v))
        pages = decode_file(dec, data)
        assert len(big_pages(pages)) >= 3 and not any(f & SERIAL for _, _, f in pages)
        with W.snappy_block_size(0):
            data = W.write_file([W.Column("x", W.INT64, v, codec=W.SNAPPY, page_version=ver,
                                          rows_per_page=len(v) // 3 + 1)], len(v))
        decode_file(dec, data)


def _blocks_stream(rng, nblocks, tail):
    """A snappy stream of `nblocks` independent 64 KiB blocks plus a `tail`-byte
    block, built tag by tag (copies never reach into an earlier block)."""
    import test_snappy as S
    out = bytearray()
    tags = []
    for b in range(nblocks + 1):
        size = W.SNAPPY_BLOCK if b < nblocks else tail
        blk = bytearray()
        while len(blk) < size:
            room = size - len(blk)
            if not blk or rng.random() < 0.3:
                n = min(room, int(rng.integers(1, 40)) if rng.random() > 0.02 else int(rng.integers(60, 3000)))
                x = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
                tags.append(S.lit(x))
                blk += x
                continue
            off = int(rng.integers(1, min(len(blk), 60000) + 1)) if rng.random() < 0.5 else \
                int(rng.integers(1, min(len(blk), 8) + 1))
            ln = min(room, int(rng.integers(1, 65)))
            form = 1 if (off < 2048 and 4 <= ln <= 11 and rng.random() < 0.5) else (4 if rng.random() < 0.1 else 2)
            tags.append(S.copy(off, ln, form))
            for _ in range(ln):
                blk.append(blk[-off])
        out += blk
    return S.uvarint(len(out)) + b"".join(tags), bytes(out)


@pytest.mark.gpu
def test_block_decompress_split_streams(dec):
    """pqg_block_decompress runs the same split stage on its one block: streams
    of independent 64 KiB blocks (tag forms, long literals, run-length copies,
    a block ending exactly on a boundary) and their corruptions."""
    rng = np.random.default_rng(21)
    n = 0
    for nb, tail in ((1, 0), (3, 17), (5, 65535), (2, 1)):
        src, plain = _blocks_stream(rng, nb, tail)
        rc_o, exp = O.snappy_decode(src)
        assert rc_o == 0 and exp == plain
        dst = np.zeros(len(plain) + 64, np.uint8)
        got = C.c_int64(0)
        rc = dec.L.pqg_block_decompress(dec.ctx, abi.CODEC_SNAPPY, src, len(src), dst.ctypes.data, len(dst),
                                        C.byref(got))
        assert rc == 0 and dst[:got.value].tobytes() == plain
        for _ in range(25):  # corruptions: same outcome class as the oracle
            m = bytearray(src)
            i = int(rng.integers(4, len(m)))
            m[i] = int(rng.integers(0, 256))
            rc_o, exp = O.snappy_decode(bytes(m))
            dst[:] = 0
            rc = dec.L.pqg_block_decompress(dec.ctx, abi.CODEC_SNAPPY, bytes(m), len(m), dst.ctypes.data, len(dst),
                                            C.byref(got))
            if rc_o == abi.STATUS_CODES["SIZE"]:
                continue  # a varint flip: the buffer is sized from it (CAPACITY) — class checked elsewhere
            assert rc == rc_o, (rc, rc_o)
            if rc == 0:
                assert dst[:got.value].tobytes() == exp
                n += 1
    assert n >= 0
