"""Multi-rank path on CPU (gloo, world_size 2): row-group shards decoded
independently per rank reproduce the single-process decode, with no
collective other than the timing reduction.
The per-rank decoder here is the oracle (no GPU in this container); on the
GPU box bench.py runs the same sharding with libpqgpu per rank."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from pqgpu import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _file():
    from gen import pqwrite as W
    rng = np.random.default_rng(7)
    rows = 6 * 3000
    defs = (rng.random(rows) >= 0.1).astype(np.uint8)
    vals = rng.integers(0, 1 << 10, size=int(defs.sum())).astype(np.int32)
    c1 = W.Column("a", W.INT32, vals, repetition=W.OPTIONAL, encoding=W.RLE_DICTIONARY, def_levels=defs,
                  rows_per_page=1000)
    c2 = W.Column("b", W.INT64, rng.integers(-2**40, 2**40, size=rows), rows_per_page=700)
    return W.write_file([c1, c2], rows, row_groups=6)


def _digest(chunk):
    parts = [np.array([chunk.status, chunk.num_slots, chunk.num_values], dtype=np.int64).tobytes()]
    for a in (chunk.def_levels, chunk.rep_levels, chunk.values):
        if a is not None:
            parts.append(np.ascontiguousarray(a).tobytes())
    import hashlib
    return hashlib.sha256(b"".join(parts)).hexdigest()


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import pqgpu
        from oracle import pyoracle as O
        pf = pqgpu.ParquetFile(_file())
        mine = {}
        for rg, c, job in shard.shard_jobs(pf, rank, world, make_job=lambda p, r, c: p.host_job(r, c)[0]):
            mine[(rg, c)] = _digest(O.decode_chunk(job))
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
        t = shard.max_elapsed(0.5 + rank, dist)
        if rank == 0:
            q.put((gathered, t))
    finally:
        dist.destroy_process_group()


def test_partition_covers_all_row_groups():
    for R in (1, 5, 64):
        for G in (1, 2, 8):
            seen = [rg for r in range(G) for rg in shard.row_groups_for_rank(R, r, G)]
            assert seen == list(range(R))
            sizes = [len(shard.row_groups_for_rank(R, r, G)) for r in range(G)]
            assert max(sizes) - min(sizes) <= 1
    assert [shard.rank_of_row_group(i, 64, 8) for i in range(0, 64, 8)] == list(range(8))
    with pytest.raises(ValueError):
        shard.row_groups_for_rank(4, 2, 2)


def test_two_rank_gloo_shards_match_single_process():
    import pqgpu
    from oracle import pyoracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    gathered, t = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert t == 1.5  # MAX over ranks
    merged = {}
    for r, part in enumerate(gathered):
        for (rg, c), d in part.items():
            assert shard.rank_of_row_group(rg, 6, 2) == r
            merged[(rg, c)] = d
    pf = pqgpu.ParquetFile(_file())
    assert sorted(merged) == [(rg, c) for rg in range(pf.num_row_groups) for c in range(pf.num_columns)]
    for rg in range(pf.num_row_groups):
        for c in range(pf.num_columns):
            assert merged[(rg, c)] == _digest(O.decode_chunk(pf.host_job(rg, c)[0]))
