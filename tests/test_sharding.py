"""Multi-rank path: row-group shards decoded
independently per rank reproduce the single-process decode, with no collective
other than the barrier and the timing reduction.

The ranks build their work exactly as bench.py does (bench.gen_workload:
pqgpu.shard.row_groups_for_rank over the C5 row groups, each generated from
its global index).  On CPU (gloo, world size 2) each rank decodes its shard
with the oracle; the GPU variant (-m gpu) runs both ranks on cuda:0 and
decodes through pqg_decode_chunks, as bench.py does per GPU."""
import argparse
import hashlib
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from pqgpu import shard

ROWS_PER_RG = 3000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _args():
    return argparse.Namespace(c5_rows_per_rg=ROWS_PER_RG, rows=0, bits="")


def _digest(status, slots, nvals, arrays):
    parts = [np.array([status, slots, nvals], dtype=np.int64).tobytes()]
    parts += [np.ascontiguousarray(a).tobytes() for a in arrays if a is not None]
    return hashlib.sha256(b"".join(parts)).hexdigest()


def _oracle_digest(job):
    from oracle import pyoracle as O
    r = O.decode_chunk(job)
    return _digest(r.status, r.num_slots, r.num_values, (r.def_levels, r.rep_levels, r.values, r.offsets))


def _decode_shard(rank, world, gpu):
    """This rank's C5 shard, built and decoded the way bench.py builds it:
    {(global rg, col): digest}."""
    import bench
    import pqgpu
    wl = bench.gen_workload("c5", _args(), rank, world)
    pf, specs, (_, info) = wl.files[0]
    rgs = info["row_groups"]
    assert rgs == list(shard.row_groups_for_rank(8 * world, rank, world))
    out = {}
    if gpu:
        dec = pqgpu.GpuDecoder(0)
        dev = dec.upload(pf.data)
        try:
            res = dec.decode_jobs([pqgpu.device_job(pf, rg, col, dev) for (rg, col) in specs])
            for i, ((rg, col), r) in enumerate(zip(specs, res)):
                d = dec.download(r, i)
                out[(rgs[rg], col)] = _digest(d.status, d.num_slots, d.num_values,
                                              (d.def_levels, d.rep_levels, d.values, d.offsets))
        finally:
            dec.free(dev)
            dec.close()
    else:
        for (rg, col) in specs:
            out[(rgs[rg], col)] = _oracle_digest(pf.host_job(rg, col)[0])
    return out


def _worker(rank, world, port, q, gpu):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "parquet-go_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = _decode_shard(rank, world, gpu)
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)  # test-side merge only; bench.py has no data-path collective
        t = shard.max_elapsed(0.5 + rank, dist)
        if rank == 0:
            q.put((gathered, t))
    finally:
        dist.destroy_process_group()


def _run_two_ranks(gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, gpu)) for r in range(2)]
    for p in procs:
        p.start()
    gathered, t = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return gathered, t


def _check_merge(gathered, world):
    """Each rank holds exactly its row groups; the union equals the
    single-process decode of the whole 8*world-row-group file."""
    import pqgpu
    from gen import pqwrite as W
    R = 8 * world
    merged = {}
    for r, part in enumerate(gathered):
        for (rg, c), d in part.items():
            assert shard.rank_of_row_group(rg, R, world) == r
            merged[(rg, c)] = d
    data, _ = W.config_c5(row_groups=range(R), rows_per_rg=ROWS_PER_RG)
    pf = pqgpu.ParquetFile(data)
    assert sorted(merged) == [(rg, c) for rg in range(R) for c in range(pf.num_columns)]
    for rg in range(R):
        for c in range(pf.num_columns):
            assert merged[(rg, c)] == _oracle_digest(pf.host_job(rg, c)[0]), (rg, c)


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
    gathered, t = _run_two_ranks(gpu=False)
    assert t == 1.5  # MAX over ranks
    _check_merge(gathered, 2)


@pytest.mark.gpu
def test_two_rank_gpu_shards_match_single_process():
    """Both ranks on cuda:0, each decoding its shard with libpqgpu."""
    gathered, t = _run_two_ranks(gpu=True)
    assert t == 1.5
    _check_merge(gathered, 2)
