"""Multi-rank path: row-group shards decoded
independently per rank reproduce the single-process decode, with no collective
other than the barrier and the timing reduction.

All ranks open ONE C5 file (8 x world row groups) by path: each reads the
footer only, takes its row groups (pqgpu.shard.row_groups_for_rank) and reads
just their byte span (pqgpu.chunk_span / span_jobs, the skipChunk seek of
chunk_reader.go:286-312 for everything else).  On CPU (gloo, world size 2)
each rank decodes its shard with the oracle; the GPU variant (-m gpu) runs both
ranks on cuda:0 through pqgpu.FileReader (span upload + pqg_decode_chunks).
bench.gen_workload's per-rank C5 generation is checked to produce the same
chunk bytes as the one file's row groups."""
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


def _decode_shard(rank, world, gpu, path):
    """This rank's row groups of the one file at `path`: {(global rg, col): digest}."""
    import pqgpu
    pf = pqgpu.ParquetFile.open(path)
    rgs = list(shard.row_groups_for_rank(pf.num_row_groups, rank, world))
    specs = [(rg, c) for rg in rgs for c in range(pf.num_columns)]
    lo, hi, _ = pqgpu.chunk_span(pf, specs)
    assert hi - lo < pf.size  # the other ranks' row groups are never read
    out = {}
    if gpu:
        fr = pqgpu.FileReader(path, decoder=pqgpu.GpuDecoder(0))
        try:
            res = fr.decode_row_groups(rgs)
            assert fr.uploaded_bytes == hi - lo
            for i, (rg, col, r) in enumerate(res):
                d = fr.dec.download(r, i)
                out[(rg, col)] = _digest(d.status, d.num_slots, d.num_values,
                                         (d.def_levels, d.rep_levels, d.values, d.offsets))
        finally:
            fr.dec.close()
    else:
        for (rg, col) in specs:
            out[(rg, col)] = _oracle_digest(pf.host_job(rg, col)[0])
    return out


def _worker(rank, world, port, q, gpu, path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "parquet-go_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = _decode_shard(rank, world, gpu, path)
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)  # test-side merge only; bench.py has no data-path collective
        t = shard.max_elapsed(0.5 + rank, dist)
        if rank == 0:
            q.put((gathered, t))
    finally:
        dist.destroy_process_group()


def _one_file(tmp_path, world):
    from gen import pqwrite as W
    data, _ = W.config_c5(row_groups=range(8 * world), rows_per_rg=ROWS_PER_RG)
    path = str(tmp_path / "c5_one_file.parquet")
    with open(path, "wb") as f:
        f.write(data)
    return path


def _run_two_ranks(gpu, path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, gpu, path)) for r in range(2)]
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


def test_two_rank_gloo_shards_match_single_process(tmp_path):
    gathered, t = _run_two_ranks(False, _one_file(tmp_path, 2))
    assert t == 1.5  # MAX over ranks
    _check_merge(gathered, 2)


def test_bench_rank_workload_is_the_one_files_row_groups():
    """bench.py generates each rank's C5 row groups on the rank (the 64-row-group
    file is ~52 GB): their chunk bytes equal those row groups' bytes in the one file."""
    import bench
    import pqgpu
    from gen import pqwrite as W
    one, _ = W.config_c5(row_groups=range(16), rows_per_rg=ROWS_PER_RG)
    pone = pqgpu.ParquetFile(one)
    wl = bench.gen_workload("c5", _args(), 1, 2)
    pf, specs, (_, info) = wl.files[0]
    assert info["row_groups"] == list(range(8, 16))
    for (i, c) in specs:
        a, b = pf.chunk_meta(i, c), pone.chunk_meta(8 + i, c)
        assert (a.total_compressed_size, a.num_values) == (b.total_compressed_size, b.num_values)
        assert bytes(pf.read_range(a.start, a.start + a.total_compressed_size)) == \
            bytes(pone.read_range(b.start, b.start + b.total_compressed_size))


@pytest.mark.gpu
def test_two_rank_gpu_shards_match_single_process(tmp_path):
    """Both ranks on cuda:0, each range-reading its shard of the one file
    through pqgpu.FileReader."""
    gathered, t = _run_two_ranks(True, _one_file(tmp_path, 2))
    assert t == 1.5
    _check_merge(gathered, 2)


@pytest.mark.gpu
def test_bench_launches_ranks():
    """`bench.py --gpus 2` with no launcher starts 2 ranks itself
    (torch.distributed.run; here both on cuda:0 over gloo) and reports n_gpus 2."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--only", "c5",
                          "--c5-rows-per-rg", "20000", "--steps", "2", "--warmup", "1", "--no-cpu"],
                         capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["verified_bit_exact"]


def test_bench_gpus8_launch_touches_no_gpu(monkeypatch):
    """`bench.py --gpus 8` (no launcher env) hands over to 8 ranks before any
    GPU work: up to launch_ranks no decoder context is created, the HIP
    library is not asked for, and torch.cuda is not initialised."""
    import sys
    import bench
    import pqgpu
    from pqgpu import _lib
    calls = []
    monkeypatch.setattr(pqgpu, "GpuDecoder", lambda *a, **k: calls.append("GpuDecoder"))
    monkeypatch.setattr(_lib, "lib", lambda: calls.append("lib"))
    seen = {}

    def fake_launch(n):
        torch = sys.modules.get("torch")
        seen.update(n=n, calls=list(calls), cuda_init=bool(torch is not None and torch.cuda.is_initialized()))
        return 0

    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setattr(bench, "launch_ranks", fake_launch)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8"])
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code == 0
    assert seen == {"n": 8, "calls": [], "cuda_init": False}


def test_rank_plans_for_eight_gpus():
    """The row groups each of 8 ranks decodes (bench.py: C2 one row group per
    width, C5 8 of the 64): disjoint, complete, equal work per rank."""
    c5 = [list(shard.row_groups_for_rank(64, r, 8)) for r in range(8)]
    assert sorted(sum(c5, [])) == list(range(64)) and all(len(x) == 8 for x in c5)
    c2 = [list(shard.row_groups_for_rank(8, r, 8)) for r in range(8)]
    assert c2 == [[r] for r in range(8)]
