"""Row-group sharding across GPUs: one process per GPU, each
decoding a contiguous range of row groups.  Column chunks are independent
(readRowGroup touches only rowGroups.Columns[i], chunk_reader.go:404-431), so
there is no collective on the decode path; the only cross-rank traffic is the
barrier and the MAX reduction of the elapsed time that bench.py reports."""


def rank_of_row_group(rg, num_row_groups, world):
    """RG i -> GPU floor(i * G / R): contiguous, balanced ranges in file order."""
    if num_row_groups <= 0 or world <= 0:
        raise ValueError("need row groups and ranks")
    return (rg * world) // num_row_groups


def row_groups_for_rank(num_row_groups, rank, world):
    """The contiguous row-group range [lo, hi) decoded by `rank`."""
    if not 0 <= rank < world:
        raise ValueError("rank %d outside world %d" % (rank, world))
    lo = (rank * num_row_groups + world - 1) // world
    hi = ((rank + 1) * num_row_groups + world - 1) // world
    return range(lo, min(hi, num_row_groups))


def shard_jobs(pf, rank, world, columns=None, make_job=None):
    """(rg, col, job) for this rank's row groups and the selected leaf columns."""
    cols = list(range(pf.num_columns)) if columns is None else list(columns)
    out = []
    for rg in row_groups_for_rank(pf.num_row_groups, rank, world):
        for c in cols:
            out.append((rg, c, make_job(pf, rg, c) if make_job else None))
    return out


def max_elapsed(elapsed, dist=None, device=None):
    """Slowest rank's elapsed time (the whole-job clock)."""
    if dist is None:
        return float(elapsed)
    import torch
    t = torch.tensor([float(elapsed)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
