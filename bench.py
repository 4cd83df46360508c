#!/usr/bin/env python3
"""Decode throughput of the MI355X Parquet column-chunk decoder (libpqgpu).

Headline (BASELINE.json configs[1], "C2"): optional INT32 column, 100M rows per
file, ~10% nulls, RLE_DICTIONARY with D = 2^b entries for every index width b in
{1, 2, 4, 8, 12, 16, 20} (one file per width), data page V1, UNCOMPRESSED,
20 000 rows per page.  A step decodes all seven column chunks (700M slots) in
one batched call, inputs resident in HBM.

Sub-results (same line, "configs"): C1 (required int64 PLAIN, 10M rows) and
its one-page variant (the reference writer's layout), C2 run-heavy (index runs
of geometric length, mean 16), C3 (int64 DELTA_BINARY_PACKED, V2, SNAPPY, 200M
rows), C4 (STRING dictionary + PLAIN fallback, SNAPPY, 50M rows) and one C5
shard (8 row groups x 15.625M rows of LIST<double> + 8 mixed columns).  Each carries its own roofline (dominant
stage + whole pipeline) and CPU baseline.

Multi-GPU (one process per GPU, weak scaling): the data set has 8N C5 row
groups and N C2 row groups per width; rank r decodes the row groups
pqgpu.shard assigns it (RG i -> rank floor(i N / R)).  No collective touches
the data path: only the timing barrier and the MAX of the elapsed time.

Metric: decoded GB/s of uncompressed output (SURVEY §8d B_out: values, 1 B per
level per slot, string chars + 4 B offsets), whole job = sum over ranks / max
time over ranks.  Outputs are verified bit-exact against the generator's
arrays after timing.  The CPU baseline is the oracle (the C++ restatement of
parquet-go's decode) timed on a bounded sample: one thread (parquet-go's
one-goroutine FileReader) and a pool of host threads over independent chunks.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "parquet-go_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

METRIC = "decoded GB/s (uncompressed output) per GPU & node at 1/2/4/8; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
STAGES = ["scan", "list", "snappy", "levels", "walk", "unused", "nn_scan", "values", "strings", "finalize"]
PROFILE_TAG = "r06"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cores():
    """Host threads for the all-cores CPU baseline: the process's CPU affinity,
    capped by the harness's per-GPU CPU share when one is declared (the GPU box
    sets OMP_NUM_THREADS=16 per GPU while sched_getaffinity shows every CPU of
    the machine).  Returns (threads, note)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS", "")
    if share.isdigit() and 0 < int(share) < aff:
        return int(share), "sched_getaffinity %d CPUs; capped at the box's per-GPU share OMP_NUM_THREADS=%s" % (
            aff, share)
    return max(1, aff), "sched_getaffinity %d CPUs" % aff


def peak_rss_gb():
    import resource
    return round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6, 2)  # ru_maxrss: KiB on Linux


# ---------------------------------------------------------------- workloads
class Workload:
    """A set of files and the chunk jobs of one step, plus a verifier."""

    def __init__(self, key, desc, files, dtype):
        self.key, self.desc, self.dtype = key, desc, dtype
        self.files = files  # list of (ParquetFile, [(rg, col)], expected)
        self.devs = []


def gen_workload(key, args, rank, world):
    import pqgpu
    from gen import pqwrite as W
    from pqgpu import shard
    t0 = time.time()
    files = []
    if key in ("c2", "c2_run_heavy"):
        rh = key == "c2_run_heavy"
        rgs = list(shard.row_groups_for_rank(world, rank, world))  # N row groups per width
        bits_list = [int(b) for b in args.bits.split(",")]
        for rg in rgs:
            for bits, data, exp in W.config_c2_family(rows=args.rows, bits_list=bits_list, seed=2 + rg,
                                                      run_heavy=rh):
                files.append((pqgpu.ParquetFile(data), [(0, 0)], ("c2", exp)))
        desc = ("C2%s: optional INT32, %d rows x %d dictionary widths (b=%s), ~10%% nulls, RLE_DICTIONARY (%s), V1, "
                "UNCOMPRESSED, 20000 rows/page" % (" run-heavy" if rh else "", args.rows, len(bits_list), args.bits,
                                                  "index runs of geometric length, mean 16" if rh
                                                  else "uniform indices"))
        dtype = "int32"
    elif key in ("c1", "c1_1page"):
        one = key == "c1_1page"
        data, info = W.config_c1(rows=args.c1_rows, rows_per_page=args.c1_rows if one else 20000)
        files.append((pqgpu.ParquetFile(data), [(0, 0)], ("flat", [info["values"]])))
        desc = ("C1: required INT64, %d rows, PLAIN, UNCOMPRESSED, 1 RG, V1, %s" % (
            args.c1_rows, "ONE data page (parquet-go's writer layout, chunk_writer.go:237-246)" if one
            else "20000 rows/page"))
        dtype = "int64"
    elif key == "c3":
        data, info = W.config_c3(rows=args.c3_rows)
        files.append((pqgpu.ParquetFile(data), [(0, 0)], ("flat", [info["values"]])))
        desc = ("C3: INT64 timestamps, %d rows, DELTA_BINARY_PACKED (128/4x32), V2, SNAPPY, 20000 rows/page"
                % args.c3_rows)
        dtype = "int64"
    elif key == "c3_gzip":
        data, info = W.config_c3(rows=args.c3gz_rows, codec=W.GZIP)
        files.append((pqgpu.ParquetFile(data), [(0, 0)], ("flat", [info["values"]])))
        desc = ("C3-GZIP: the C3 column (INT64 timestamps, DELTA_BINARY_PACKED, V2, 20000 rows/page), %d rows, "
                "GZIP pages (one zlib-default member per page, as Go's gzip.NewWriter)" % args.c3gz_rows)
        dtype = "int64"
    elif key == "c4":
        data, info = W.config_c4(rows=args.c4_rows)
        files.append((pqgpu.ParquetFile(data), [(0, 0)], ("str", info)))
        desc = ("C4: required STRING, %d rows, 65536-word vocabulary (len U[4,32], Zipf 1.1), dictionary pages "
                "then PLAIN fallback after 1 MiB, SNAPPY, V1, 20000 rows/page" % args.c4_rows)
        dtype = "u8"
    elif key == "c5":
        R = 8 * world  # 8 row groups per GPU (64 at 8 GPUs, the C5 file)
        rgs = list(shard.row_groups_for_rank(R, rank, world))
        data, info = W.config_c5(row_groups=rgs, rows_per_rg=args.c5_rows_per_rg, as_array=True)
        pf = pqgpu.ParquetFile(data)
        files.append((pf, [(i, c) for i in range(len(rgs)) for c in range(pf.num_columns)], ("c5", info)))
        desc = ("C5 shard: row groups %s of %d (RG i -> GPU floor(i*%d/%d)), %d rows each: LIST<double> + int32, "
                "int64 DBP, double, float, int96, optional int32 (PLAIN), string dict, int64 SNAPPY; the columns with "
                "nulls or a dictionary (LIST, optional int32, string) one data page per chunk with one bit-packed "
                "run per level/index stream (parquet-go's writer layout: quirk-free), the others 20000 rows/page"
                % (rgs, R, world, R, args.c5_rows_per_rg))
        dtype = "mixed"
    else:
        raise ValueError(key)
    log("rank %d: %s generated in %.1fs (%.1f MB)" % (rank, key, time.time() - t0,
                                                      sum(len(f[0].data) for f in files) / 1e6))
    return Workload(key, desc, files, dtype)


# ---------------------------------------------------------------- byte accounting
def _level_sections(pf, meta, pg, desc):
    """(level bytes, value-section bytes) of a data page, from its header and,
    for V1 pages, the u32 length prefixes of the level sections."""
    if pg.page_type == 3:
        lv = pg.def_len + pg.rep_len
        return lv, pg.uncompressed_size - lv
    if desc.max_def == 0 and desc.max_rep == 0:
        return 0, pg.uncompressed_size
    at = meta.start + pg.payload_offset
    body = pf.data[at:at + pg.compressed_size]
    if meta.codec == 2:
        import gzip
        body = gzip.decompress(body)
    elif meta.codec != 0:
        import pyarrow as pa
        body = pa.decompress(body, decompressed_size=pg.uncompressed_size, codec="snappy").to_pybytes()
    pos = 0
    for present in (desc.max_rep > 0, desc.max_def > 0):
        if present:
            pos += 4 + int.from_bytes(body[pos:pos + 4], "little")
    return pos, pg.uncompressed_size - pos


def account(wl, pages_of, res):
    """B_in/B_out of the step and algorithmic bytes per stage.
    pages_of(ji): the page records of job ji (from the context that decoded it)."""
    b_in = b_out = 0
    st = dict.fromkeys(STAGES, 0)
    ji = 0
    for pf, specs, _ in wl.files:
        for (rg, col) in specs:
            r = res[ji]
            meta = pf.chunk_meta(rg, col)
            desc = pf.columns[col].desc
            b_in += meta.total_compressed_size
            nlev = (desc.max_def > 0) + (desc.max_rep > 0)
            slots_out = r.num_slots * nlev
            if r.value_width:
                vout = r.num_values * r.value_width
                b_out += vout + slots_out
            else:
                vout = r.values_bytes + (r.num_values + 1) * 8  # chars + int64 offsets written
                b_out += r.values_bytes + (r.num_values + 1) * 4 + slots_out
            st["scan"] += meta.total_compressed_size
            lev_in = val_in = dict_in = 0
            for pg in pages_of(ji):
                if pg.page_type == 2:
                    dict_in += pg.uncompressed_size
                    continue
                lv, vb = _level_sections(pf, meta, pg, desc)
                lev_in += lv
                val_in += vb
                if pg.encoding == 8:
                    st["walk"] += vb
                if meta.codec != 0:
                    lv2 = lv if pg.page_type == 3 else 0
                    st["snappy"] += pg.compressed_size - lv2 + pg.uncompressed_size - lv2
            st["levels"] += lev_in + slots_out
            st["values" if r.value_width else "strings"] += val_in + dict_in + vout
            ji += 1
    return b_in, b_out, st


# ---------------------------------------------------------------- verification
def verify(wl, dec, res):
    """Every decoded chunk against the generator's arrays.  C5: the expected
    arrays of one row group at a time (regenerated, then dropped), so a rank
    holds its file plus one row group's arrays."""
    ok = True
    ji = 0
    for pf, specs, (kind, exp) in wl.files:
        cur_rg, cur = None, None
        for (rg, col) in specs:
            r = res[ji]
            ji += 1
            if r.status != 0:
                return False
            if kind == "c5" and rg != cur_rg:
                cur_rg, cur = rg, None
                cur = exp["part"](rg)
            if kind == "c2":
                defs, vals = exp
                ok &= np.array_equal(dec.d2h(r.def_levels, r.num_slots), defs)
                ok &= np.array_equal(dec.d2h(r.values, r.values_bytes).view(vals.dtype), vals)
            elif kind == "flat":
                v = exp[0]
                ok &= np.array_equal(dec.d2h(r.values, r.values_bytes).view(v.dtype), v)
            elif kind == "str":
                ok &= np.array_equal(dec.d2h(r.offsets, (r.num_values + 1) * 8, np.int64), exp["offsets"])
                ok &= np.array_equal(dec.d2h(r.values, r.values_bytes), exp["chars"])
            elif kind == "c5":
                e = cur[pf.columns[col].path.decode().split(".")[0]]
                if "offsets" in e:
                    ok &= np.array_equal(dec.d2h(r.offsets, (r.num_values + 1) * 8, np.int64), e["offsets"])
                ok &= np.array_equal(dec.d2h(r.values, r.values_bytes), np.ascontiguousarray(e["values"]).view(np.uint8))
                if e.get("def_levels") is not None:
                    ok &= np.array_equal(dec.d2h(r.def_levels, r.num_slots), e["def_levels"])
                if e.get("rep_levels") is not None:
                    ok &= np.array_equal(dec.d2h(r.rep_levels, r.num_slots), e["rep_levels"])
    return bool(ok)


# ---------------------------------------------------------------- CPU baseline
def cpu_baseline(wl, seconds):
    """The oracle (C++ restatement of parquet-go's readPages/readPageData) on a
    bounded sample of the workload's chunks.  Both legs run the SAME tasks —
    each sampled chunk cut into page ranges (pqo_decode_page_range: the
    dictionary page, then the range's pages decoded and their outputs
    materialised) — once on one thread (parquet-go's one goroutine per
    FileReader, file_reader.go:27-118) and once over a pool of the host's
    threads (pages decode independently once the dictionary is read; ctypes
    releases the GIL), so the ratio is a true speed-up."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import pyoracle as O
    OL = O.lib()
    jobs = []
    for pf, specs, _ in wl.files:
        for (rg, col) in specs:
            jobs.append(pf.host_job(rg, col)[0])
    cores, note = host_cores()

    def run_range(task):
        job, lo, hi = task
        b = C.c_int64(0)
        rc = OL.pqo_decode_page_range(C.byref(job), lo, hi, C.byref(b))
        assert rc >= 0, rc
        return b.value

    def ranges(job):  # ~4 ranges per pool thread over the chunk's pages
        n = int(OL.pqo_decode_page_range(C.byref(job), 0, 0, None))
        per = max(1, -(-n // (4 * cores)))
        return [(job, lo, min(n, lo + per)) for lo in range(0, n, per)]

    done, t1, k, tasks = 0, 0.0, 0, []
    while k < len(jobs) and t1 < seconds / 2:
        tk = ranges(jobs[k])
        t = time.perf_counter()
        done += sum(run_range(x) for x in tk)
        t1 += time.perf_counter() - t
        tasks += tk
        k += 1
    single = done / t1 / 1e9
    t = time.perf_counter()
    with ThreadPoolExecutor(max_workers=cores) as ex:
        pool_bytes = sum(ex.map(run_range, tasks))
    tp = time.perf_counter() - t
    assert pool_bytes == done
    return ({"value": round(single, 4), "unit": "GB/s", "cores": 1, "kind": "port",
             "sample": "oracle (C++ restatement of parquet-go readPages/readPageData) on %d of %d chunks as %d page "
                       "ranges run in turn on one thread, like parquet-go's one-goroutine FileReader; %.1fs"
                       % (k, len(jobs), len(tasks), t1)},
            {"value": round(pool_bytes / tp / 1e9, 4), "unit": "GB/s", "cores": cores, "kind": "port",
             "speedup": round(t1 / tp, 2), "cores_note": note,
             "sample": "the same %d page ranges over a pool of %d host threads; %.1fs" % (len(tasks), cores, tp)})


# ---------------------------------------------------------------- PMC traffic (committed passes)
# every kernel each stage timer brackets (pqg_runtime.hip launch_pipeline; a
# name matches kernels it prefixes: k_page_levels covers k_page_levels_w1)
STAGE_KERNELS = {"scan": ["k_scan_pages", "k_tile_jobs", "k_page_cands", "k_cand_parse", "k_tile_scan", "k_cand_link",
                          "k_page_chain"],
                 "list": ["k_page_list"],
                 "snappy": ["k_snap_plan", "k_snap_seg", "k_snap_link", "k_snap_decode", "k_snappy", "k_inflate_s", "k_inflate"],
                 "levels": ["k_dict_resolve", "k_page_levels", "k_level_long"],
                 "walk": ["k_hybrid_walk", "k_walk_long"], "unused": [], "nn_scan": ["k_nn_scan"],
                 "values": ["k_values", "k_dict_plan", "k_dict4"],
                 "strings": ["k_str_dict", "k_str_plain", "k_str_count", "k_str_delta", "k_char_scan", "k_str_copy",
                             "k_str_dba"],
                 "finalize": ["k_finalize"]}


def pmc_traffic(key, kernels, workload):
    """HBM bytes per step of a stage's kernels from the committed PMC passes
    (profiles/<tag>_pmc_<config>.json, tools/pmc_traffic.py), if they were taken
    on this same workload; else None."""
    path = os.path.join(ROOT, "profiles", "%s_pmc_%s.json" % (PROFILE_TAG, key))
    if not os.path.exists(path):
        return None
    d = json.load(open(path))
    if d.get("workload") != workload:
        return None
    tot = sum(v["traffic"] for k, v in d["kernels"].items() if any(k.startswith("pqg::" + p) for p in kernels))
    return tot or None


# ---------------------------------------------------------------- run one workload
def split_jobs(jobs, k):
    """Jobs dealt to k decode contexts, largest first to the least loaded
    (by TotalCompressedSize): [(context, [job indices])]."""
    load = [0] * k
    parts = [[] for _ in range(k)]
    for i in sorted(range(len(jobs)), key=lambda i: -jobs[i].total_compressed_size):
        c = min(range(k), key=lambda c: load[c])
        parts[c].append(i)
        load[c] += jobs[i].total_compressed_size
    return [sorted(p) for p in parts if p]


def run_workload(wl, decs, args, steps, warmup, barrier, dist, world, rank, cpu_seconds):
    """One workload's line.  decs: the decode contexts (each with its own HIP
    stream); the chunks are dealt over them and decoded concurrently
    (pqg_decode_chunks_async on each, then pqg_sync on each), so one
    context's level stage overlaps another's values stage."""
    dec = decs[0]
    import pqgpu
    from pqgpu import abi
    L = dec.L
    jobs = []
    wl.uploaded = 0
    for pf, specs, _ in wl.files:
        # only the selected chunks' bytes go to HBM (skipChunk, chunk_reader.go:286-312)
        fj, dev, nbytes = pqgpu.span_jobs(pf, specs, dec)
        wl.devs.append(dev)
        wl.uploaded += nbytes
        jobs += fj
    n = len(jobs)
    parts = split_jobs(jobs, max(1, min(len(decs), n)))
    K = len(parts)
    arrs = [(abi.ChunkJob * len(p))(*[jobs[i] for i in p]) for p in parts]
    ress = [(abi.ChunkResult * len(p))() for p in parts]
    where = {i: (c, j) for c, p in enumerate(parts) for j, i in enumerate(p)}
    tmp = (C.c_float * 16)()

    def step():
        for c in range(K):
            rc = L.pqg_decode_chunks_async(decs[c].ctx, arrs[c], len(parts[c]))
            if rc != 0:
                raise RuntimeError("decode failed: %d" % rc)
        for c in range(K):
            rc = L.pqg_sync(decs[c].ctx, ress[c], len(parts[c]))
            if rc != 0:
                raise RuntimeError("decode failed: %d" % rc)

    def set_timing(on):
        for c in range(K):
            L.pqg_set_timing(decs[c].ctx, on)

    for _ in range(max(warmup, 1)):
        step()
    res = (abi.ChunkResult * n)()
    for i, (c, j) in where.items():
        res[i] = ress[c][j]
    bad = [abi.status_name(res[i].status) for i in range(n) if res[i].status != 0]
    assert not bad, "%s: %s" % (wl.key, bad)
    # the timed steps run without the per-stage HIP events (instrumentation,
    # a few us of stream time each).  The stage breakdown and the roofline come
    # from as many instrumented steps after them on ONE context (all chunks,
    # one stream): each kernel alone on the GPU, so its launch duration is its
    # own (with K streams the stages of different contexts share the GPU and
    # every launch stretches).  rocprofv3 summaries of `--streams 1` runs agree
    # with these durations.
    set_timing(0)
    barrier()
    t_start = time.perf_counter()
    for _ in range(steps):
        step()
    t_end = time.perf_counter()
    barrier()
    for i, (c, j) in where.items():
        res[i] = ress[c][j]
    verified = None
    if not args.no_verify:  # the timed path's outputs (the one-context pass below re-allocates context 0's arenas)
        verified = verify(wl, dec, res)
    arr1 = (abi.ChunkJob * n)(*jobs)
    res1 = (abi.ChunkResult * n)()
    L.pqg_set_timing(dec.ctx, 1)
    stage_acc = np.zeros(len(STAGES))
    for _ in range(steps):
        rc = L.pqg_decode_chunks(dec.ctx, arr1, n, res1)
        if rc != 0:
            raise RuntimeError("decode failed: %d" % rc)
        k = L.pqg_last_timings(dec.ctx, tmp, 16)
        stage_acc += np.array([tmp[i] for i in range(1, min(k, 1 + len(STAGES)))])
    elapsed = t_end - t_start
    if dist is not None:
        import torch
        on_gpu = dist.get_backend() == "nccl"
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if on_gpu else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    b_in, b_out, alg = account(wl, dec.pages, res1)
    stage_ms = stage_acc / steps
    dev_ms = float(stage_ms.sum())
    dom = int(np.argmax(stage_ms))
    dom_name = STAGES[dom]
    achieved = alg[dom_name] / (stage_ms[dom] * 1e-3) / 1e9 if stage_ms[dom] > 0 else 0.0
    # the decompression stage runs k_inflate_s (+ k_inflate) for GZIP chunks, the snappy kernels otherwise
    gz = wl.key == "c3_gzip"
    dom_label = ("inflate" if gz else "snappy") if dom_name == "snappy" else dom_name
    dom_kernels = [k for k in STAGE_KERNELS[dom_name] if dom_name != "snappy" or k.startswith("k_inflate") == gz]
    out = {
        "workload": wl.desc,
        "value": round(b_out * world / elapsed * steps / 1e9, 3),
        "unit": "GB/s",
        "ms_per_step": round(elapsed / steps * 1e3, 4),
        "steps": steps,
        "chunks_per_step": n,
        "bytes_in": b_in,
        "bytes_out": b_out,
        "h2d_bytes_per_rank": wl.uploaded,
        "roofline": {
            "bound": "hbm",
            "kernel": "stage " + dom_label + " (" + "+".join(dom_kernels) + ")",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": pmc_traffic(wl.key, dom_kernels, wl.desc),
            "alg_bytes_per_launch": alg[dom_name],
            "kernel_ms": round(float(stage_ms[dom]), 4),
            "measured_on": "one context (all chunks on one stream), instrumented steps after the timed ones",
            "pipeline_device_ms": round(dev_ms, 4),
            "pipeline_frac": round((b_in + b_out) / (dev_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if dev_ms else 0.0,
            "stage_ms": {s: round(float(x), 4) for s, x in zip(STAGES, stage_ms)},
            "stage_alg_bytes": alg,
        },
        "streams": K,
    }
    if verified is not None:
        out["verified_bit_exact"] = verified
        if not verified:
            log("VERIFY FAILED:", wl.key)
    out["host_peak_rss_gb"] = peak_rss_gb()  # this rank, so far (generation, upload, verification)
    if rank == 0 and not args.no_cpu:
        single, pool = cpu_baseline(wl, cpu_seconds)
        out["cpu_baseline"] = single
        out["cpu_baseline_all_cores"] = pool
    return out, res1  # context 0's one-stream results: valid until its next decode


def k8_c2(dec, wl, res, args):
    """K8 (pqg_assemble) on the first C2 chunk's device arrays: validity bitmap +
    spaced values.  Host-timed including the sync; not part of `value`."""
    from pqgpu import abi
    L = dec.L
    r = res[0]
    a, vb, sb, _ = dec.assemble(r.def_levels, r.rep_levels, r.values, r.num_slots, 1, 0, 4,
                                validity=True, spaced=True, offsets=False)
    reps = 5
    ms, host_ms = 0.0, 0.0
    dm = C.c_float()
    for _ in range(reps):
        t1 = time.perf_counter()
        rc = L.pqg_assemble(dec.ctx, C.byref(a))
        host_ms += (time.perf_counter() - t1) * 1e3
        assert rc == 0, abi.status_name(rc)
        L.pqg_last_assemble_ms(dec.ctx, C.byref(dm))
        ms += dm.value
    ms /= reps
    n = r.num_slots
    nbytes = n + r.num_values * 4 + n * 4 + (n + 7) // 8
    out = {"kernels": "k_asm_count+k_asm_scan+k_asm_write<4>", "slots": n, "ms": round(ms, 4), "alg_bytes": nbytes,
           "achieved_GBs": round(nbytes / (ms * 1e-3) / 1e9, 1),
           "frac": round(nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "timer": "HIP events on the decode stream around the K8 kernels (pqg_last_assemble_ms)",
           "host_ms_incl_sync": round(host_ms / reps, 4)}
    if not args.no_verify:
        defs, vals = wl.files[0][2][1]
        valid = defs == 1
        sp = dec.d2h(sb, n * 4).view(np.int32)
        bm = np.unpackbits(dec.d2h(vb, (n + 7) // 8), bitorder="little")[:n].astype(bool)
        out["verified"] = bool(np.array_equal(bm, valid) and np.array_equal(sp[valid], vals)
                               and not sp[~valid].any() and a.num_valid == int(valid.sum()))
    dec.free(vb)
    dec.free(sb)
    return out


def k8_list_c5(dec, wl, res, args):
    """K8 list export (pqg_assemble_list) of the C5 shard's LIST<double> chunks."""
    from pqgpu import abi
    L = dec.L
    pf, specs, (_, info) = wl.files[0]
    idx = [i for i, (rg, col) in enumerate(specs) if col == 0]
    tot_ms, tot_bytes, ok = 0.0, 0, True
    for i in idx:
        r = res[i]
        a, lvp, lop, evp, vvp = dec.assemble_list(r.def_levels, r.rep_levels, r.values, r.num_slots, 3, 1, 2, 8)
        rc = L.pqg_assemble_list(dec.ctx, C.byref(a))
        assert rc == 0, abi.status_name(rc)
        dm = C.c_float()
        L.pqg_last_assemble_ms(dec.ctx, C.byref(dm))
        tot_ms += dm.value
        n = r.num_slots
        tot_bytes += 2 * n + r.num_values * 8 + (a.num_rows + 1) * 4 + (a.num_rows + 7) // 8 + \
            (a.num_elements + 7) // 8 + a.num_elements * 8
        if not args.no_verify:
            rows = a.num_rows
            ok &= rows == info["rows_per_rg"] and a.num_valid == r.num_values
            lo = dec.d2h(lop, (rows + 1) * 4, np.int32)
            e = info["part"](specs[i][0])["lst"]
            starts = np.flatnonzero(e["rep_levels"] == 0)
            el = e["def_levels"] >= 2
            ok &= bool(np.array_equal(lo, np.r_[np.cumsum(el)[starts] - el[starts], el.sum()].astype(np.int32)))
        for p in (lvp, lop, evp, vvp):
            dec.free(p)
    out = {"kernels": "k_list_count+k_list_scan+k_list_write<8>", "chunks": len(idx), "ms": round(tot_ms, 4),
           "alg_bytes": tot_bytes, "achieved_GBs": round(tot_bytes / (tot_ms * 1e-3) / 1e9, 1),
           "frac": round(tot_bytes / (tot_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "timer": "HIP events on the decode stream around the K8 kernels (pqg_last_assemble_ms)"}
    if not args.no_verify:
        out["verified"] = bool(ok)
    return out


def compact_line(out):
    """The bench line without its bulky fields: the headline's roofline and
    CPU baseline, and per config value / ms per step / dominant-stage and
    pipeline roofline fractions / bit-exactness."""
    keep_roof = ("bound", "kernel", "achieved", "peak", "unit", "frac", "traffic", "kernel_ms", "pipeline_frac")
    c = {k: out[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                             "higher_is_better", "scaling", "vs_baseline", "dtype", "data")}
    c["config"] = {"workload": "C2: optional INT32 x 7 dictionary widths (see the full line above)",
                   "parallelism": out["config"]["parallelism"]}
    c["roofline"] = {k: out["roofline"][k] for k in keep_roof if k in out["roofline"]}
    cb = out.get("cpu_baseline") or {}
    c["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind") if k in cb} or None
    c["verified_bit_exact"] = out.get("verified_bit_exact")
    c["configs"] = {k: {"value": v["value"], "ms_per_step": v["ms_per_step"],
                        "frac": v["roofline"]["frac"], "dominant": v["roofline"]["kernel"].split(" (")[0],
                        "pipeline_frac": v["roofline"]["pipeline_frac"],
                        "verified_bit_exact": v.get("verified_bit_exact"),
                        "cpu_1thread": (v.get("cpu_baseline") or {}).get("value")}
                    for k, v in out["configs"].items()}
    c["compact"] = True
    return c


def launch_ranks(n):
    """`bench.py --gpus N` without a launcher: run this script as N ranks under
    torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1) and
    return their exit code.  Called before this process touches the GPU."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    log("launching %d ranks: %s" % (n, " ".join(cmd)))
    return subprocess.run(cmd).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=100_000_000, help="C2 rows per file")
    ap.add_argument("--bits", type=str, default="1,2,4,8,12,16,20")
    ap.add_argument("--configs", type=str, default="c1,c1_1page,c2_run_heavy,c3,c3_gzip,c4,c5",
                    help="sub-results besides the C2 headline")
    ap.add_argument("--sub-steps", type=int, default=5)
    ap.add_argument("--c1-rows", type=int, default=10_000_000)
    ap.add_argument("--c3-rows", type=int, default=200_000_000)
    ap.add_argument("--c3gz-rows", type=int, default=50_000_000)
    ap.add_argument("--c4-rows", type=int, default=50_000_000)
    ap.add_argument("--c5-rows-per-rg", type=int, default=15_625_000)
    ap.add_argument("--streams", type=int, default=2, help="decode contexts (HIP streams) the chunks are dealt over")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=16.0, help="bound on the headline CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--only", type=str, default="", help="profiling: run one config alone and print its result")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))  # nothing above touched the GPU
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py: WORLD_SIZE=%d but --gpus %d" % (world, args.gpus))
    dist = None
    device = local
    if world > 1:
        import torch
        import torch.distributed as dist
        ndev = torch.cuda.device_count()  # counting devices does not initialise the GPU
        device = local % max(ndev, 1)
        torch.cuda.set_device(device)
        if ndev >= world:  # one GPU per rank: RCCL for the barrier and the max-time reduction
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:  # ranks sharing a GPU (a 1-GPU test box): the same clock over gloo
            dist.init_process_group("gloo")

    def barrier():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    import pqgpu
    # decode contexts, one HIP stream each (run_workload deals the chunks over them)
    decs = [pqgpu.GpuDecoder(device) for _ in range(max(1, args.streams))]
    dec = decs[0]

    def release(wl):
        for d in wl.devs:
            dec.free(d)
        wl.devs = []

    if args.only:  # profiling runs (tools/gpu_profile.sh): one workload, its own JSON line
        w = gen_workload(args.only, args, rank, world)
        sub, _ = run_workload(w, decs, args, args.steps, args.warmup, barrier, dist, world, rank, 6.0)
        if rank == 0:
            print(json.dumps({"only": args.only, "n_gpus": world, **sub}), flush=True)
        release(w)
        for d in decs:
            d.close()
        return

    wl = gen_workload("c2", args, rank, world)
    head, res = run_workload(wl, decs, args, args.steps, args.warmup, barrier, dist, world, rank, args.cpu_seconds)
    k8 = k8_c2(dec, wl, res, args) if rank == 0 else None
    release(wl)
    del wl
    subs = {}
    for key in [k for k in args.configs.split(",") if k]:
        w = gen_workload(key, args, rank, world)
        # C1's steps take ~0.2 ms: ten times the steps, so host jitter averages out
        n_steps = args.sub_steps * (10 if key in ("c1", "c1_1page") else 1)
        sub, sres = run_workload(w, decs, args, n_steps, 1, barrier, dist, world, rank, 6.0)
        if key == "c5" and rank == 0:
            sub["k8_list_export"] = k8_list_c5(dec, w, sres, args)
        subs[key + ("_shard" if key == "c5" else "")] = sub
        release(w)
        del w

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": head["value"],
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": head["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic",
            "config": {
                "workload": head["workload"],
                "chunks_per_step": head["chunks_per_step"],
                "bytes_in": head["bytes_in"],
                "bytes_out": head["bytes_out"],
                "streams": head["streams"],
                "parallelism": ("row-group shards: one process per GPU, RG i -> GPU floor(i*N/R), no data-path "
                                "collective" if world > 1 else "single GPU"),
            },
            "roofline": head["roofline"],
            "cpu_baseline": head.get("cpu_baseline"),
            "cpu_baseline_all_cores": head.get("cpu_baseline_all_cores"),
            "verified_bit_exact": head.get("verified_bit_exact"),
            "k8_assemble": k8,
            "configs": subs,
        }
        print(json.dumps(out), flush=True)
        # the same line again, compact, LAST: every config's numbers survive a
        # truncated stdout tail (the full line above carries the details)
        print(json.dumps(compact_line(out)), flush=True)
    for d in decs:
        d.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
