#!/usr/bin/env python3
"""Decode throughput of the MI355X Parquet column-chunk decoder.

Workload (BASELINE.json configs[1], "C2"): optional INT32 column, 100M rows per
file, ~10% nulls, RLE_DICTIONARY with D = 2^b entries for every index width
b in {1, 2, 4, 8, 12, 16, 20} (one file per width, uniform index draws), data
page V1, UNCOMPRESSED, 20 000 rows per page.  A step decodes all seven column
chunks (700M slots) in one batched call, inputs resident in HBM.

Metric: decoded GB/s of uncompressed output (values[:nn] x 4 B + 1 B per
def level), whole job = Σ over ranks / max time over ranks.  One process per
GPU; row groups are independent, so ranks share nothing on the data path
(weak scaling, no collective besides the timing barrier).

Prints ONE JSON line (rank 0).  Outputs are verified bit-exact against the
generator's arrays after timing; the CPU baseline is the oracle (the C++
restatement of parquet-go's decode, single thread like parquet-go's reader)
timed on a bounded sample.
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
STAGES = ["scan", "list", "snappy", "setup", "walk", "levels", "nn_scan", "values", "strings", "finalize"]


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def pmc_traffic(kernel, args):
    """HBM bytes per launch of `kernel` from the committed PMC passes
    (profiles/r01_pmc_traffic.json, made by tools/pmc_traffic.py from two
    rocprofv3 --pmc runs of this same workload), or None for other workloads."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r01_pmc_traffic.json")
    if args.rows != 100_000_000 or args.bits != "1,2,4,8,12,16,20" or not os.path.exists(path):
        return None
    ks = json.load(open(path))["kernels"]
    # the values stage is k_values<1> (4-byte dictionaries) + k_values<0> (all else)
    names = [k for k in ks if k.split("<")[0] == "pqg::" + kernel]
    return sum(ks[k]["traffic"] for k in names) or None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--bits", type=str, default="1,2,4,8,12,16,20")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="bound on the CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import pqgpu
    from gen import pqwrite as W
    from pqgpu import abi

    bits_list = [int(b) for b in args.bits.split(",")]
    t0 = time.time()
    files = list(W.config_c2_family(rows=args.rows, bits_list=bits_list))
    log("rank %d: generated %d files in %.1fs (%.1f MB)" % (rank, len(files), time.time() - t0,
                                                            sum(len(f[1]) for f in files) / 1e6))
    dec = pqgpu.GpuDecoder(local)
    jobs, pfs = [], []
    b_in = 0
    for bits, data, _ in files:
        pf = pqgpu.ParquetFile(data)
        dev = dec.upload(pf.data)
        for rg in range(pf.num_row_groups):
            jobs.append(pqgpu.device_job(pf, rg, 0, dev))
            b_in += pf.chunk_meta(rg, 0).total_compressed_size
        pfs.append(pf)
    n_jobs = len(jobs)
    arr = (abi.ChunkJob * n_jobs)(*jobs)
    res = (abi.ChunkResult * n_jobs)()
    L = dec.L

    def step():
        rc = L.pqg_decode_chunks(dec.ctx, arr, n_jobs, res)
        if rc != 0:
            raise RuntimeError("decode failed: %d" % rc)

    stage_acc = np.zeros(len(STAGES))
    tmp = (C.c_float * 16)()

    def stage_times():
        k = L.pqg_last_timings(dec.ctx, tmp, 16)
        return np.array([tmp[i] for i in range(1, min(k, 1 + len(STAGES)))])

    for _ in range(max(args.warmup, 1)):
        step()
    for i in range(n_jobs):
        assert res[i].status == 0, abi.status_name(res[i].status)

    def barrier():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    barrier()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
        stage_acc += stage_times()
    t_end = time.perf_counter()
    barrier()
    elapsed = t_end - t_start
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # ---- bytes
    nn_total = sum(res[i].num_values for i in range(n_jobs))
    slots_total = sum(res[i].num_slots for i in range(n_jobs))
    b_out = nn_total * 4 + slots_total * 1
    value = b_out * world * args.steps / elapsed / 1e9
    ms_per_step = elapsed / args.steps * 1e3
    stage_ms = stage_acc / args.steps
    dev_ms = float(stage_ms.sum())

    # dominant kernel: values (dictionary gather) or levels
    pages_info = [dec.pages(i) for i in range(n_jobs)]
    val_in = sum(p.uncompressed_size for pl in pages_info for p in pl if p.page_type == 0)
    dom = int(np.argmax(stage_ms))
    # exact level-stream sizes: read the u32 length prefix of each V1 page body
    def_stream = 0
    for pf, pl, j in zip(pfs, pages_info, jobs):
        m = pf.chunk_meta(0, 0)
        for p in pl:
            if p.page_type == 0:
                at = m.start + p.payload_offset
                def_stream += 4 + int.from_bytes(pf.data[at:at + 4], "little")
    alg = {
        "levels": def_stream + slots_total,                      # def-level stream in, 1 B/slot out
        "values": (val_in - def_stream) + nn_total * 4,          # index stream in, values out
        "scan": 0, "list": 0, "snappy": 0, "nn_scan": 0, "finalize": 0,
    }
    dom_name = STAGES[dom]
    dom_bytes = alg.get(dom_name, 0)
    achieved = dom_bytes / (stage_ms[dom] * 1e-3) / 1e9 if stage_ms[dom] > 0 else 0.0
    pipeline_gbs = (b_in + b_out) / (dev_ms * 1e-3) / 1e9 if dev_ms > 0 else 0.0

    # ---- verify bit-exact against the generator's arrays (size-independent check)
    verified = None
    if not args.no_verify:
        ok = True
        for i, (bits, data, (defs, vals)) in enumerate(files):
            r = res[i]
            got_d = dec.d2h(r.def_levels, r.num_slots)
            got_v = dec.d2h(r.values, r.values_bytes).view(np.int32)
            ok &= r.num_slots == len(defs) and np.array_equal(got_d, defs) and np.array_equal(got_v, vals)
        verified = bool(ok)
        if not ok:
            log("VERIFY FAILED")

    # ---- K8 (pqg_assemble) on chunk 0's decoded arrays: validity bitmap + spaced
    # values (row offsets are trivial for a flat column).  Not part of `value`.
    k8 = None
    if rank == 0:
        r = res[0]
        a, vb, sb, _ = dec.assemble(r.def_levels, r.rep_levels, r.values, r.num_slots, 1, 0, 4,
                                    validity=True, spaced=True, offsets=False)
        reps = 5
        t1 = time.perf_counter()
        for _ in range(reps):
            rc = L.pqg_assemble(dec.ctx, C.byref(a))
            assert rc == 0, abi.status_name(rc)
        k8_ms = (time.perf_counter() - t1) / reps * 1e3
        n = r.num_slots
        k8_bytes = n + r.num_values * 4 + n * 4 + (n + 7) // 8
        k8 = {"kernels": "k_asm_count+k_asm_scan+k_asm_write<4>", "slots": n, "ms": round(k8_ms, 4),
              "alg_bytes": k8_bytes, "achieved_GBs": round(k8_bytes / (k8_ms * 1e-3) / 1e9, 1),
              "frac": round(k8_bytes / (k8_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "timer": "host wall, incl. sync"}
        if not args.no_verify:
            defs, vals = files[0][2]
            valid = defs == 1
            sp = dec.d2h(sb, n * 4).view(np.int32)
            bm = np.unpackbits(dec.d2h(vb, (n + 7) // 8), bitorder="little")[:n].astype(bool)
            k8["verified"] = bool(np.array_equal(bm, valid) and np.array_equal(sp[valid], vals)
                                  and not sp[~valid].any() and a.num_valid == int(valid.sum()))
        dec.free(vb)
        dec.free(sb)

    # ---- CPU baseline: oracle (single thread) on a bounded sample
    cpu = None
    if rank == 0 and not args.no_cpu:
        from oracle import pyoracle as O
        OL = O.lib()
        done_bytes, t_cpu, names = 0, 0.0, []
        for bits, data, _ in files:
            pf = pqgpu.ParquetFile(data)
            job, _ = pf.host_job(0, 0)
            r = abi.ChunkResult()
            pages = (abi.PageInfo * 1)()
            n = C.c_int(0)
            t1 = time.perf_counter()
            OL.pqo_decode_chunk(C.byref(job), C.byref(r), pages, 1, C.byref(n))
            t_cpu += time.perf_counter() - t1
            done_bytes += r.num_values * 4 + r.num_slots
            OL.pqo_free_result(C.byref(r))
            names.append("b=%d" % bits)
            if t_cpu >= args.cpu_seconds:
                break
        cpu = {"value": round(done_bytes / t_cpu / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": "port",
               "sample": "oracle (C++ restatement of parquet-go readPages/readPageData) on %d of the %d C2 files "
                         "(%s; %d rows each), single thread like parquet-go's one-goroutine FileReader; %.1fs"
                         % (len(names), len(files), ",".join(names), args.rows, t_cpu)}

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic",
            "config": {
                "workload": "C2: optional INT32, %d rows x %d dictionary widths (b=%s), ~10%% nulls, "
                            "RLE_DICTIONARY, V1, UNCOMPRESSED, 20000 rows/page" % (args.rows, len(bits_list), args.bits),
                "chunks_per_step": n_jobs,
                "bytes_in": b_in,
                "bytes_out": b_out,
                "parallelism": "replicas: one process per GPU, independent row groups" if world > 1 else "single GPU",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "k_%s" % dom_name,
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": pmc_traffic("k_" + dom_name, args),
                "alg_bytes_per_launch": dom_bytes,
                "kernel_ms": round(float(stage_ms[dom]), 4),
                "pipeline_device_ms": round(dev_ms, 4),
                "pipeline_frac": round(pipeline_gbs / HBM_PEAK_GBS, 4),
                "stage_ms": {n: round(float(x), 4) for n, x in zip(STAGES, stage_ms)},
            },
            "cpu_baseline": cpu,
            "verified_bit_exact": verified,
            "k8_assemble": k8,
        }
        print(json.dumps(out), flush=True)
    dec.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
