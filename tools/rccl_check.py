#!/usr/bin/env python3
"""The RCCL calls bench.py makes for N > 1 (bench.py:624-639, 423-428), run
as one rank under torch.distributed.run on a 1-GPU box: nccl (RCCL) init with
device_id, barrier after a device sync, float64 MAX all-reduce of the elapsed
time on the GPU.  Two ranks cannot share one GPU under RCCL, so this is the
closest rehearsal of that branch a 1-GPU box allows."""
import os
import time

import torch
import torch.distributed as dist

local = int(os.environ.get("LOCAL_RANK", "0"))
torch.cuda.set_device(local)
dist.init_process_group("nccl", device_id=torch.device("cuda", local))
torch.cuda.synchronize()
dist.barrier()
t0 = time.perf_counter()
torch.cuda.synchronize()
dist.barrier()
elapsed = time.perf_counter() - t0
t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
dist.all_reduce(t, op=dist.ReduceOp.MAX)
assert dist.get_backend() == "nccl" and float(t.item()) == elapsed
print("rccl ok: backend %s, world %d, max-reduced %.6f s" % (dist.get_backend(), dist.get_world_size(), float(t.item())))
dist.destroy_process_group()
