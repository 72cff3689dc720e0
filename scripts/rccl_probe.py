#!/usr/bin/env python3
"""Probe: can several ranks share one GPU in one RCCL communicator on this box?
Run: python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1
     --master-port 29533 scripts/rccl_probe.py
Each rank all-to-alls a small tensor over the nccl (= RCCL) backend and checks it."""
import os
import sys

import torch
import torch.distributed as dist


def main() -> int:
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    x = torch.arange(world * 4, device=dev, dtype=torch.int64) + 1000 * rank
    y = torch.empty_like(x)
    dist.all_to_all_single(y, x)
    torch.cuda.synchronize()
    want = torch.cat([torch.arange(4, device=dev, dtype=torch.int64) + 4 * rank + 1000 * g for g in range(world)])
    ok = bool(torch.equal(y, want))
    print(f"rank {rank}/{world}: all_to_all_single over RCCL on one GPU: {'ok' if ok else 'MISMATCH'}", flush=True)
    dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
