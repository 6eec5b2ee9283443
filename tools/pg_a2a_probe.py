#!/usr/bin/env python3
"""Host cost of torch's process-group all-to-all at RCCL world 1 (the call the lagged schedule makes each
round, distributed.py HaloExchange), for the same sizes as tools/rccl_probe.cpp: `pg.alltoall_base` on a
side stream set current, then `work.wait()` -- host microseconds per call, 400 calls in bursts of 20."""
import os
import time

import torch
import torch.distributed as dist


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    pg = dist.distributed_c10d._get_default_group()
    side = torch.cuda.Stream(dev)
    for nbytes in (64 << 10, 3538944, 27557888):
        sb = torch.ones(nbytes, dtype=torch.uint8, device=dev)
        rb = torch.empty_like(sb)
        with torch.cuda.stream(side):
            for _ in range(20):
                pg.alltoall_base(rb, sb, [nbytes], [nbytes], dist.AllToAllOptions()).wait()
        torch.cuda.synchronize()
        host, reps = 0.0, 400
        with torch.cuda.stream(side):
            for _ in range(reps // 20):
                t0 = time.perf_counter()
                for _ in range(20):
                    pg.alltoall_base(rb, sb, [nbytes], [nbytes], dist.AllToAllOptions()).wait()
                host += time.perf_counter() - t0
                torch.cuda.synchronize()
        print(f"pg alltoall_base bytes {nbytes:9d}  host {host / reps * 1e6:6.2f} us/call", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
