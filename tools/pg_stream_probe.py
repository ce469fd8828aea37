"""Which stream does a non-async torch.distributed collective run on, and does it
block the host?  One-rank "nccl" (RCCL) group; run under
`rocprofv3 --kernel-trace` and compare the queue of the gather's copy with the
queue of the kernel launched right before it on the same side stream.
usage: python tools/pg_stream_probe.py"""
import os
import time

import torch
import torch.distributed as dist


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    x = torch.ones(3 << 20, device="cuda")
    out = torch.empty_like(x)
    side = torch.cuda.Stream()
    dist.all_gather_into_tensor(out, x)  # communicator set up
    torch.cuda.synchronize()
    for async_op in (True, False):
        with torch.cuda.stream(side):
            torch.cuda._sleep(20_000_000)
            x.mul_(1.0)  # a kernel on the side stream right before the collective
            t0 = time.perf_counter()
            w = dist.all_gather_into_tensor(out, x, async_op=async_op)
            t1 = time.perf_counter()
            if w is not None:
                w.wait()
            x.add_(0.0)  # and one right after
        busy = not side.query()
        torch.cuda.synchronize()
        print(f"async_op={async_op}: host {1e6 * (t1 - t0):.0f} us, side stream busy after the call: {busy}",
              flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
