"""Which engine serves a 4 GB device -> pinned host copy (SDMA or a blit kernel), by
stream and concurrency: run under rocprofv3 --kernel-trace --memory-copy-trace."""
import time

import torch

dev = torch.device("cuda:0")
n = 1 << 30
src = torch.rand(n, device=dev)
dst = torch.empty(n, pin_memory=True)
hsrc = torch.empty(3 * n, pin_memory=True)
hdst = torch.empty(3 * n, device=dev)
side = torch.cuda.Stream(dev)
side2 = torch.cuda.Stream(dev)


def timed(tag, fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    print(f"{tag}: {1e3 * (time.perf_counter() - t):.1f} ms", flush=True)


timed("d2h default stream", lambda: dst.copy_(src, non_blocking=True))


def on_side():
    with torch.cuda.stream(side):
        dst.copy_(src, non_blocking=True)


timed("d2h side stream", on_side)


def with_h2d():
    with torch.cuda.stream(side2):
        hdst.copy_(hsrc, non_blocking=True)
    with torch.cuda.stream(side):
        dst.copy_(src, non_blocking=True)


timed("h2d side2 + d2h side", with_h2d)


def with_h2d_same():
    with torch.cuda.stream(side):
        hdst.copy_(hsrc, non_blocking=True)
        dst.copy_(src, non_blocking=True)


timed("h2d then d2h, one side stream", with_h2d_same)


def d2h_after_h2d_done():
    with torch.cuda.stream(side2):
        hdst.copy_(hsrc, non_blocking=True)
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        dst.copy_(src, non_blocking=True)


timed("h2d (done), then d2h side", d2h_after_h2d_done)
