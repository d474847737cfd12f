"""Find the size at which a 1-rank RCCL all_to_all_single / self send-recv goes wrong."""
import os

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29556")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
for mb in (256, 512, 768, 1000, 1023, 1024, 1025, 1100, 1536, 2047, 2048, 2049, 3000):
    n = mb * (1 << 20) // 4
    x = torch.arange(n, dtype=torch.int32, device=dev)
    r = torch.full_like(x, -1)
    dist.all_to_all_single(r, x, output_split_sizes=[n], input_split_sizes=[n])
    ok_a2a = bool(torch.equal(r, x))
    bad = (r != x).nonzero()
    first_bad = int(bad[0]) * 4 if bad.numel() else -1
    r2 = torch.full_like(x, -1)
    for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, x, 0), dist.P2POp(dist.irecv, r2, 0)]):
        w.wait()
    ok_p2p = bool(torch.equal(r2, x))
    bad2 = (r2 != x).nonzero()
    x8 = x.view(torch.uint8)
    r3 = torch.full_like(x8, 7)
    dist.all_to_all_single(r3, x8)
    ok_eq = bool(torch.equal(r3, x8))
    print(f"{mb} MiB: a2a_v {ok_a2a} (first bad byte {first_bad}, nbad {bad.numel()}), "
          f"p2p {ok_p2p} (nbad {bad2.numel()}), a2a_equal_u8 {ok_eq}", flush=True)
    del x, r, r2, r3, x8
    torch.cuda.empty_cache()
dist.destroy_process_group()
