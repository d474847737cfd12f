"""Run under `mpirun -n P`: every MpiComm collective against values each rank can
predict (uneven and empty blocks, pieces smaller than the messages). Prints "ok <rank>"."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mpi_cuda_largescaleknn_amd.parallel import mpi as M  # noqa: E402

dev = torch.device(sys.argv[1] if len(sys.argv) > 1 else "cpu")
c = M.MpiComm(dev, force=os.environ.get("LSKNN_FORCE_DIST") == "1")
r, P = c.rank, c.size
c.max_msg_bytes = 40  # force multi-piece messages

# allreduce: sum / min / max over float32, int64, float64
t = torch.arange(5, dtype=torch.float32, device=dev) + r
c.allreduce_(t, "sum")
assert torch.equal(t.cpu(), torch.arange(5, dtype=torch.float32) * P + sum(range(P))), t
t = torch.full((3,), r, dtype=torch.int64, device=dev)
c.allreduce_(t, "max")
assert (t.cpu() == P - 1).all()
t = torch.full((3,), float(r), dtype=torch.float64, device=dev)
c.allreduce_(t, "min")
assert (t.cpu() == 0).all()

# allgather
g = c.allgather(torch.tensor([r, 10 * r], dtype=torch.int32, device=dev))
assert g.shape == (P, 2) and torch.equal(g.cpu()[:, 1], 10 * torch.arange(P, dtype=torch.int32))


# all-to-all-v of float3 rows: rank i sends (i + j) % 3 rows to rank j (some empty)
def rows(i, j):
    n = (i + j) % 3
    return torch.tensor([[i, j, q] for q in range(n)], dtype=torch.float32).reshape(-1, 3)


send = torch.cat([rows(r, j) for j in range(P)]).to(dev)
counts = [(r + j) % 3 for j in range(P)]
recv, rc = c.alltoallv(send, counts)
exp = torch.cat([rows(i, r) for i in range(P)])
assert rc == [(i + r) % 3 for i in range(P)] and torch.equal(recv.cpu(), exp), (recv, exp)

# grouped point-to-point: a ring (the reference's rotation pattern)
nxt, prv = (r + 1) % P, (r - 1) % P
out = c.p2p([(nxt, torch.full((7,), r, dtype=torch.int64, device=dev))], [(prv, (7,), torch.int64)])
assert (out[0].cpu() == prv).all()
c.barrier()
print("ok", r, flush=True)
M.finalize()
