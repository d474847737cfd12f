"""launch.bring_up_native: a native communicator whose init is a blocking
collective is brought up without hanging when one rank cannot. Two gloo ranks on the CPU
with fake communicators: the local step fails on rank 1 only, or on rank 0 before it could
publish anything, or the blocking init fails on one rank while its peer is inside it."""
import os
import socket
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mpi_cuda_largescaleknn_amd.parallel import faults as F
from mpi_cuda_largescaleknn_amd.parallel import launch as LA


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _Fake:
    def __init__(self, rank, store, connect_fails=-1, block=False):
        self.rank, self.store, self.connect_fails, self.block = rank, store, connect_fails, block

    def connect(self):
        if self.rank == self.connect_fails:
            raise RuntimeError("init failed here")
        if self.block:  # a peer inside a collective init that never completes
            time.sleep(120)

    def async_error(self):
        return None

    def abort(self):
        pass


def _worker(rank, port, case, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LSKNN_TIMEOUT="60")
    dist.init_process_group("gloo", rank=rank, world_size=2)
    store = dist.distributed_c10d._get_default_store()
    failing = {"rank1_local": 1, "rank0_local": 0, "nofallback": 1}.get(case, -1)

    def make():
        if rank == failing:
            raise OSError(f"dlopen failed on rank {rank}")
        return _Fake(rank, store, connect_fails=1 if case == "init_fails" else -1, block=case == "init_fails")

    res = "?"
    try:
        comm, wd = LA.bring_up_native(make, rank, 2, store,
                                      fallback=None if case == "nofallback" else (lambda: "fallback"))
        res = "fallback" if comm == "fallback" else "native"
        wd.stop()
    except Exception as e:  # noqa: BLE001
        res = "raised: " + str(e)
    with open(os.path.join(out, f"r{rank}.txt"), "w") as f:
        f.write(res)
    if case != "init_fails":
        dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("case,expect", [
    ("ok", ["native", "native"]),
    ("rank1_local", ["fallback", "fallback"]),
    ("rank0_local", ["fallback", "fallback"]),
    ("nofallback", ["raised: the native communicator could not be set up on another rank",
                    "raised: dlopen failed on rank 1"]),
])
def test_agreement_before_the_blocking_init(tmp_path, case, expect):
    t = time.time()
    mp.spawn(_worker, args=(_port(), case, str(tmp_path)), nprocs=2, join=True)
    got = [open(tmp_path / f"r{r}.txt").read() for r in range(2)]
    assert got == expect
    assert time.time() - t < 60


def test_init_failure_on_one_rank_ends_the_blocked_peer(tmp_path):
    """rank 1's init fails while rank 0 is blocked inside its own: rank 1 raises and
    publishes the abort key, rank 0's watchdog (started before the init) ends it."""
    t = time.time()
    ctx = mp.spawn(_worker, args=(_port(), "init_fails", str(tmp_path)), nprocs=2, join=False)
    with pytest.raises(mp.ProcessExitedException) as e:
        while not ctx.join(timeout=30):
            assert time.time() - t < 90, "a rank stayed blocked in the init"
    assert e.value.exit_code == F.EXIT_PEER_ABORT and e.value.error_index == 0
    assert open(tmp_path / "r1.txt").read() == "raised: init failed here"
    assert time.time() - t < 60
