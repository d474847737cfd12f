"""Process-group bootstrap for the CLI apps: one process per GPU.

Accepted launchers (all run the same code):

* ``torchrun --nproc-per-node N -m mpi_cuda_largescaleknn_amd.apps.unordered ...``
  (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* from the environment);
* ``mpirun -n N bin/hipKNN_unorderedData ...`` — MPICH (PMI_RANK/PMI_SIZE) or Open MPI
  (OMPI_COMM_WORLD_*) environment, rendezvous on MASTER_ADDR (default 127.0.0.1) /
  MASTER_PORT (default 29511); MPI itself is not used (the reference's MPI_Init /
  MPIComm, unorderedDataVariant.cu:30-39, 107);
* a plain single process.

Device selection follows the reference's ``-g G`` (device = rank % G,
unorderedDataVariant.cu:138-143); without ``-g`` the local rank picks the device
(the reference would put every rank on GPU 0).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist

from .comm import Comm, SingleComm, TorchComm


@dataclass
class Launch:
    rank: int
    size: int
    local_rank: int
    device: torch.device
    comm: Comm


def _env_int(*names, default=None):
    for n in names:
        v = os.environ.get(n)
        if v is not None and v != "":
            return int(v)
    return default


def init(device_pref: str = "auto", gpu_affinity: int = 0, verbose: bool = False) -> Launch:
    rank = _env_int("RANK", "PMI_RANK", "OMPI_COMM_WORLD_RANK", "PMIX_RANK", default=0)
    size = _env_int("WORLD_SIZE", "PMI_SIZE", "OMPI_COMM_WORLD_SIZE", default=1)
    local = _env_int("LOCAL_RANK", "MPI_LOCALRANKID", "OMPI_COMM_WORLD_LOCAL_RANK", default=rank)
    use_gpu = device_pref != "cpu" and torch.cuda.is_available()
    if device_pref == "cuda" and not torch.cuda.is_available():
        raise RuntimeError("--device cuda requested but no GPU is available")
    if use_gpu:
        ndev = torch.cuda.device_count()
        dev_id = rank % gpu_affinity if gpu_affinity else local % max(1, ndev)
        if gpu_affinity:
            print(f"#{rank}/{size}setting active GPU #{dev_id}", flush=True)
        torch.cuda.set_device(dev_id)
        device = torch.device("cuda", dev_id)
    else:
        device = torch.device("cpu")
    if size > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        os.environ["RANK"], os.environ["WORLD_SIZE"] = str(rank), str(size)
        if use_gpu:
            dist.init_process_group("nccl", rank=rank, world_size=size, device_id=device)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=size)
        comm: Comm = TorchComm(device)
    else:
        comm = SingleComm(device)
    return Launch(rank, size, local, device, comm)


def finalize(launch: Launch) -> None:
    if launch.size > 1 and dist.is_initialized():
        launch.comm.barrier()
        dist.destroy_process_group()
