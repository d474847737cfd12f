"""Process-group bootstrap for the CLI apps: one process per GPU.

Accepted launchers (all run the same code):

* ``torchrun --nproc-per-node N -m mpi_cuda_largescaleknn_amd.apps.unordered ...``
  (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* from the environment);
* ``mpirun -n N bin/hipKNN_unorderedData ...`` — MPICH (PMI_RANK/PMI_SIZE) or Open MPI
  (OMPI_COMM_WORLD_*) environment, rendezvous on MASTER_ADDR (default 127.0.0.1) /
  MASTER_PORT (default 29511); MPI itself carries data only with
  ``LSKNN_DIST_BACKEND=mpi`` (the reference's MPI_Init / MPIComm,
  unorderedDataVariant.cu:30-39, 107);
* a plain single process.

Device selection follows the reference's ``-g G`` (device = rank % G,
unorderedDataVariant.cu:138-143); without ``-g`` the local rank picks the device
(the reference would put every rank on GPU 0).

GPU runs move data with RCCL: by default the native communicator (``rccl``,
parallel/rccl.py: RCCL 2.27 called from C++ on the pipeline's own streams, a gloo group
for control; measured faster than torch's group, default_gpu_backend), or torch's
ProcessGroupNCCL (``LSKNN_DIST_BACKEND=nccl``, torch's bundled RCCL 2.26). CPU runs use
gloo.
``LSKNN_DIST_BACKEND=mpi`` moves the data with MPI (parallel/mpi.py, the native host-staged
communicator; launch with mpirun).
``LSKNN_DIST_BACKEND=gloo`` forces gloo with GPU data (collectives staged through host
memory, see TorchComm): the only way to run several GPU ranks on one device, since RCCL
refuses two ranks on the same GPU.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist

from ..utils import numa
from . import faults as F
from .comm import Comm, SingleComm, TorchComm


@dataclass
class Launch:
    rank: int
    size: int
    local_rank: int
    device: torch.device
    comm: Comm
    store: object = None
    watchdog: F.Watchdog | None = None


def _env_int(*names, default=None):
    for n in names:
        v = os.environ.get(n)
        if v is not None and v != "":
            return int(v)
    return default


_RANK_VARS = {
    "env": (("RANK",), ("WORLD_SIZE",), ("LOCAL_RANK",)),
    "mpi": (("PMI_RANK", "OMPI_COMM_WORLD_RANK", "PMIX_RANK"), ("PMI_SIZE", "OMPI_COMM_WORLD_SIZE"),
            ("MPI_LOCALRANKID", "OMPI_COMM_WORLD_LOCAL_RANK")),
}


def rank_info(bootstrap: str = "auto") -> tuple[int, int, int]:
    """(rank, size, local rank) from the launcher's environment: torchrun / spawn
    (`env`: RANK, WORLD_SIZE, LOCAL_RANK), MPICH / Open MPI / PMIx (`mpi`), or either
    (`auto`, torchrun variables first)."""
    if bootstrap == "auto":
        names = [sum(v, ()) for v in zip(_RANK_VARS["env"], _RANK_VARS["mpi"])]
    elif bootstrap in _RANK_VARS:
        names = list(_RANK_VARS[bootstrap])
    else:
        raise ValueError(f"bootstrap must be auto, env or mpi, not {bootstrap!r}")
    rank = _env_int(*names[0], default=0)
    size = _env_int(*names[1], default=1)
    local = _env_int(*names[2], default=rank)
    if not (0 <= rank < size):
        raise ValueError(f"bad rank {rank} of {size} from the {bootstrap} bootstrap")
    return rank, size, local


def pick_device(rank: int, local: int, ndev: int, gpu_affinity: int = 0,
                device_map: list[int] | None = None) -> int:
    """GPU of this rank: --device-map [local % len] if given, else the reference's
    -g G (rank % G, unorderedDataVariant.cu:138-143), else the local rank (fixes D9)."""
    if device_map:
        return device_map[local % len(device_map)]
    if gpu_affinity:
        return rank % gpu_affinity
    return local % max(1, ndev)


def default_gpu_backend() -> str:
    """The GPU data path when LSKNN_DIST_BACKEND is unset: "rccl" (the native communicator,
    parallel/rccl.py, on ROCm's RCCL 2.27) when its library is built and an RCCL library
    is present, else "nccl" (torch's ProcessGroupNCCL on its bundled RCCL 2.26). Measured
    on a forced 1-rank group, 1e8 points, stream of sets: native 1056.2 / 1058.9 Mpts/s
    against torch 1036.2 / 1042.3 (alltoallv of the points 0.94-0.97 ms against 1.27-1.28;
    profiles/r5_rccl_ab/); 2.27 also carries the fix for the > 1 GiB corruption that
    comm.MAX_MSG_BYTES works around on 2.26. The answer depends only on files of the
    image, so every rank of a job makes the same choice."""
    from .. import _build
    from .rccl import rccl_path
    return "rccl" if os.path.exists(_build.COMM_LIB) and os.path.exists(rccl_path()) else "nccl"


def init(device_pref: str = "auto", gpu_affinity: int = 0, verbose: bool = False,
         force_distributed: bool | None = None, bootstrap: str = "auto",
         device_map: list[int] | None = None) -> Launch:
    """Bootstrap this rank. `force_distributed` (default: env LSKNN_FORCE_DIST=1) builds a
    process group and the multi-rank pipeline even for a single rank, so that a 1-GPU run
    executes every collective through RCCL."""
    if force_distributed is None:
        force_distributed = os.environ.get("LSKNN_FORCE_DIST", "0") == "1"
    rank, size, local = rank_info("auto" if bootstrap == "spawn" else bootstrap)
    use_gpu = device_pref != "cpu" and torch.cuda.is_available()
    if device_pref == "cuda" and not torch.cuda.is_available():
        raise RuntimeError("--device cuda requested but no GPU is available")
    if use_gpu:
        ndev = torch.cuda.device_count()
        dev_id = pick_device(rank, local, ndev, gpu_affinity, device_map)
        if not 0 <= dev_id < ndev:
            raise ValueError(f"rank {rank}: GPU {dev_id} does not exist ({ndev} visible)")
        if gpu_affinity:
            print(f"#{rank}/{size}setting active GPU #{dev_id}", flush=True)
        torch.cuda.set_device(dev_id)
        device = torch.device("cuda", dev_id)
        # before any pinned allocation: host buffers land on the GPU's NUMA node
        bound = numa.bind_to_device(device)
        if bound and verbose:
            print(f"#{rank}/{size}: bound to {bound}", flush=True)
    else:
        device = torch.device("cpu")
    fault = F.parse_fault(os.environ.get("LSKNN_FAULT"))
    store = watchdog = None
    if size > 1 or force_distributed:
        port_given = bool(os.environ.get("MASTER_PORT"))
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        os.environ["RANK"], os.environ["WORLD_SIZE"] = str(rank), str(size)
        # collective timeout = watchdog timeout; RCCL errors surface asynchronously
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        timeout = datetime.timedelta(seconds=F.timeout_s())
        chosen = os.environ.get("LSKNN_DIST_BACKEND")
        backend = chosen or (default_gpu_backend() if use_gpu else "gloo")
        if backend not in ("nccl", "gloo", "rccl", "mpi"):
            raise ValueError(f"LSKNN_DIST_BACKEND must be nccl, rccl, gloo or mpi, not {backend!r}")
        if backend == "mpi":
            # native MPI host communicator (parallel/mpi.py): the data path is MPI (the
            # reference's transport, host-staged); rank / size come from MPI_COMM_WORLD;
            # a gloo group on a port broadcast over MPI carries the store and the watchdog
            # (a rank that exits early makes mpirun end the others)
            from . import mpi as M
            comm = M.MpiComm(device, force=force_distributed)
            if (comm.rank, comm.size) != (rank, size):
                raise RuntimeError(f"MPI_COMM_WORLD says rank {comm.rank} of {comm.size}, the launcher "
                                   f"environment {rank} of {size}")
            port = M.bcast_port(rank)
            if not port_given:
                os.environ["MASTER_PORT"] = str(port)
            dist.init_process_group("gloo", rank=rank, world_size=size, timeout=timeout)
            store = dist.distributed_c10d._get_default_store()
            watchdog = F.Watchdog(rank, size, store).start()
            return Launch(rank, size, local, device, F.MonitoredComm(comm, fault), store, watchdog)
        if backend == "rccl":
            # native RCCL communicator (parallel/rccl.py); a gloo group carries the store,
            # the watchdog and host-side control
            if not use_gpu:
                raise ValueError("LSKNN_DIST_BACKEND=rccl needs a GPU run")
            from .rccl import RcclComm
            dist.init_process_group("gloo", rank=rank, world_size=size, timeout=timeout)
            store = dist.distributed_c10d._get_default_store()

            def torch_group() -> Comm:
                if rank == 0:
                    print("lsknn: native RCCL communicator unavailable on some rank; using torch's process group",
                          flush=True)
                opts = dist.ProcessGroupNCCL.Options()
                opts.is_high_priority_stream = True
                group = dist.new_group(backend="nccl", pg_options=opts)
                return TorchComm(device, group=group, force=force_distributed)

            comm, watchdog = bring_up_native(
                lambda: RcclComm(device, rank, size, store, force=force_distributed, connect=False),
                rank, size, store, fallback=None if chosen else torch_group)
            return Launch(rank, size, local, device, F.MonitoredComm(comm, fault), store, watchdog)
        if backend == "nccl":
            if not use_gpu:
                raise ValueError("LSKNN_DIST_BACKEND=nccl needs a GPU run")
            # RCCL's internal streams at high priority: the halo exchange runs while the
            # local k-NN grid fills every CU (pipelines.knn_with_halo), and a normal-priority
            # collective kernel would only get CUs when that grid drains
            opts = dist.ProcessGroupNCCL.Options()
            opts.is_high_priority_stream = True
            dist.init_process_group("nccl", rank=rank, world_size=size, device_id=device, timeout=timeout,
                                    pg_options=opts)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=size, timeout=timeout)
        comm: Comm = TorchComm(device, force=force_distributed)
        store = dist.distributed_c10d._get_default_store()
        watchdog = F.Watchdog(rank, size, store).start()
    else:
        comm = SingleComm(device)
    return Launch(rank, size, local, device, F.MonitoredComm(comm, fault), store, watchdog)


def bring_up_native(make, rank: int, size: int, store, fallback=None):
    """Bring up a native communicator whose init is a blocking collective (RCCL's
    ncclCommInitRank) without hanging when some rank cannot.

    1. `make()` runs the local steps only (load the library; rank 0 publishes the unique
       id): a failure there is caught;
    2. the ranks agree over the gloo control group (MIN of the local results) BEFORE any
       of them enters the blocking init: if some rank failed, none enters it, and every
       rank takes `fallback()` (or, with no fallback — the backend was the user's choice —
       re-raises the local error, or reports the failing peer);
    3. the watchdog starts, then `connect()`: a rank that fails inside the init publishes
       the abort key, so the peers' watchdogs end them instead of leaving them blocked.
    Returns (comm, watchdog). (one non-zero rank failing, or rank 0
    failing before it published the id, used to leave the others blocked.)"""
    comm, err = None, None
    try:
        comm = make()
    except Exception as e:  # noqa: BLE001 (decided together below)
        err = e
    ok = torch.tensor([0 if comm is None else 1], dtype=torch.int32)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if int(ok.item()) == 0:
        if fallback is not None:
            comm = fallback()
            return comm, F.Watchdog(rank, size, store).start()
        if err is not None:
            raise err
        raise RuntimeError("the native communicator could not be set up on another rank")
    watchdog = F.Watchdog(rank, size, store).start()
    try:
        comm.connect()
    except Exception as e:
        try:
            store.set(F.ABORT_KEY, f"rank {rank}: communicator init failed: {e}")
        except Exception:  # noqa: BLE001 - raising anyway
            pass
        raise
    watchdog.comm_check, watchdog.on_abort = comm.async_error, comm.abort
    return comm, watchdog


def launcher_env() -> bool:
    """True when a launcher (torchrun, spawn_local, mpirun) has set this process's rank."""
    return any(os.environ.get(v) not in (None, "") for v in
               ("RANK", "WORLD_SIZE", "PMI_RANK", "OMPI_COMM_WORLD_RANK", "PMIX_RANK"))


def spawn_local(nproc: int, module: str, argv: list[str]) -> int:
    """--bootstrap spawn: start `nproc` local ranks of `python -m module argv...` (each
    with RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* set, bootstrap env) and wait for them.
    Called before anything touches the GPU. A failing rank's peers abort through the
    watchdog; the launcher returns the first non-zero exit code."""
    import sys

    return spawn_ranks(nproc, [sys.executable, "-m", module, *argv, "--bootstrap", "env"])


def spawn_ranks(nproc: int, cmd: list[str]) -> int:
    """Run `cmd` as `nproc` local ranks (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR /
    MASTER_PORT on a free loopback port), the torchrun contract, and wait for all of them.
    Must be called before this process touches the GPU (the children open it). Returns
    the first non-zero exit code; once a rank fails, the others get 60 s to end through
    the abort broadcast (parallel/faults.py) before they are terminated."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(nproc):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(nproc), LOCAL_RANK=str(r),
                   LOCAL_WORLD_SIZE=str(nproc), MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"),
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=env))
    rc = 0
    live = list(procs)
    deadline = None
    import time
    while live:
        for p in list(live):
            code = p.poll()
            if code is not None:
                live.remove(p)
                if code and not rc:
                    rc = code
                    deadline = time.monotonic() + 60.0
        if live and deadline is not None and time.monotonic() > deadline:
            for p in live:
                p.terminate()
            for p in live:
                p.wait()
            break
        time.sleep(0.05)
    return rc


def finalize(launch: Launch) -> None:
    # the watchdog stops first: peers leaving the final barrier early close the store
    if launch.watchdog is not None:
        launch.watchdog.stop()
    if dist.is_initialized():
        launch.comm.barrier()
        inner = getattr(launch.comm, "inner", launch.comm)
        if hasattr(inner, "destroy"):  # native RCCL communicator
            inner.destroy()
        dist.destroy_process_group()
        if getattr(inner, "backend", None) == "mpi":
            from . import mpi as M
            M.finalize()


def fail(launch: Launch, exc: BaseException) -> None:
    """Report a rank failure (stderr + abort broadcast to the peers) and end the
    process with exit code 1 without running teardown that could block on a peer."""
    import sys
    import traceback

    sys.stdout.flush()
    msg = f"{type(exc).__name__}: {exc}"
    sys.stderr.write(f"#{launch.rank}/{launch.size}: error: {msg}\n")
    if os.environ.get("LSKNN_TRACEBACK"):
        traceback.print_exception(exc)
    sys.stderr.flush()
    F.announce_failure(launch.store, launch.rank, launch.size, exc)
    os._exit(1)
