"""Shared driver code of the two entrypoints (run, timing, --stats JSON)."""
from __future__ import annotations

import json
import sys
import time

import torch

from ..models.knn_engine import KnnConfig
from ..parallel import pipelines as PL
from ..parallel.launch import Launch


def make_info(launch: Launch, enabled: bool) -> PL.RunInfo:
    return PL.RunInfo(PL.PhaseTimer(enabled, launch.device))


def config(args) -> KnnConfig:
    return KnnConfig(k=args.k, max_radius=args.max_radius, collect_stats=bool(args.stats))


def write_stats(launch: Launch, args, info: PL.RunInfo, extra: dict, t_total: float) -> None:
    if not args.stats:
        return
    rec = {
        "rank": launch.rank,
        "phases_s": info.timer.times,
        "counts": info.plain_counts(),
        "knn": info.stats.counters,
        "total_s": t_total,
        **extra,
    }
    blob = json.dumps(rec).encode()
    t = torch.zeros(1 << 16, dtype=torch.uint8)
    t[: len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
    allv = launch.comm.allgather_host(t)
    if launch.rank == 0:
        recs = []
        for r in range(launch.size):
            raw = bytes(allv[r].tolist()).rstrip(b"\0")
            recs.append(json.loads(raw.decode()))
        with open(args.stats, "w") as f:
            json.dump({"ranks": recs, "k": args.k, "mode": args.mode, "world": launch.size}, f, indent=1)


def log(launch: Launch, msg: str) -> None:
    print(msg, flush=True)


def now(launch: Launch) -> float:
    if launch.device.type == "cuda":
        torch.cuda.synchronize(launch.device)
    return time.perf_counter()


def guarded(launch: Launch, fn) -> int:
    """Run fn(); any error on this rank is reported and broadcast to the peers (whose
    watchdogs then abort) and the process exits 1 — a failing rank never leaves the
    others blocked in a collective (parallel/faults.py)."""
    try:
        return fn()
    except SystemExit:
        raise
    except BaseException as e:  # noqa: BLE001 - every failure ends the job, loudly
        from ..parallel import launch as L
        L.fail(launch, e)
        return 1


def without_spawn(argv: list[str]) -> list[str]:
    """argv minus `--bootstrap spawn` and `--nproc N` (the children's command line)."""
    out, i = [], 0
    while i < len(argv):
        if argv[i] in ("--bootstrap", "--nproc") and i + 1 < len(argv):
            i += 2
            continue
        out.append(argv[i])
        i += 1
    return out


def fail(msg: str, code: int = 1) -> None:
    sys.stderr.write(msg + "\n")
    sys.exit(code)
