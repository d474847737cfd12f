"""Reference command-line grammar (parsed by the native host runtime).

    hipKNN_unorderedData      <in.float3>   -o <out.float> -k <k> [-r <maxRadius>] [-g <gpusPerNode>]
    hipKNN_prePartitionedData <fileList.txt> -o <prefix>    -k <k> [-r <maxRadius>] [-g <gpusPerNode>]

Semantics (unorderedDataVariant.cu:114-135, prePartitionedDataVariant.cu:185-206):
last positional argument wins; `-k` >= 1, `-o` and the positional are required; any
other dash-argument is an error; on error the reference's stderr text is printed and
the process exits with 1. Extensions (long options only, defaults unchanged):
``--mode {auto,halo,ring,peer}``, ``--device {auto,cuda,cpu}``, ``--stats <json>``,
``-v/--verbose``, ``--bootstrap {auto,env,mpi,spawn}`` (+ ``--nproc N`` for spawn: the
launcher starts N local ranks itself), ``--device-map 0,1,..`` (local rank -> GPU) and
``--balance {auto,on,off}`` (prePartitioned: spatial rebalancing of skewed files).
"""
from __future__ import annotations

import ctypes as C
import math
import sys
from dataclasses import dataclass

from .. import _native

UNORDERED, PREPARTITIONED = 0, 1


@dataclass
class Args:
    input: str
    output: str
    k: int
    max_radius: float
    gpu_affinity: int
    mode: str
    device: str
    stats: str
    verbose: bool
    bootstrap: str = "auto"
    nproc: int = 0
    device_map: list | None = None
    balance: str = "auto"


class UsageError(Exception):
    def __init__(self, text: str, code: int):
        super().__init__(text)
        self.text = text
        self.code = code


def parse(variant: int, argv: list[str]) -> Args:
    """Parse argv (argv[0] = program name). Raises UsageError with the reference text."""
    lib = _native.host()
    arr = (C.c_char_p * len(argv))(*[a.encode() for a in argv])
    out = _native.CliArgs()
    err = C.create_string_buffer(8192)
    rc = lib.lsk_cli_parse(variant, len(argv), arr, C.byref(out), err, len(err))
    if rc != 0:
        raise UsageError(err.value.decode(), rc)
    r = float(out.max_radius)
    return Args(
        input=out.input.decode(),
        output=out.output.decode(),
        k=int(out.k),
        max_radius=r if not math.isnan(r) else math.inf,
        gpu_affinity=int(out.gpu_affinity),
        mode=out.mode.decode(),
        device=out.device.decode(),
        stats=out.stats.decode(),
        verbose=bool(out.verbose),
        bootstrap=out.bootstrap.decode(),
        nproc=int(out.nproc),
        device_map=[int(x) for x in out.device_map.decode().split(",")] if out.device_map else None,
        balance=out.balance.decode(),
    )


def parse_or_exit(variant: int, argv: list[str]) -> Args:
    try:
        return parse(variant, argv)
    except UsageError as e:
        sys.stderr.write(e.text)
        sys.stderr.flush()
        sys.exit(e.code)
