"""NUMA placement of a rank's host side next to its GPU.

Every step starts with the rank's points crossing PCIe from pinned host memory (12 B per
point; 1.5 GB per rank at 1B / 8 GPUs) and, on one rank, ends with the distances written
back the same way. On a two-socket MI355X node half of the GPUs sit behind the other
socket: a rank whose process — and so, by first touch, whose pinned buffers — lives on
the far socket pulls its input over the inter-socket link instead of the local memory
controllers. ``bind_to_device`` restricts the calling process to the CPUs of its GPU's
NUMA node (read from sysfs through the PCI address torch reports) before any pinned
allocation. Anything unknown (no sysfs entry, node -1, a CPU set outside the allowed
cgroup) leaves the process as it was. Opt out with ``LSKNN_NUMA_BIND=0``.
"""
from __future__ import annotations

import os


def _parse_cpulist(text: str) -> set[int]:
    cpus: set[int] = set()
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            cpus.update(range(int(a), int(b) + 1))
        else:
            cpus.add(int(part))
    return cpus


def device_numa_cpus(device_index: int, sysfs: str = "/sys") -> tuple[int, set[int]] | None:
    """(numa node, its CPUs) of GPU `device_index`, or None when unknown."""
    import torch

    props = torch.cuda.get_device_properties(device_index)
    addr = f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}.0"
    dev = os.path.join(sysfs, "bus", "pci", "devices", addr)
    try:
        with open(os.path.join(dev, "numa_node")) as f:
            node = int(f.read().strip())
        if node < 0:
            return None
        with open(os.path.join(sysfs, "devices", "system", "node", f"node{node}", "cpulist")) as f:
            cpus = _parse_cpulist(f.read())
    except (OSError, ValueError):
        return None
    return (node, cpus) if cpus else None


def bind_cpus(cpus: set[int]) -> set[int] | None:
    """Restrict this process to `cpus` ∩ its allowed set; returns the new set or None."""
    if not hasattr(os, "sched_setaffinity"):
        return None
    allowed = os.sched_getaffinity(0)
    target = allowed & cpus
    if not target or target == allowed:
        return None
    try:
        os.sched_setaffinity(0, target)
    except OSError:
        return None
    return target


def bind_to_device(device) -> str | None:
    """Bind the calling process to the NUMA node of `device` (a cuda torch.device).
    Returns a short description of what was done, or None."""
    if os.environ.get("LSKNN_NUMA_BIND", "1") == "0" or getattr(device, "type", "cpu") != "cuda":
        return None
    try:
        info = device_numa_cpus(device.index if device.index is not None else 0)
    except Exception:  # noqa: BLE001 — placement is an optimisation, never an error
        return None
    if info is None:
        return None
    node, cpus = info
    got = bind_cpus(cpus)
    return f"numa node {node} ({len(got)} cpus)" if got else None
