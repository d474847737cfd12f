"""NUMA placement helper (utils/numa.py): sysfs parsing against a fake tree, and the
binding never fails or widens the allowed CPU set."""
import os
from types import SimpleNamespace

import torch

from mpi_cuda_largescaleknn_amd.utils import numa


def test_parse_cpulist():
    assert numa._parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert numa._parse_cpulist("") == set()


def _fake_sysfs(tmp_path, node, cpulist):
    dev = tmp_path / "bus" / "pci" / "devices" / "0000:c1:00.0"
    dev.mkdir(parents=True)
    (dev / "numa_node").write_text(f"{node}\n")
    nd = tmp_path / "devices" / "system" / "node" / "node1"
    nd.mkdir(parents=True)
    (nd / "cpulist").write_text(cpulist)


def _props(monkeypatch):
    props = SimpleNamespace(pci_domain_id=0, pci_bus_id=0xC1, pci_device_id=0)
    monkeypatch.setattr(torch.cuda, "get_device_properties", lambda i: props)


def test_device_numa_cpus_from_sysfs(tmp_path, monkeypatch):
    _fake_sysfs(tmp_path, 1, "48-95,144-191\n")
    _props(monkeypatch)
    node, cpus = numa.device_numa_cpus(0, sysfs=str(tmp_path))
    assert node == 1 and len(cpus) == 96 and 48 in cpus and 191 in cpus


def test_unknown_node_is_none(tmp_path, monkeypatch):
    _fake_sysfs(tmp_path, -1, "0-3")
    _props(monkeypatch)
    assert numa.device_numa_cpus(0, sysfs=str(tmp_path)) is None
    assert numa.device_numa_cpus(0, sysfs=str(tmp_path / "missing")) is None


def test_bind_cpus_never_widens():
    allowed = os.sched_getaffinity(0)
    assert numa.bind_cpus(set(allowed)) is None          # nothing to restrict
    assert numa.bind_cpus({10 ** 6}) is None              # outside the allowed set
    assert os.sched_getaffinity(0) == allowed


def test_bind_to_device_opt_out_and_cpu(monkeypatch):
    assert numa.bind_to_device(torch.device("cpu")) is None
    monkeypatch.setenv("LSKNN_NUMA_BIND", "0")
    assert numa.bind_to_device(torch.device("cuda", 0)) is None
