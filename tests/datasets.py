"""Synthetic point sets for tests (uniform, clustered, degenerate)."""
import math

import torch


def uniform(n, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand((n, 3), generator=g) * scale


def clustered(n, seed=0, nclusters=20, sigma=0.01):
    g = torch.Generator().manual_seed(seed)
    centers = torch.rand((nclusters, 3), generator=g)
    which = torch.randint(0, nclusters, (n,), generator=g)
    return (centers[which] + sigma * torch.randn((n, 3), generator=g)).float()


def duplicates(n, seed=0, ndistinct=50):
    g = torch.Generator().manual_seed(seed)
    base = torch.rand((ndistinct, 3), generator=g)
    return base[torch.randint(0, ndistinct, (n,), generator=g)].clone()


def planar(n, seed=0):
    p = uniform(n, seed)
    p[:, 2] = 0.5
    return p


def tilted_plane(n, seed=0, angle=0.6):
    """Uniform points on a plane through the cube's centre, tilted about x (not axis-aligned:
    every coordinate varies)."""
    p = uniform(n, seed) - 0.5
    p[:, 2] = 0.0
    c, s = math.cos(angle), math.sin(angle)
    rot = torch.tensor([[1.0, 0.0, 0.0], [0.0, c, -s], [0.0, s, c]])
    return (p @ rot.T + 0.5).contiguous()


def line(n, seed=0):
    """Uniform points on a segment (1-D data in 3-D)."""
    g = torch.Generator().manual_seed(seed)
    t = torch.rand(n, generator=g)
    return torch.stack([t, 0.3 + 0.2 * t, 0.7 - 0.1 * t], dim=1).contiguous()


def lattice(m):
    r = torch.arange(m, dtype=torch.float32) / m
    x, y, z = torch.meshgrid(r, r, r, indexing="ij")
    return torch.stack([x.flatten(), y.flatten(), z.flatten()], dim=1).contiguous()


def mixed_scale(n, seed=0):
    g = torch.Generator().manual_seed(seed)
    a = torch.rand((n // 2, 3), generator=g) * 1000.0
    b = torch.rand((n - n // 2, 3), generator=g) * 0.001 + 500.0
    return torch.cat([a, b])


GENERATORS = {
    "uniform": uniform,
    "clustered": clustered,
    "duplicates": duplicates,
    "planar": planar,
    "mixed_scale": mixed_scale,
    "tilted_plane": tilted_plane,
    "line": line,
}
