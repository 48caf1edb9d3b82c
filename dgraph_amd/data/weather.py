"""Synthetic ERA5-shaped weather data (experiments/GraphCast/dataset.py:24-226 behaviour).

Temperatures on a 721 x 1440 latitude/longitude grid for ``C`` atmospheric channels:
``T = base + amplitude * cos(lat) * sin(2 pi day / 365 + lon) - 0.5 * channel + noise``.
Every rank materialises only ITS grid points (rows of ``graph.grid_global_ids``) and the
noise is a deterministic function of (day, channel, global grid id), so the data do not
depend on the number of ranks (the reference generated the whole year x grid on every
rank, then padded and sliced it). A sample is ``(x_t, x_{t+1})`` as ``[L_grid, C]`` rows.
"""
from __future__ import annotations

import math
from typing import Tuple

import torch

from .graphcast_graph import DistributedGraphCastGraph, lat_lon_grid


def _hash_noise(day: int, ch: torch.Tensor, gid: torch.Tensor, std: float) -> torch.Tensor:
    """Counter-based standard normal noise (Box-Muller on a splitmix-style hash)."""
    key = (gid.to(torch.int64).unsqueeze(1) * 1_000_003 + ch.unsqueeze(0) * 7919
           + day * 104_729)
    def mix(z):
        z = (z ^ (z >> 31)) * 0x5DEECE66D
        z = (z ^ (z >> 29)) & 0xFFFFFFFFFF
        return z
    u1 = (mix(key) % 1_000_003 + 1).double() / 1_000_004.0
    u2 = (mix(key + 0x9E3779B9) % 1_000_003).double() / 1_000_003.0
    return (torch.sqrt(-2.0 * torch.log(u1)) * torch.cos(2.0 * math.pi * u2) * std).float()


class SyntheticWeatherDataset(torch.utils.data.Dataset):
    def __init__(self, graph: DistributedGraphCastGraph, num_channels: int = 73,
                 num_samples_per_year: int = 4, num_steps: int = 1,
                 base_temp: float = 15.0, amplitude: float = 10.0, noise_level: float = 2.0,
                 dtype: torch.dtype = torch.float32):
        self.graph = graph
        self.num_channels = num_channels
        self.num_days = num_samples_per_year
        self.num_steps = num_steps
        self.base, self.amp, self.noise = base_temp, amplitude, noise_level
        self.dtype = dtype
        lat, lon = lat_lon_grid(graph.grid_shape)
        gid = graph.grid_global_ids.cpu().long()
        Wd = graph.grid_shape[1]
        self._lat = torch.from_numpy(lat).float()[gid // Wd]
        self._lon = torch.from_numpy(lon).float()[gid % Wd]
        self._gid = gid

    def state(self, day: int) -> torch.Tensor:
        ch = torch.arange(self.num_channels)
        lat = torch.deg2rad(self._lat).unsqueeze(1)
        lon = torch.deg2rad(self._lon).unsqueeze(1)
        t = (self.base + self.amp * torch.cos(lat) * torch.sin(2 * math.pi * day / 365.0 + lon)
             - 0.5 * ch.float().unsqueeze(0))
        t = t + _hash_noise(day, ch, self._gid, self.noise)
        return t.to(self.dtype)

    def __len__(self) -> int:
        return max(self.num_days - self.num_steps, 1)

    def __getitem__(self, idx: int) -> Tuple[torch.Tensor, torch.Tensor]:
        return self.state(idx), self.state(idx + self.num_steps)
