"""Certificate sharding across ranks and the verdict-bitmap all-gather.

Certificates are independent: rank r of W verifies the
contiguous certificate-index range [r*C, (r+1)*C) of the seeded stream, with
no data-path collective.  The only exchange is one all-gather of the per-rank
certificate-accept bitmaps (RCCL over xGMI with backend "nccl"; "gloo" on CPU
for tests), after which every rank holds the verdicts of the whole batch.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np


def shard_range(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) certificate range of `rank` (sizes differ by at most 1)."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    lo = n_total * rank // world
    hi = n_total * (rank + 1) // world
    return lo, hi


def words_for(n_bits: int) -> int:
    return (n_bits + 31) // 32


def allgather_bitmaps(local_bits, world: int, group=None):
    """all_gather_into_tensor of equal-length int32 bitmaps -> [world * words] tensor."""
    import torch
    import torch.distributed as dist

    out = torch.empty(world * local_bits.numel(), dtype=local_bits.dtype, device=local_bits.device)
    dist.all_gather_into_tensor(out, local_bits.contiguous(), group=group)
    return out


def unpack_gathered(gathered_words: np.ndarray, certs_per_rank: int, world: int) -> np.ndarray:
    """Gathered per-rank bitmaps (each padded to whole words) -> bool[world * certs_per_rank]."""
    w = words_for(certs_per_rank)
    g = np.ascontiguousarray(gathered_words, dtype=np.uint32).reshape(world, w)
    bits = np.unpackbits(g.view(np.uint8).reshape(world, -1), axis=1, bitorder="little")[:, :certs_per_rank]
    return bits.reshape(-1).astype(bool)
