"""Search-space partitioning across ranks and devices.

The search index is hierarchical: ``variant ‖ nonce32`` where a variant is one
(extranonce2, BIP320 version bits, ntime offset) combination with its own
midstate. The variant stripes are two-level:

* rank ``r`` of ``W`` owns the residue class ``v ≡ r (mod W)``;
* its ``s`` live devices split that class: device ``i`` searches
  ``v = r + W*i, r + W*i + W*s, ...`` (start ``r + W*i``, stride ``W*s``).

Stripes are disjoint and cover everything, so no per-nonce coordination ever
crosses a GPU boundary. A rank that loses a device (GPU fault)
re-splits only its own class among the survivors (``s`` shrinks), with no
collective and no change on any other rank.

The reference instead hands every device the identical Work
(internal/engine/run.go:1294-1296) and wraps the nonce at 2^32
(internal/miner/worker.go:279) — both defects are fixed here.
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class Stripe:
    start: int
    stride: int

    def variants(self, n: int) -> list[int]:
        return [self.start + k * self.stride for k in range(n)]


def stripe_for(rank: int, world_size: int, device_index: int = 0, devices_per_rank: int = 1) -> Stripe:
    """Stripe of live device ``device_index`` of ``devices_per_rank`` on ``rank``."""
    if not 0 <= rank < world_size or not 0 <= device_index < devices_per_rank:
        raise ValueError("rank/device out of range")
    return Stripe(rank + world_size * device_index, world_size * devices_per_rank)


def apply_stripe(job: dict, stripe: Stripe) -> dict:
    out = dict(job)
    out["variant_start"] = stripe.start
    out["variant_stride"] = stripe.stride
    return out
