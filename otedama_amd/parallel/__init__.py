"""Multi-GPU node parallelism: one rank per GPU over torch.distributed (RCCL).

Exports resolve lazily (PEP 562) so that importing the stripe planner from the engine does not pull in torch:
a CPU-only ``otedama run`` starts in well under a second.
"""
import importlib

_EXPORTS = {
    "DistInfo": "comm", "NodeComm": "comm", "barrier": "comm", "init_from_env": "comm", "shutdown": "comm",
    "Stripe": "partition", "apply_stripe": "partition", "stripe_for": "partition",
}
__all__ = list(_EXPORTS)


def __getattr__(name):
    mod = _EXPORTS.get(name)
    if mod is None:
        raise AttributeError(f"module {__name__!r} has no attribute {name!r}")
    return getattr(importlib.import_module(f"{__name__}.{mod}"), name)
