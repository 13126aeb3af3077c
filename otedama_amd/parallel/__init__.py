"""Multi-GPU node parallelism: one rank per GPU over torch.distributed (RCCL)."""
from otedama_amd.parallel.comm import DistInfo, NodeComm, barrier, init_from_env, shutdown
from otedama_amd.parallel.partition import Stripe, apply_stripe, stripe_for

__all__ = ["DistInfo", "NodeComm", "barrier", "init_from_env", "shutdown", "Stripe", "apply_stripe", "stripe_for"]
