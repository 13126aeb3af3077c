"""PoW algorithm families and header / target math."""
from otedama_amd.models.algorithms import ALGORITHMS, PowAlgorithm, get
from otedama_amd.models.header import (
    DIFF1_TARGET_INT,
    Header,
    TargetError,
    difficulty_from_target,
    hash_header,
    less_or_equal,
    meets_target,
    nbits_from_target,
    sha256d,
    target_from_difficulty,
    target_from_nbits,
)

__all__ = [
    "ALGORITHMS", "PowAlgorithm", "get", "DIFF1_TARGET_INT", "Header", "TargetError", "difficulty_from_target",
    "hash_header", "less_or_equal", "meets_target", "nbits_from_target", "sha256d", "target_from_difficulty",
    "target_from_nbits",
]
