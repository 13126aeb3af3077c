"""Pool protocols (Stratum V1 / V2 client sessions) behind one registry."""
from otedama_amd.poolproto import stratumv1, stratumv2  # noqa: F401  (register dialers)
from otedama_amd.poolproto.base import (
    Credentials,
    Dialer,
    FatalPoolError,
    HandshakeFailed,
    Job,
    PoolProtoError,
    ProtocolID,
    Session,
    ShareRejected,
    ShareResult,
    ShareSubmission,
    UnknownProtocol,
    available,
    dial_url,
    from_url,
    lookup,
    register,
    strip_scheme,
)

__all__ = [
    "Credentials", "Dialer", "FatalPoolError", "HandshakeFailed", "Job", "PoolProtoError", "ProtocolID", "Session",
    "ShareRejected", "ShareResult", "ShareSubmission", "UnknownProtocol", "available", "dial_url", "from_url",
    "lookup", "register", "strip_scheme",
]
