"""TLS transport for stratum+tls:// and stratum+v2tls:// (certificate-verified).

Parity: internal/stratum/tls.go — defaultTLSConfig (TLS >= 1.2, :34-36),
TLSConfigWithExtraCAs (system roots + PEM bundle, :44-56), DialTLS (:63-69);
internal/poolproto/stratumv1/tls.go:59-65. The reference's SV2 adapter silently
ignores TLS; here both protocols honour it.
"""
from __future__ import annotations

import asyncio
import ssl


def default_context() -> ssl.SSLContext:
    ctx = ssl.create_default_context(ssl.Purpose.SERVER_AUTH)
    ctx.minimum_version = ssl.TLSVersion.TLSv1_2
    return ctx


def context_with_extra_cas(pem: bytes | str | None) -> ssl.SSLContext:
    ctx = default_context()
    if pem:
        ctx.load_verify_locations(cadata=pem.decode() if isinstance(pem, bytes) else pem)
    return ctx


def server_context(certfile: str, keyfile: str) -> ssl.SSLContext:
    ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
    ctx.minimum_version = ssl.TLSVersion.TLSv1_2
    ctx.load_cert_chain(certfile, keyfile)
    return ctx


async def open_connection(host: str, port: int, use_tls: bool, ca_pem: bytes | None = None, timeout: float = 10.0):
    ssl_ctx = context_with_extra_cas(ca_pem) if use_tls else None
    return await asyncio.wait_for(
        asyncio.open_connection(host, port, ssl=ssl_ctx, server_hostname=host if use_tls else None,
                                limit=64 * 1024),
        timeout)
