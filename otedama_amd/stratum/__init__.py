"""Stratum V2 wire protocol: framing, messages, TLS (and Noise NX transport)."""
from otedama_amd.stratum.frame import (  # noqa: F401
    CHANNEL_MSG_BIT,
    DEFAULT_MAX_FRAME_SIZE,
    HEADER_SIZE,
    MAX_MESSAGE_LENGTH,
    Decoder,
    Frame,
    FrameError,
    Header,
    decode_header,
    encode_frame,
)
