"""av1dec_amd -- MI355X (gfx950) native AV1 block-reconstruction + in-loop filter backend.

Drop-in below the reference decoder's parse/reconstruct seam (oddstone/av1dec
Decoder::decodeFrame, decoder/Av1Decoder.cpp:128-192): host-parsed frame batches in,
reconstructed + deblocked + CDEF + loop-restored frames out, bit-exact with the reference.
"""
from . import abi, batchfile  # noqa: F401
from .decoder import BackendError, Decoder  # noqa: F401

__all__ = ["Decoder", "BackendError", "batchfile", "abi"]
