"""delta_compression_amd — MI355X-native batched delta codec (host mirror).

Python view of the C ABI in ``include/delta_gpu.h`` (``lib/libdeltagpu.so``).
Names and argument meanings follow the reference's interface for this path:

* ``encode(R, V, algorithm, p, q)``  — ``delta encode`` (src/c/main.c:257-292;
  src/python/delta.py:1579-1629): CRC-64/XZ of both buffers, onepass or
  correcting differencing, placement, DLT\\x03 serialisation.
* ``encode_batch(pairs, ...)``      — the same for many pairs at once.
* ``encode_pipelined(pairs, ...)``  — host arenas in chunks, H2D / encode / D2H overlapped.
* ``EncodePlan``                    — device-resident batches (the hot path).
* ``crc64_xz(data)``                — ``delta_crc64_xz`` (src/c/delta.h:294).
* ``decode(R, delta)``              — ``delta decode`` (main.c:323-400).
* ``info(delta)``                   — ``delta info`` (main.c:402-425).
* ``diff`` / ``diff_onepass`` / ``diff_correcting``, ``place_commands``,
  ``unplace_commands``, ``encode_delta``, ``decode_delta`` — the command-list
  level of src/python/delta.py:376-999 (the differencing on the GPU, the
  container walk in the library's host code).

Everything runs on the GPU.  Importing this package without the built
library, or calling it without a visible GPU, raises — there is no CPU
fallback.
"""
from __future__ import annotations

from ._lib import (  # noqa: F401
    ALGO_CORRECTING,
    ALGO_GREEDY,
    ALGO_ONEPASS,
    BUF_CAP,
    MAX_TABLE_SIZE,
    SEED_LEN,
    TABLE_SIZE,
    AddCmd,
    Context,
    CopyCmd,
    PlacedAdd,
    PlacedCopy,
    DeltaError,
    DiffOptions,
    EncodePlan,
    DecodePlan,
    LIB_PATH,
    LIMIT_ONEPASS_MEMBERS,
    LIMIT_TABLE_POOL_BYTES,
    MEMBERS_AUTO,
    MEMBERS_OFF,
    MEMBERS_ON,
    crc64_xz,
    decode,
    decode_delta,
    default_context,
    diff,
    diff_correcting,
    diff_onepass,
    diff_placed,
    encode,
    encode_batch,
    encode_delta,
    encode_pipelined,
    info,
    lib,
    make_inplace,
    output_size,
    place_commands,
    status_string,
    unplace_commands,
)

__all__ = [
    "ALGO_ONEPASS", "ALGO_CORRECTING", "ALGO_GREEDY", "SEED_LEN", "TABLE_SIZE",
    "MAX_TABLE_SIZE", "BUF_CAP", "Context", "DeltaError", "DiffOptions", "EncodePlan", "DecodePlan",
    "crc64_xz", "decode", "default_context", "encode", "encode_batch", "encode_pipelined", "info", "lib",
    "make_inplace", "status_string", "LIB_PATH", "LIMIT_TABLE_POOL_BYTES",
    "LIMIT_ONEPASS_MEMBERS", "MEMBERS_AUTO", "MEMBERS_ON", "MEMBERS_OFF",
    "CopyCmd", "AddCmd", "PlacedCopy", "PlacedAdd", "diff", "diff_onepass", "diff_correcting",
    "diff_placed", "place_commands", "unplace_commands", "output_size", "encode_delta", "decode_delta",
]
