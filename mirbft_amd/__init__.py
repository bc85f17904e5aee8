"""mirbft_amd -- MI355X-native batched SHA-256 engine for MirBFT's hash path.

The product is ``libmirsha.so`` (C ABI: include/mirsha.h; HIP kernels in
mirbft_amd/csrc/). This package is its Python binding plus a mirror of the
reference's ``processor.Hasher`` / ``ProcessHashActions`` surface.
"""
from .engine import Engine, MshaError, blocks_for_len, device_count, pack_parts, partition_by_blocks
from .processor import (Action, ActionHashRequest, ActionList, EventHashResult, EventList, GPUHasher,
                        HashOrigin, HashOriginBatch, HashOriginEpochChange, HashOriginVerifyBatch,
                        ProcessHashActions, ProcessorError, action_hash, checkpoint_hashes)

__all__ = [
    "Engine", "MshaError", "blocks_for_len", "device_count", "pack_parts", "partition_by_blocks",
    "Action", "ActionHashRequest", "ActionList", "EventHashResult", "EventList", "GPUHasher",
    "HashOrigin", "HashOriginBatch", "HashOriginEpochChange", "HashOriginVerifyBatch",
    "ProcessHashActions", "ProcessorError", "action_hash", "checkpoint_hashes",
]
