"""deoss_amd -- MI355X-native replacement for DeOSS ``common/hashtree`` (SHA-256 Merkle root).

The compute path is ``libdeoss_merkle.so`` (hand-written HIP for gfx950, C ABI in
``include/deoss_merkle.h``); this package is its host-side mirror of the reference Go API.
"""
from ._lib import DeossMerkleError, LIB_PATH, load_library  # noqa: F401
from .merkle import MerkleContext, PinnedBuffer  # noqa: F401
from .hashtree import (  # noqa: F401
    HashTreeContent, Init, MerkleTree, NewHashTree, NewHashTreeFromBuffer, NewHashTreesBatch, NewStream, Node,
    Stream,
)
from .sharding import ShardPlan, plan_shards  # noqa: F401
