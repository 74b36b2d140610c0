"""foundationdb_amd — MI355X-native MVCC conflict resolution (FoundationDB resolver hot path).

The product is the HIP engine libfdbcs.so (C-ABI: include/fdb_conflict_set.h); this package
holds its Python host mirror of fdbserver/ConflictSet.h, batch packing, workload generators
and key-range sharding across GPUs.
"""
from .packing import CommitTransaction, KeyRange, PackedBatch, single_key_range  # noqa: F401

__all__ = ["CommitTransaction", "KeyRange", "PackedBatch", "single_key_range"]
