"""vds_amd -- MI355X-native object-chunk erasure codec of lboss75/vds kernel/vds_data.

The hot path (chunk_generator::write / chunk_restore::restore over GF(2^16))
runs as hand-written gfx950 HIP kernels behind the C ABI in include/vds_ec.h;
this package is the Python host mirror of the reference's API.
"""
from ._lib import VdsEcError, device_count
from .chunk import (ChunkGenerator, ChunkRestore, ChunkStorage, chunk_cells, encode_device,
                    encode_host_batch, fill_splitmix_device, inverse, multipliers, replica_size,
                    restore_device, restore_host_batch)

__all__ = [
    "ChunkGenerator", "ChunkRestore", "ChunkStorage", "chunk_cells", "encode_device", "restore_device",
    "fill_splitmix_device", "encode_host_batch", "restore_host_batch", "inverse", "multipliers", "replica_size", "VdsEcError",
    "device_count",
]
