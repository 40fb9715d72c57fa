"""evolu_amd -- MI355X batch-merge engine for Evolu's CRDT sync hot path.

libevm.so (HIP, gfx950) implements the hot path behind the C ABI in
include/evm.h; this package is its Python host side, mirroring the
reference's function API (packages/evolu/src/{timestamp,merkleTree,
applyMessages}.ts and apps/server/src/index.ts).
"""
__all__ = ["engine", "dist", "server", "synth", "wire"]
