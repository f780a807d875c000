"""MI355X-native Citadels self-play engine.

The rules engine (Agent.get_options / option.carry_out of the reference
davpat108/CITADELS_self_play) runs as hand-written HIP kernels over packed
game rows resident in HBM; this package is the host side: the C-ABI loader
(`_lib`), the batched API (`engine.GameBatch`) and the reference-shaped
facade (`game.Game`, `game.Agent`, `game.option`).

Importing the package does not touch the GPU; the native library is loaded
on first use and its absence is an error (there is no CPU fallback).
"""

__all__ = ["layout", "rules", "canon"]
