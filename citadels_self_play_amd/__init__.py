"""MI355X-native Citadels self-play engine.

The rules engine (Agent.get_options / option.carry_out of the reference
davpat108/CITADELS_self_play) and the MCCFR search (algorithms/deep_mccfr.py)
run as hand-written HIP kernels over packed game rows and node pools
resident in HBM; this package is the host side:

* `_lib`      - ctypes loader of libcitadels_hip.so (include/citadels.h);
* `engine`    - `GameBatch`, the batched API (B games as device tensors);
* `api`       - the reference's object API (`Game`, `Agent`, `Option`,
                `CFRNode`, the run_utils functions) over single device lanes;
* `selfplay`  - one-process-per-GPU drivers (configs 3-5, RCCL pooling);
* `models` / `train` - ValueOnlyNN and its trainer;
* `train_from_scratch`, `compare_to_random`, `generate_test_data` - the
  reference's entry points.

Importing the package does not touch the GPU; the native library is loaded
on first use and its absence is an error (there is no CPU fallback).
"""

__all__ = ["layout", "rules", "canon"]
