"""ctypes binding of libcitadels_hip.so (include/citadels.h).

The library is built in-tree by `__graft_entry__.build()` (hipcc
--offload-arch=gfx950).  There is no CPU fallback: if the library is missing
or no GPU is visible, using the engine raises.
"""
import ctypes as C
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CIT_LIB_PATH") or os.path.join(HERE, "libcitadels_hip.so")   # override: A/B builds only
HEADER = os.path.join(os.path.dirname(HERE), "include", "citadels.h")

_lib = None

vp, i32, i64, u64 = C.c_void_p, C.c_int, C.c_int64, C.c_uint64

_SIGS = {
    "cit_abi_version": ([], i32),
    "cit_game_bytes": ([], i32),
    "cit_seer_scratch_words": ([], i32),
    "cit_layout": ([vp, i32], i32),
    "cit_mt_seed": ([vp, vp, i32, vp, i32, vp], i32),
    "cit_mt_draw": ([vp, vp, i32, i32, vp, vp], i32),
    "cit_init": ([vp, vp, vp, i32, vp, i32, vp], i32),
    "cit_get_options": ([vp, vp, vp, vp, i32, vp, i32, vp, vp], i32),
    "cit_get_options_lanes": ([vp, vp, vp, vp, i32, vp, i32, vp, vp], i32),
    "cit_random_choice": ([vp, vp, vp, i32, vp, i32, vp, vp, vp, vp], i32),
    "cit_carry_out": ([vp, vp, vp, i32, vp, vp, vp], i32),
    "cit_rollout_random": ([vp, vp, vp, vp, i32, i32, i32, vp, vp, vp], i32),
    "cit_rollout_queue": ([vp, vp, vp, vp, i32, i32, i32, vp, vp, vp, vp], i32),
    "cit_encode_games": ([vp, i32, i32, vp, vp], i32),
    "cit_encode_options": ([vp, vp, vp, i32, vp, vp], i32),
    "cit_mlp_forward": ([vp, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp], i32),
    "cit_mlp_packed_bytes": ([], u64),
    "cit_mlp_pack": ([vp, vp, vp, vp, vp, vp, vp, vp, vp, vp], i32),
    "cit_mlp_work_bytes": ([i32], u64),
    "cit_mlp_forward_packed": ([vp, i32, vp, vp, vp, vp, u64, vp], i32),
    "cit_mlp_wave_bytes": ([], u64),
    "cit_mlp_pack_wave": ([vp, vp, vp, vp, vp, vp, vp, vp, vp, vp], i32),
    "cit_mlp_forward_wave": ([vp, i32, vp, vp, vp, vp], i32),
    "cit_cfr_pool_bytes": ([i32, i32], i64),
    "cit_cfr_arena_bytes": ([i32, i32], i64),
    "cit_cfr_block_sizes": ([vp], i32),
    "cit_cfr_arena_reset": ([vp, i32, i32, i32, i32, i32, vp], i32),
    "cit_cfr_arena_bytes_rows": ([i32, i32, i32], i64),
    "cit_cfr_arena_reset_rows": ([vp, i32, i32, i32, i32, i32, i32, vp], i32),
    "cit_cfr_arena_bytes_fmt": ([i32, i32, i32, i32], i64),
    "cit_cfr_arena_reset_fmt": ([vp, i32, i32, i32, i32, i32, i32, i32, vp], i32),
    "cit_cfr_arena_release": ([vp, i32, i32, i32, vp, i32, vp], i32),
    "cit_cfr_train_slice": ([vp, vp, vp, vp, vp, vp, i32, i32, i32, vp, vp, i32, i32, vp, vp, i64, vp, vp, vp, vp], i32),
    "cit_count_options": ([vp, vp, vp, vp, i32, vp, vp], i32),
    "cit_determinize": ([vp, vp, vp, i32, vp, i32, vp], i32),
    "cit_skip_false_choice": ([vp, vp, vp, vp, i32, vp, vp], i32),
    "cit_cfr_opt_cap": ([], i32),
    "cit_advance_random": ([vp, vp, vp, vp, i32, i32, i32, vp, vp], i32),
    "cit_cfr_decide": ([vp, vp, vp, vp, vp, vp, i32, i32, i32, vp, vp, i32, i32, vp, vp, vp, vp], i32),
    "cit_cfr_state_bytes": ([], i32),
    "cit_randbelow": ([vp, vp, i32, i32, vp, vp], i32),
    "cit_advance_policy": ([vp, vp, vp, vp, i32, i32, i32, vp, vp, vp], i32),
    "cit_random_position": ([vp, vp, vp, vp, i32, i32, vp, vp, vp], i32),
    "cit_cfr_target_count": ([vp, i32, i32, i32, vp, i32, vp, vp], i32),
    "cit_cfr_targets": ([vp, i32, i32, i32, vp, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp], i32),
    "cit_close_rows": ([], i32),
    "cit_cfr_action_choice": ([vp, i32, i32, i32, vp, vp, vp, vp, vp, vp], i32),
    "cit_close_position": ([vp, vp, vp, vp, i32, vp, vp, vp], i32),
    "cit_cfr_pred_step": ([vp, vp, vp, vp, vp, vp, i32, i32, i32, vp, i32, vp, i32, i32, vp, vp, vp, vp, vp, vp,
                           vp], i32),
    "cit_cfr_pred_slice": ([vp, vp, vp, vp, vp, vp, i32, i32, i32, vp, i32, vp, i32, i32, vp, vp, vp, vp, vp, i64,
                            vp, vp, vp], i32),
    "cit_cfr_pred_fused": ([vp, vp, vp, vp, vp, vp, i32, i32, i32, vp, i32, vp, i32, i32, vp, vp, vp, vp, vp,
                            vp], i32),
}


class NativeError(RuntimeError):
    pass


def declared_symbols():
    """Function names declared in include/citadels.h."""
    with open(HEADER) as f:
        txt = f.read()
    return sorted(set(re.findall(r"\b(?:int|int64_t)\s+(cit_\w+)\s*\(", txt)))


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeError("libcitadels_hip.so is not built (run __graft_entry__.build()); "
                          "the Citadels engine has no CPU fallback")
    # One HIP runtime per process: torch bundles its own libamdhip64.so.7, and
    # the library's NEEDED entry resolves to whichever copy is already loaded
    # (same SONAME).  Importing torch first makes that torch's copy, so device
    # pointers and streams from torch are valid in our launches.
    import torch  # noqa: F401
    lib = C.CDLL(LIB_PATH)
    for name, (args, res) in _SIGS.items():
        fn = getattr(lib, name, None)
        if fn is None and os.environ.get("CIT_LIB_PATH"):
            continue                      # an older A/B build without this entry point
        if fn is None:
            raise NativeError("%s does not export %s (stale build?)" % (LIB_PATH, name))
        fn.argtypes = args
        fn.restype = res
    _lib = lib
    return lib


def check(rc, what):
    if rc != 0:
        raise NativeError("%s failed with code %d" % (what, rc))
