"""Loader for the TEST-ONLY device library (csrc/cit_testkit.hip ->
build/libcitadels_testkit.so): self-test kernels kept out of the product
library libcitadels_hip.so and its header (include/citadels.h)."""
import ctypes as C
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "citadels_self_play_amd", "csrc")
LIB = os.path.join(ROOT, "build", "libcitadels_testkit.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

_lib = None
vp, i32 = C.c_void_p, C.c_int
SIGS = {"citk_area_test": ([vp, vp, vp, i32, vp, i32, vp, vp], i32),
        "citk_bench_shuffle": ([i32, i32, i32, i32, vp, vp, vp], i32),
        "citk_shuffle_check": ([i32, i32, i32, vp, vp, vp, vp, vp], i32)}


def sources():
    return [os.path.join(SRC, f) for f in ("cit_testkit.hip", "cit_area_test.h", "cit_engine.h", "cit_core.h")]


def build(force=False):
    srcs = sources()
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= max(os.path.getmtime(s) for s in srcs):
        return LIB
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-O2", "-std=c++17", "-fPIC", "-shared",
                           "-ffp-contract=off", "-fno-strict-aliasing", srcs[0], "-o", LIB])
    return LIB


def lib():
    """The prebuilt library (built by __graft_entry__.build(), never on the GPU box)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError("%s is not built (run __graft_entry__.build())" % LIB)
        import torch  # noqa: F401  (one HIP runtime: torch's, as _lib.load())
        _lib = C.CDLL(LIB)
        for name, (args, res) in SIGS.items():
            fn = getattr(_lib, name)
            fn.argtypes, fn.restype = args, res
    return _lib
