"""Build A/B variants of one translation unit (default the rollout's,
cit_hip.hip; AB_UNIT=cit_cfr.hip for the search) with extra flags, linked
against the main build's other objects:
    python tools/ab_build.py NAME [flags...]   ->  build/ab/libNAME.so
(`tools/_ablib.py build/ab/libNAME.so` benchmarks one on the GPU box;
AB_ARGS passes bench.py arguments, e.g. "--config 3".)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as G  # noqa: E402


def build(name, extra):
    out = os.path.join(ROOT, "build", os.environ.get("ABDIR", "ab"))
    os.makedirs(out, exist_ok=True)
    o = os.path.join(out, name + ".o")
    unit = os.environ.get("AB_UNIT", "cit_hip.hip")
    flags = [f for f in G.HIP_FLAGS + G.UNIT_FLAGS.get(unit, [])
             if not (f.startswith("-O") and any(e.startswith("-O") for e in extra))]
    subprocess.check_call([G.HIPCC] + flags + extra + ["-c", os.path.join(G.CSRC, unit), "-o", o])
    others = [os.path.join(ROOT, "build", "hip", u.replace(".hip", ".o")) for u in G.HIP_UNITS if u != unit]
    lib = os.path.join(out, "lib%s.so" % name)
    subprocess.check_call([G.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", o] + others + ["-o", lib])
    return lib


if __name__ == "__main__":
    print(build(sys.argv[1], sys.argv[2:]))
