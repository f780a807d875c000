"""Every global name the package's functions load exists (a NameError in a
GPU-only code path would otherwise surface only on the GPU box)."""
import builtins
import dis
import importlib
import os
import types

import pytest

PKG = "citadels_self_play_amd"
MODULES = sorted(f[:-3] for f in os.listdir(os.path.join(os.path.dirname(os.path.dirname(__file__)), PKG))
                 if f.endswith(".py") and f != "__init__.py")


def _codes(co):
    yield co
    for c in co.co_consts:
        if isinstance(c, types.CodeType):
            yield from _codes(c)


@pytest.mark.parametrize("name", MODULES)
def test_global_names_resolve(name):
    mod = importlib.import_module("%s.%s" % (PKG, name))
    src = open(mod.__file__).read()
    missing = set()
    for co in _codes(compile(src, mod.__file__, "exec")):
        for ins in dis.get_instructions(co):
            if ins.opname == "LOAD_GLOBAL":
                n = ins.argval
                if n not in mod.__dict__ and not hasattr(builtins, n):
                    missing.add((co.co_name, n))
    assert not missing, missing
