"""Load the upstream reference's hot-path modules for golden-vector generation.

TEST INFRASTRUCTURE ONLY — used by ``make_golden.py`` in the build container
(where ``/root/reference`` exists).  Nothing in the product, the GPU tests,
``smoke()`` or ``bench.py`` imports this file.

The reference's simulator modules decorate everything with ``numba.njit`` and
``f110_env.py`` imports ``gymnasium`` and ``pyglet``; none of the three is
installed here.  We register tiny in-memory stand-ins for those *third-party*
modules (an identity ``njit``, a minimal ``gymnasium.Env``/``spaces.Box`` and
a ``pyglet.options`` dict) and then execute the reference's own source files
(``dynamic_models.py``, ``laser_models.py``, ``collision_models.py``,
``base_classes.py``, ``f110_env.py``) by file path under the package names
they import each other by (``f110_gym.envs.*``).  The reference tree is never
written to: bytecode caching is disabled before any of it is loaded.

The @njit bodies therefore run as plain Python/NumPy.  That is the same
source Numba compiles (no fastmath, no FMA contraction in either), so parity
is pinned against the reference *source*; parity against Numba's machine code
itself cannot be checked offline.
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types

REF_ROOT = os.environ.get("F110_REFERENCE_ROOT", "/root/reference")
ENVS_DIR = os.path.join(REF_ROOT, "f110_gymnasium", "gym", "f110_gym", "envs")

_loaded: dict[str, types.ModuleType] = {}


def _install_stubs() -> None:
    sys.dont_write_bytecode = True
    if "numba" not in sys.modules:
        numba = types.ModuleType("numba")

        def njit(*args, **kwargs):
            if len(args) == 1 and callable(args[0]) and not kwargs:
                return args[0]
            return lambda f: f

        numba.njit = njit
        sys.modules["numba"] = numba

    if "gymnasium" not in sys.modules:
        gym = types.ModuleType("gymnasium")

        class Env:  # minimal base: F110Env only subclasses it
            pass

        class Box:
            def __init__(self, low=None, high=None, shape=None, dtype=None):
                self.low, self.high, self.shape, self.dtype = low, high, shape, dtype

        spaces = types.ModuleType("gymnasium.spaces")
        spaces.Box = Box
        error = types.ModuleType("gymnasium.error")
        utils = types.ModuleType("gymnasium.utils")
        gym.Env = Env
        gym.spaces, gym.error, gym.utils = spaces, error, utils
        sys.modules.update({"gymnasium": gym, "gymnasium.spaces": spaces,
                            "gymnasium.error": error, "gymnasium.utils": utils})

    if "pyglet" not in sys.modules:
        pyglet = types.ModuleType("pyglet")
        pyglet.options = {}
        gl = types.ModuleType("pyglet.gl")
        pyglet.gl = gl
        sys.modules.update({"pyglet": pyglet, "pyglet.gl": gl})

    if "f110_gym" not in sys.modules or not hasattr(sys.modules["f110_gym"], "_REFLOAD"):
        pkg = types.ModuleType("f110_gym")
        pkg.__path__ = []
        pkg._REFLOAD = True
        envs = types.ModuleType("f110_gym.envs")
        envs.__path__ = []
        rendering = types.ModuleType("f110_gym.envs.rendering")
        rendering.EnvRenderer = None
        pkg.envs = envs
        sys.modules.update({"f110_gym": pkg, "f110_gym.envs": envs,
                            "f110_gym.envs.rendering": rendering})


def load(name: str) -> types.ModuleType:
    """Load ``f110_gym.envs.<name>`` from the reference tree by file path."""
    if name in _loaded:
        return _loaded[name]
    _install_stubs()
    full = f"f110_gym.envs.{name}"
    path = os.path.join(ENVS_DIR, name + ".py")
    spec = importlib.util.spec_from_file_location(full, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[full] = mod
    spec.loader.exec_module(mod)
    setattr(sys.modules["f110_gym.envs"], name, mod)
    _loaded[name] = mod
    return mod


def load_all():
    dm = load("dynamic_models")
    lm = load("laser_models")
    cm = load("collision_models")
    bc = load("base_classes")
    return dm, lm, cm, bc


def load_env():
    load_all()
    return load("f110_env")


def load_path(modname: str, relpath: str) -> types.ModuleType:
    """Load a plain-NumPy reference module outside f110_gym by file path,
    e.g. load_path("gap_follow", "rl_training/utils/gap_follow.py")."""
    if modname in _loaded:
        return _loaded[modname]
    spec = importlib.util.spec_from_file_location("_ref_" + modname, os.path.join(REF_ROOT, relpath))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    _loaded[modname] = mod
    return mod
