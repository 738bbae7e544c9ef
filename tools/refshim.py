"""Import harness for the read-only reference (TEST INFRASTRUCTURE, container only).

The reference (priban42/quad-swarm-rl-stable-baselines3, mounted at /root/reference) needs
numba, gymnasium, cv2, bezier, pyglet and sample_factory, none of which exist in this image.
This module writes minimal stand-ins for those *third-party* packages into a temp directory
and puts it (plus /root/reference) on sys.path, so the reference's own Python code can run
as the golden-vector generator.  Nothing here is shipped; nothing here runs on the GPU box.

Stand-in semantics:
  * numba: njit/jit/vectorize/jitclass/overload are identity decorators, so the @njit kernels
    run as plain NumPy.  numba's RNG is replaced by NumPy's global RNG (numba.random = np.random).
  * gymnasium: Env/Wrapper base classes, spaces.Box, utils.seeding.np_random.
  * cv2, bezier: empty modules.  sample_factory.utils.utils.experiment_dir: stub.
  * gym_art.quadrotor_multi.quadrotor_multi_visualization: stub (pyglet/OpenGL).
"""
import os
import sys
import tempfile
import textwrap

REF_ROOT = os.environ.get("QS_REFERENCE_ROOT", "/root/reference")

_SHIMS = {
    "numba/__init__.py": """
        import numpy as _np
        def _ident_deco(*a, **k):
            if len(a) == 1 and callable(a[0]) and not k:
                return a[0]
            return lambda f: f
        njit = jit = vectorize = guvectorize = _ident_deco
        class _T:
            def __getattr__(self, n): return self
            def __getitem__(self, k): return self
            def __call__(self, *a, **k): return self
        types = _T(); int32 = int64 = float32 = float64 = double = boolean = _T()
        random = _np.random
        prange = range
    """,
    "numba/core/__init__.py": "",
    "numba/core/errors.py": "class TypingError(Exception):\n    pass\n",
    "numba/extending.py": """
        def overload(*a, **k):
            return lambda f: f
    """,
    "numba/experimental/__init__.py": """
        def jitclass(*a, **k):
            if len(a) == 1 and isinstance(a[0], type):
                return a[0]
            return lambda c: c
    """,
    "gymnasium/__init__.py": """
        from . import spaces, utils
        class Env:
            metadata = {}
            def __init__(self, *a, **k): pass
            def close(self): pass
            @property
            def unwrapped(self): return self
        class Wrapper(Env):
            def __init__(self, env):
                self.env = env
            def __getattr__(self, n):
                return getattr(self.env, n)
            @property
            def unwrapped(self): return self.env.unwrapped
    """,
    "gymnasium/spaces.py": """
        import numpy as _np
        class Space: pass
        class Box(Space):
            def __init__(self, low, high, shape=None, dtype=_np.float32):
                low = _np.asarray(low, dtype=_np.float64); high = _np.asarray(high, dtype=_np.float64)
                if shape is not None:
                    low = _np.broadcast_to(low, shape).copy(); high = _np.broadcast_to(high, shape).copy()
                self.low = low.astype(dtype); self.high = high.astype(dtype)
                self.shape = self.low.shape; self.dtype = _np.dtype(dtype)
            def sample(self):
                return _np.random.uniform(self.low, self.high).astype(self.dtype)
        class Dict(Space): pass
        class Tuple(Space): pass
        class Discrete(Space):
            def __init__(self, n): self.n = n
    """,
    "gymnasium/utils/__init__.py": "from . import seeding\n",
    "gymnasium/utils/seeding.py": """
        import numpy as _np
        def np_random(seed=None):
            return _np.random.default_rng(seed), seed
    """,
    "cv2/__init__.py": "",
    "bezier/__init__.py": "",
    "sample_factory/__init__.py": "",
    "sample_factory/utils/__init__.py": "",
    "sample_factory/utils/utils.py": "def experiment_dir(cfg=None, **k):\n    return '/tmp'\n",
}

_installed = None


def install():
    """Write the stand-ins once per process and make the reference importable."""
    global _installed
    if _installed is not None:
        return _installed
    if not os.path.isdir(REF_ROOT):
        raise RuntimeError(f"reference not found at {REF_ROOT}")
    d = tempfile.mkdtemp(prefix="qs_refshim_")
    for rel, src in _SHIMS.items():
        p = os.path.join(d, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(textwrap.dedent(src))
    sys.path.insert(0, d)
    sys.path.insert(1, REF_ROOT)
    import types
    viz = types.ModuleType("gym_art.quadrotor_multi.quadrotor_multi_visualization")
    viz.Quadrotor3DSceneMulti = object
    sys.modules[viz.__name__] = viz
    _installed = d
    return d
