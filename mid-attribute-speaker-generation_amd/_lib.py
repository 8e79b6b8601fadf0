"""ctypes binding of ``csrc/libfs2hip.so`` (the C-ABI declared in ``include/fs2hip.h``).

The signatures are read from the header itself, so the binding cannot drift from the
declarations.  There is no fallback: if the library is missing or fails to load, every
kernel call raises.  ``torch`` is imported first on purpose — the library then binds to the
HIP runtime PyTorch already loaded (same SONAME), so device pointers and streams are shared.
"""
import ctypes
import os
import re

import torch  # noqa: F401  (load torch's HIP runtime before ours)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FS2HIP_LIB") or os.path.join(_HERE, "csrc", "libfs2hip.so")
HEADER = os.path.join(os.path.dirname(_HERE), "include", "fs2hip.h")
if not os.path.exists(HEADER):  # installed layout: header shipped next to csrc/
    HEADER = os.path.join(_HERE, "csrc", "fs2hip.h")

_CT = {
    "int": ctypes.c_int,
    "int64_t": ctypes.c_int64,
    "uint64_t": ctypes.c_uint64,
    "float": ctypes.c_float,
    "double": ctypes.c_double,
    "const char*": ctypes.c_char_p,
    "void*": ctypes.c_void_p,
    "void": None,
}


def parse_header(path=HEADER):
    """``{name: (restype, [argtypes])}`` for every ``fs2_*`` entry point in the header."""
    with open(path) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    out = {}
    for m in re.finditer(r"(const char\*|int64_t|int|void\*|void)\s+(fs2_\w+)\s*\(([^)]*)\)\s*;", src):
        ret, name, args = m.group(1), m.group(2), m.group(3).strip()
        argtypes = []
        if args and args != "void":
            for a in args.split(","):
                a = a.strip()
                if "*" in a:
                    argtypes.append(ctypes.c_void_p)
                else:
                    typ = a.rsplit(None, 1)[0]
                    argtypes.append(_CT[typ])
        out[name] = (_CT[ret], argtypes)
    return out


class KernelError(RuntimeError):
    pass


class _Lib:
    def __init__(self):
        self._dll = None
        self._missing = frozenset()
        self._sigs = parse_header()

    def load(self):
        if self._dll is None:
            if not os.path.exists(LIB_PATH):
                raise KernelError(
                    f"libfs2hip.so not found at {LIB_PATH}; build it with "
                    "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
            dll = ctypes.CDLL(LIB_PATH)
            override = bool(os.environ.get("FS2HIP_LIB"))
            missing = []
            for name, (res, args) in self._sigs.items():
                if override and not hasattr(dll, name):
                    missing.append(name)  # an older library selected for an A/B run
                    continue
                fn = getattr(dll, name)
                fn.restype = res
                fn.argtypes = args
            if missing:
                import warnings
                warnings.warn(f"FS2HIP_LIB={LIB_PATH} lacks {len(missing)} entry points of "
                              f"{HEADER}: {', '.join(sorted(missing))}", RuntimeWarning, stacklevel=2)
            self._missing = frozenset(missing)
            self._dll = dll
        return self._dll

    def symbols(self):
        return sorted(self._sigs)

    def __getattr__(self, name):
        if not name.startswith("fs2_"):
            raise AttributeError(name)
        dll = self.load()
        if name in self._missing:
            raise KernelError(f"{name} is not in FS2HIP_LIB={LIB_PATH} (a library built before it "
                              "was added to include/fs2hip.h)")
        fn = getattr(dll, name)
        if fn.restype is ctypes.c_int and name not in ("fs2_abi_version", "fs2_weight_prep_tile_channels",
                                                        "fs2_resblock1_supported"):
            def call(*args, _fn=fn, _name=name):
                rc = _fn(*args)
                if rc != 0:
                    raise KernelError(f"{_name} failed ({rc}): "
                                      f"{dll.fs2_last_error().decode(errors='replace')}")
                return rc
            call.__name__ = name
            setattr(self, name, call)
            return call
        setattr(self, name, fn)
        return fn


lib = _Lib()
