"""bench.py with module-level switches set first, for same-box A/B of host-side choices:

    python scripts/bench_ab.py optimizer.OVERLAP_UPDATE=0 -- [bench.py arguments]
"""
import importlib
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
i = sys.argv.index("--")
for spec in sys.argv[1:i]:
    name, val = spec.split("=")
    mod, attr = name.rsplit(".", 1)
    m = importlib.import_module("mid-attribute-speaker-generation_amd." + mod)
    setattr(m, attr, type(getattr(m, attr))(int(val)))
sys.argv = [os.path.join(sys.path[0], "bench.py")] + sys.argv[i + 1:]
runpy.run_path(sys.argv[0], run_name="__main__")
