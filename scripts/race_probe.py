"""Repeat the two tests that failed once each this round (C-ABI vs per-kernel step bitwise;
stand-in collectives vs plain step) with the pitch predictor's forward on the side stream on
and off, counting failures: which schedule change, if any, they follow."""
import importlib
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
tdp = importlib.import_module("test_dp")
tpar = importlib.import_module("test_gpu_parity")
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
for va in (True, False):
    M.VA_SIDE = va
    fails = {"collective[True]": 0, "collective[False]": 0, "c_blocks[0]": 0}
    for r in range(reps):
        for name, fn in (("collective[True]", lambda: tdp.test_collective_model_step_equals_plain_step(True)),
                         ("collective[False]", lambda: tdp.test_collective_model_step_equals_plain_step(False)),
                         ("c_blocks[0]", lambda: tpar.test_c_blocks_step_bitwise(0))):
            try:
                fn()
            except AssertionError as e:
                fails[name] += 1
                print(f"VA_SIDE={va} rep {r} {name}: FAIL {str(e)[:200]}", flush=True)
        print(f"VA_SIDE={va} after rep {r}: {fails}", flush=True)
