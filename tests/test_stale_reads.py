"""Stale-read regression tests: a training step must not depend on what memory held before it.

Round 5 saw two-model bitwise tests fail intermittently, depending on what had run earlier in
the same process: a kernel read memory that nothing had written in the step, so its result
followed the allocator's history.  ``tests/stale_probe.py`` runs a step in a fresh process
with every device allocation, every workspace and the split-K scratch filled with one byte
(the library's debug allocator and ``fs2_debug_poison``); a stale read then sees that byte.
Two processes with different bytes must produce bitwise the same gradients, weights, Adam
moments, BatchNorm statistics and losses.
"""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import stale_probe  # noqa: E402


def _probe(tmp, byte, *args):
    out = os.path.join(tmp, f"p{byte}.pt")
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    r = subprocess.run([sys.executable, os.path.join(REPO, "tests", "stale_probe.py"), "--poison",
                        str(byte), "--out", out, *args], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return torch.load(out, weights_only=True)


@pytest.mark.parametrize("args", [(), ("--dtype", "f32")], ids=["bf16-c", "f32"])
def test_step_independent_of_stale_memory(tmp_path, args):
    a = _probe(str(tmp_path), 0, *args)
    b = _probe(str(tmp_path), 63, *args)
    d = stale_probe.diff(a, b)
    assert not d, "results depend on unwritten memory:\n" + "\n".join(d[:20])
