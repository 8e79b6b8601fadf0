"""CPU-only checks of the host side: the C-ABI library loads and binds every declared entry
point, the module tree is the reference's (state-dict names/shapes, parameter order), the
flat-arena layout is complete, and the synthetic batch generator keeps its invariants."""
import importlib
import re

import numpy as np
import pytest
import torch

from conftest import REPO
from oracle import fs2_cpu

PKG = importlib.import_module("mid-attribute-speaker-generation_amd")
LIB = importlib.import_module("mid-attribute-speaker-generation_amd._lib")
M = importlib.import_module("mid-attribute-speaker-generation_amd.model")


def test_library_exports_every_header_symbol():
    src = open(f"{REPO}/include/fs2hip.h").read()
    declared = set(re.findall(r"\b(fs2_\w+)\s*\(", re.sub(r"/\*.*?\*/", " ", src, flags=re.S)))
    sigs = LIB.parse_header()
    assert declared == set(sigs), declared ^ set(sigs)
    dll = LIB.lib.load()
    for name in declared:
        assert getattr(dll, name) is not None
    assert LIB.lib.fs2_abi_version() == 1


def test_kernel_call_without_gpu_raises():
    K = importlib.import_module("mid-attribute-speaker-generation_amd.kernels")
    with pytest.raises(RuntimeError):
        K.fill_(torch.zeros(4), 1.0)  # CPU tensor: no silent CPU fallback


def _models():
    pp, mc, tc, path = PKG.config.load_configs("JVS-VCTK")
    ours = M.FastSpeech2(pp, mc, path, device="cpu")
    ref, _ = fs2_cpu.build("JVS-VCTK", seeded=False)
    return ours, ref


def test_state_dict_and_parameter_order_match_reference():
    ours, ref = _models()
    a, b = ours.state_dict(), ref.state_dict()
    assert list(a) == list(b) and len(a) == 242
    for k in a:
        assert a[k].shape == b[k].shape, k
    assert [n for n, _ in ours.named_parameters()] == [n for n, _ in ref.named_parameters()]
    n_train = sum(p.numel() for p in ours.parameters() if p.requires_grad)
    assert n_train == 34_726_226
    torch.testing.assert_close(a["encoder.position_enc"], b["encoder.position_enc"], rtol=0, atol=0)
    torch.testing.assert_close(a["variance_adaptor.pitch_bins"], b["variance_adaptor.pitch_bins"],
                               rtol=0, atol=0)
    ours.load_state_dict(ref.state_dict())  # reference checkpoints load unchanged


def test_flat_layout_covers_parameters_and_fuses_qkv():
    ours, _ = _models()
    order = M._flat_order(ours)
    assert len(order) == len([p for p in ours.parameters() if p.requires_grad])
    blk = ours.decoder.layer_stack[0]
    o = M.fft_param_order(blk)
    a = blk.slf_attn
    ids = [id(p) for p in o]
    i = ids.index(id(a.w_qs.weight))
    assert ids[i:i + 6] == [id(p) for p in (a.w_qs.weight, a.w_ks.weight, a.w_vs.weight,
                                            a.w_qs.bias, a.w_ks.bias, a.w_vs.bias)]
    assert [id(p) for p in order[:4]] == [id(p) for p in M.postnet_param_order(ours.postnet)[:4]]


def test_gpu_only_model_refuses_cpu_arena():
    ours, _ = _models()
    with pytest.raises(RuntimeError):
        ours.arena()


@pytest.mark.parametrize("B,Ts,seed", [(1, 8, 0), (4, 32, 1), (48, 128, 0)])
def test_syn_batch_invariants(B, Ts, seed):
    b = PKG.data.syn_batch(B, Ts, seed=seed)
    src, mel, dur = b[4], b[7], b[11]
    assert src[0] == Ts and np.all(np.diff(src) <= 0) and src.min() >= Ts // 2
    assert np.array_equal(dur.sum(1), mel) and np.array_equal(mel, 4 * src)
    assert b[5] == Ts and b[8] == mel.max() and b[6].shape == (B, 4 * Ts, 80)
    for i in range(B):
        assert np.all(b[3][i, :src[i]] >= 1) and np.all(b[3][i, src[i]:] == 0)
        assert np.all(dur[i, src[i]:] == 0) and np.all(b[6][i, mel[i]:] == 0)
    assert np.array_equal(b[12].sum(1), np.full(B, 2.0))
    assert np.array_equal(PKG.data.syn_batch(B, Ts, seed=seed)[6], b[6])  # deterministic


def test_seeded_weights_are_name_functions():
    a = PKG.seeded.seeded_array("decoder.layer_stack.0.slf_attn.w_qs.weight", (256, 256))
    b = PKG.seeded.seeded_array("decoder.layer_stack.0.slf_attn.w_qs.weight", (256, 256))
    c = PKG.seeded.seeded_array("decoder.layer_stack.1.slf_attn.w_qs.weight", (256, 256))
    assert np.array_equal(a, b) and not np.array_equal(a, c)
    assert PKG.seeded.seeded_array("encoder.position_enc", (1, 1001, 256)) is None
    w = PKG.seeded.seeded_array("encoder.src_word_emb.weight", (429, 256))
    assert np.all(w[0] == 0)


def test_optimizer_lr_schedule_matches_reference_formula():
    for s in (1, 2, 100, 4000, 4001, 300001):
        lr = fs2_cpu.lr_at(s)
        want = 256 ** -0.5 * min(s ** -0.5, 4000 ** -1.5 * s) * (0.3 if s > 300000 else 1.0)
        assert abs(lr - want) < 1e-15
    assert abs(fs2_cpu.lr_at(1) - 2.4705e-7) < 1e-10


def _bench(*argv, env=None):
    import json
    import os
    import subprocess
    import sys
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    r = subprocess.run([sys.executable, f"{REPO}/bench.py", *argv], capture_output=True,
                       text=True, timeout=300, env=e)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    return r.returncode, (json.loads(lines[-1]) if lines else None), r.stderr


def test_bench_launcher_starts_n_ranks():
    """bench.py --gpus 2 with no launcher spawns two rank processes (gloo probe on CPU)."""
    rc, out, err = _bench("--gpus", "2", "--launch-check")
    assert rc == 0, err
    assert out == {"world": 2, "ranks_seen": 2, "parallelism": "dp2"}


def test_bench_rejects_world_size_mismatch():
    rc, out, err = _bench("--gpus", "4", "--launch-check",
                          env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc == 2 and out is None and "WORLD_SIZE=2" in err


def test_jsut_config_shapes():
    """BASELINE config 1 (config/JSUT/model.yaml:42-43): one speaker, one GMM component,
    gender-only metadata (width 2); the synthetic batch follows the config."""
    pp, mc, tc, path = PKG.config.load_configs("JSUT")
    ours = M.FastSpeech2(pp, mc, path, device="cpu")
    sd = ours.state_dict()
    assert sd["speaker_emb.weight"].shape == (1, 256)
    assert sd["speaker_enc.pi_linear.0.weight"].shape == (1, 2)
    assert sd["speaker_enc.sigma_linear.0.weight"].shape == (256, 2)
    ref, _ = fs2_cpu.build("JSUT", seeded=False)
    assert {k: tuple(v.shape) for k, v in ref.state_dict().items()} == \
        {k: tuple(v.shape) for k, v in sd.items()}
    b = PKG.data.syn_batch_for("JSUT", 4, 128, seed=0)
    assert b[12].shape == (4, 2) and np.all(b[2] == 0) and np.all(b[12].sum(1) == 1)
