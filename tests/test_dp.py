"""Data-parallel path, world_size 2.

CPU (gloo): the bucketed, backward-overlapped all-reduce of the flat gradient buffer
(GradBuckets) sums every bucket exactly once, whatever order parameters become ready in.
GPU (gloo on one device, two processes): a Trainer step sharded over 2 ranks produces the
same summed gradient as one process running both shards with the global denominators
(the equivalence SURVEY.md §8e asks for; per-rank BatchNorm on both sides).
"""
import importlib
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _FakeArena:
    def __init__(self, sizes):
        self.params = [torch.nn.Parameter(torch.zeros(n)) for n in sizes]
        self.offsets, n = [], 0
        for p in self.params:
            self.offsets.append(n)
            n += (p.numel() + 3) // 4 * 4
        self.grad = torch.zeros(n)


def _bucket_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tr = importlib.import_module("mid-attribute-speaker-generation_amd.train")
    sizes = [7, 1000, 33, 5000, 12, 4096, 3]
    arena = _FakeArena(sizes)
    gb = tr.GradBuckets(arena, bucket_bytes=16 << 10)
    for step in range(2):
        for p, o in zip(arena.params, arena.offsets):
            arena.grad[o:o + p.numel()] = (rank + 1) * (step + 1) * torch.arange(p.numel()).float()
        order = list(range(len(sizes)))
        if rank == 1:
            order = order[::-1]  # completion order may differ across ranks within a step
        for i in order:
            gb.ready([arena.params[i]])
        gb.finish()
        torch.save(arena.grad.clone(), f"{out}/r{rank}_s{step}.pt")
    dist.destroy_process_group()


def test_grad_buckets_gloo_cpu():
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_bucket_worker, args=(2, _port(), out), nprocs=2, join=True)
        for step in range(2):
            g0, g1 = torch.load(f"{out}/r0_s{step}.pt"), torch.load(f"{out}/r1_s{step}.pt")
            assert torch.equal(g0, g1)
            arena = _FakeArena([7, 1000, 33, 5000, 12, 4096, 3])
            for p, o in zip(arena.params, arena.offsets):
                want = 3 * (step + 1) * torch.arange(p.numel()).float()
                assert torch.equal(g0[o:o + p.numel()], want)


def _shard(pkg, rank, dev):
    return pkg.data.to_device(pkg.data.syn_batch(8, 32, seed=10 + rank), dev)


def _dp_worker(rank, world, port, out, backend):
    import sys
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", rank if backend == "nccl" else 0)
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    pkg = importlib.import_module("mid-attribute-speaker-generation_amd")
    M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
    tr = importlib.import_module("mid-attribute-speaker-generation_amd.train")
    pp, mc, tc, path = pkg.config.load_configs("JVS-VCTK")
    model = M.FastSpeech2(pp, mc, path, device=dev)
    pkg.seeded.load_seeded_(model)
    model.dropout = False
    model.train()
    t = tr.Trainer(model, pp, mc, tc)
    grads = []
    clip = t.opt.clip_grad_norm_

    def capture(max_norm):  # the all-reduced gradient, as Trainer.step hands it to the clip
        model.join_side()
        grads.append(model.arena().grad.detach().cpu().clone())
        return clip(max_norm)

    t.opt.clip_grad_norm_ = capture
    batch = _shard(pkg, rank, dev)
    losses = [float(t.step(batch)[0][0]) for _ in range(2)]
    torch.save({"g": grads, "loss": losses, "glob": torch.cat([t.Loss.denoms, t.eLoss.denom]).cpu(),
                "w": model.arena().flat.cpu()}, f"{out}/dp{rank}.pt")
    dist.destroy_process_group()


def _emulate(glob):
    """One process, both shards per step: global denominators, gradients accumulated, then
    the clip + Adam step of Trainer (per-shard BatchNorm, as per-rank BN)."""
    pkg = importlib.import_module("mid-attribute-speaker-generation_amd")
    M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
    tr = importlib.import_module("mid-attribute-speaker-generation_amd.train")
    pp, mc, tc, path = pkg.config.load_configs("JVS-VCTK")
    model = M.FastSpeech2(pp, mc, path, device="cuda:0")
    pkg.seeded.load_seeded_(model)
    model.dropout = False
    model.train()
    t = tr.Trainer(model, pp, mc, tc)
    glob = glob.cuda()
    t.Loss.denoms, t.eLoss.denom = glob[0:2], glob[2:3]
    shards = [_shard(pkg, r, "cuda:0") for r in range(2)]
    grads = []
    for _ in range(2):
        for b in shards:
            out_ = model(*(b[2:12]), accents=b[13], speaker_meta=b[12])
            t.Loss(b[:12], out_[:-2])[0].backward()
            (-t.eLoss(out_[-1], out_[-2])).backward()
        model.join_side()
        grads.append(model.arena().grad.detach().cpu().clone())
        t.opt.clip_grad_norm_(t.clip)
        t.opt.step_and_update_lr()
        t.opt.zero_grad()
    return grads, model.arena().flat.cpu()


def _check_dp(out):
    r0, r1 = torch.load(f"{out}/dp0.pt"), torch.load(f"{out}/dp1.pt")
    for g0, g1 in zip(r0["g"], r1["g"]):
        assert torch.equal(g0, g1)  # every rank holds the same all-reduced gradient
    assert torch.equal(r0["w"], r1["w"])
    assert float(r0["glob"][2]) == 16.0  # global batch: 2 x 8 utterances
    grads, w = _emulate(r0["glob"])
    for s, (g, ge) in enumerate(zip(r0["g"], grads)):
        scale = ge.abs().max().item()
        assert (g - ge).abs().max().item() <= 1e-5 * scale, f"step {s}"
    assert (r0["w"] - w).abs().max().item() <= 1e-6 * w.abs().max().item()


@pytest.mark.gpu
def test_data_parallel_trainer_matches_emulation():
    """Trainer.step on 2 ranks (gloo, both on cuda:0), 2 steps at SYN-8x32 per rank."""
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_dp_worker, args=(2, _port(), out, "gloo"), nprocs=2, join=True)
        _check_dp(out)


@pytest.mark.gpu
@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="RCCL needs 2 GPUs")
def test_data_parallel_trainer_nccl_matches_emulation():
    """The RCCL path (backend "nccl": GradBuckets' async all-reduces joined with the
    weight-gradient side stream), one GPU per rank."""
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_dp_worker, args=(2, _port(), out, "nccl"), nprocs=2, join=True)
        _check_dp(out)
