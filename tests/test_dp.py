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


def _dp_worker(rank, world, port, out):
    import sys
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pkg = importlib.import_module("mid-attribute-speaker-generation_amd")
    M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
    tr = importlib.import_module("mid-attribute-speaker-generation_amd.train")
    pp, mc, tc, path = pkg.config.load_configs("JVS-VCTK")
    model = M.FastSpeech2(pp, mc, path, device="cuda:0")
    pkg.seeded.load_seeded_(model)
    model.dropout = False
    model.train()
    t = tr.Trainer(model, pp, mc, tc)
    batch = pkg.data.to_device(pkg.data.syn_batch(3, 16, seed=10 + rank), "cuda:0")
    captured = {}

    def capture():
        t.buckets.finish()
        captured["g"] = model.arena().grad.detach().cpu().clone()

    glob = t._global_denominators(batch)
    t.Loss.denoms, t.eLoss.denom = glob[0:2], glob[2:3]
    losses, eloss, _, _ = tr.train_step(model, t.opt, t.Loss, t.eLoss, batch, t.clip, grad_sync=capture)
    torch.save({"g": captured["g"], "loss": float(losses[0]), "glob": glob.cpu()},
               f"{out}/dp{rank}.pt")
    dist.destroy_process_group()


@pytest.mark.gpu
def test_data_parallel_trainer_matches_emulation():
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_dp_worker, args=(2, _port(), out), nprocs=2, join=True)
        r0, r1 = torch.load(f"{out}/dp0.pt"), torch.load(f"{out}/dp1.pt")
        assert torch.equal(r0["g"], r1["g"])
        # one process: both shards with the global denominators, gradients accumulated
        pkg = importlib.import_module("mid-attribute-speaker-generation_amd")
        M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
        tr = importlib.import_module("mid-attribute-speaker-generation_amd.train")
        pp, mc, tc, path = pkg.config.load_configs("JVS-VCTK")
        model = M.FastSpeech2(pp, mc, path, device="cuda:0")
        pkg.seeded.load_seeded_(model)
        model.dropout = False
        model.train()
        t = tr.Trainer(model, pp, mc, tc)
        glob = r0["glob"].cuda()
        t.Loss.denoms, t.eLoss.denom = glob[0:2], glob[2:3]
        for r in range(2):
            b = pkg.data.to_device(pkg.data.syn_batch(3, 16, seed=10 + r), "cuda:0")
            out_ = model(*(b[2:12]), accents=b[13], speaker_meta=b[12])
            t.Loss(b[:12], out_[:-2])[0].backward()
            (-t.eLoss(out_[-1], out_[-2])).backward()
        g = model.arena().grad.detach().cpu()
        scale = g.abs().max().item()
        assert (g - r0["g"]).abs().max().item() <= 1e-5 * scale
        assert np.isclose(float(glob[2]), 6.0)
