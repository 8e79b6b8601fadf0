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
        if rank % 2 == 1:
            order = order[::-1]  # completion order may differ across ranks within a step
        for i in order:
            gb.ready([arena.params[i]])
        gb.finish()
        torch.save(arena.grad.clone(), f"{out}/r{rank}_s{step}.pt")
    dist.destroy_process_group()


def _lengths_worker(rank, world, port, out):
    import types
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pkg = importlib.import_module("mid-attribute-speaker-generation_amd")
    tr = importlib.import_module("mid-attribute-speaker-generation_amd.train")
    # the state Trainer(data_parallel) leaves on a gloo default group: _host_pg None (the
    # default group), which round 6's first version took for "no group" and skipped
    fake = types.SimpleNamespace(cm=None, _agree=True, _host_pg=None)
    b = pkg.data.to_device(pkg.data.syn_batch(8, (40, 32)[rank], seed=10 + rank), "cpu")
    got = tr.Trainer._agree_lengths(fake, b)
    torch.save([x for x in got[2:] if torch.is_tensor(x) or isinstance(x, int)], f"{out}/len{rank}.pt")
    dist.destroy_process_group()


def test_data_parallel_shard_lengths_agree_gloo_cpu():
    """Trainer._agree_lengths on 2 gloo ranks (CPU): shards of 40 / 32 phonemes (160 / 128
    frames) both come out padded to the global maxima, as DataParallel replicas of the
    reference's collated batch are (dataset.py:133-140, train.py:67-68); the longer shard is
    unchanged."""
    pkg = importlib.import_module("mid-attribute-speaker-generation_amd")
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_lengths_worker, args=(2, _port(), out), nprocs=2, join=True)
        for rank, ts in enumerate((40, 32)):
            got = torch.load(f"{out}/len{rank}.pt")
            want = pkg.data.to_device(_pad_np(pkg.data.syn_batch(8, ts, seed=10 + rank), 40, 160), "cpu")
            want = [x for x in want[2:] if torch.is_tensor(x) or isinstance(x, int)]
            assert len(got) == len(want)
            for g, w in zip(got, want):
                assert (g == w) if isinstance(w, int) else (g.shape == w.shape and torch.equal(g, w))


@pytest.mark.parametrize("world", [2, 4])
def test_grad_buckets_gloo_cpu(world):
    """GradBuckets on `world` gloo ranks (CPU): every rank ends each step with the sum of the
    ranks' gradients, whatever order its parameters became ready in (odd ranks reverse it)."""
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_bucket_worker, args=(world, _port(), out), nprocs=world, join=True)
        for step in range(2):
            gs = [torch.load(f"{out}/r{r}_s{step}.pt") for r in range(world)]
            for g in gs[1:]:
                assert torch.equal(gs[0], g)
            arena = _FakeArena([7, 1000, 33, 5000, 12, 4096, 3])
            scale = world * (world + 1) // 2  # sum over ranks of (rank + 1)
            for p, o in zip(arena.params, arena.offsets):
                want = scale * (step + 1) * torch.arange(p.numel()).float()
                assert torch.equal(gs[0][o:o + p.numel()], want)


def _shard(pkg, rank, dev, micro=0):
    return pkg.data.to_device(pkg.data.syn_batch(8, 32, seed=10 + rank + 2 * micro), dev)


def _dp_worker(rank, world, port, out, backend, acc=1):
    import sys
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", rank if backend == "nccl" else 0)
    torch.cuda.set_device(dev)
    if backend == "nccl":
        importlib.import_module("mid-attribute-speaker-generation_amd.train").init_data_parallel(
            dev, rank=rank, world_size=world)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    pkg = importlib.import_module("mid-attribute-speaker-generation_amd")
    M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
    tr = importlib.import_module("mid-attribute-speaker-generation_amd.train")
    pp, mc, tc, path = pkg.config.load_configs("JVS-VCTK")
    tc["optimizer"]["grad_acc_step"] = acc
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
    # bucket launches against the backward's progress: the decoder backward's end is logged
    # next to the launched bucket indices
    log = t.buckets.log = []
    dec_bwd = M.DecoderFn.backward

    def traced(fctx, *a):
        r = dec_bwd(fctx, *a)
        log.append("decoder_bwd_end")
        return r

    M.DecoderFn.backward = staticmethod(traced)
    losses, globs = [], []
    for _ in range(2):
        for m in range(acc):
            losses.append(float(t.step(_shard(pkg, rank, dev, m))[0][0]))
            globs.append(torch.cat([t.Loss.denoms, t.eLoss.denom]).cpu())
    torch.save({"g": grads, "loss": losses, "glob": globs, "log": log,
                "w": model.arena().flat.cpu()}, f"{out}/dp{rank}.pt")
    dist.destroy_process_group()


def _emulate(globs, acc=1):
    """One process, both shards per step: global denominators, gradients accumulated (over the
    shards and, with grad_acc_step = acc, over the micro-batches with the losses divided by
    acc, train.py:159,165), then the clip + Adam step of Trainer (per-shard BatchNorm, as
    per-rank BN)."""
    pkg = importlib.import_module("mid-attribute-speaker-generation_amd")
    M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
    tr = importlib.import_module("mid-attribute-speaker-generation_amd.train")
    pp, mc, tc, path = pkg.config.load_configs("JVS-VCTK")
    model = M.FastSpeech2(pp, mc, path, device="cuda:0")
    pkg.seeded.load_seeded_(model)
    model.dropout = False
    model.train()
    t = tr.Trainer(model, pp, mc, tc)
    shards = [[_shard(pkg, r, "cuda:0", m) for r in range(2)] for m in range(acc)]
    grads = []
    arena = model.arena()
    for _ in range(2):
        # each rank's micro-batches accumulate in its own buffer, then the two buffers are
        # summed: the fp32 addition order of the ranks' local accumulation + the all-reduce
        per_rank = []
        for r in range(2):
            for m in range(acc):
                glob = globs[m].cuda()
                t.Loss.denoms, t.eLoss.denom = glob[0:2], glob[2:3]
                b = shards[m][r]
                out_ = model(*(b[2:12]), accents=b[13], speaker_meta=b[12])
                loss = t.Loss(b[:12], out_[:-2])[0]
                (loss / acc if acc != 1 else loss).backward()
                el = -t.eLoss(out_[-1], out_[-2])
                (el / acc if acc != 1 else el).backward()
            model.join_side()
            per_rank.append(arena.grad.clone())
            t.opt.zero_grad()
        with torch.no_grad():
            arena.grad.copy_(per_rank[0] + per_rank[1])
        grads.append(model.arena().grad.detach().cpu().clone())
        t.opt.clip_grad_norm_(t.clip)
        t.opt.step_and_update_lr()
        t.opt.zero_grad()
    return grads, model.arena().flat.cpu()


def _check_dp(out, acc=1):
    r0, r1 = torch.load(f"{out}/dp0.pt"), torch.load(f"{out}/dp1.pt")
    assert len(r0["g"]) == 2  # the optimiser stepped twice (every acc-th batch)
    for g0, g1 in zip(r0["g"], r1["g"]):
        assert torch.equal(g0, g1)  # every rank holds the same all-reduced gradient
    assert torch.equal(r0["w"], r1["w"])
    assert float(r0["glob"][0][2]) == 16.0  # global batch: 2 x 8 utterances
    # overlap: the first bucket (PostNet, mel head, the last decoder blocks) is all-reduced
    # while the decoder backward is still being issued, on every optimiser step
    log = r0["log"]
    ends = [i for i, e in enumerate(log) if e == "decoder_bwd_end"]
    starts = [i for i, e in enumerate(log) if e == 0]
    assert len(starts) == 2 and len(ends) == 2 * acc
    for i, st in enumerate(starts):
        # the decoder backward of the stepping micro-batch (index (i + 1) acc - 1) has not
        # ended yet when bucket 0 goes out
        assert sum(e < st for e in ends) == (i + 1) * acc - 1, log
    grads, w = _emulate(r0["glob"][:acc], acc)
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
def test_data_parallel_grad_accumulation_matches_emulation():
    """grad_acc_step = 2 on 2 ranks (gloo, both on cuda:0), 2 optimiser steps: the bucket hook
    is off on the micro-batch that does not step and the accumulated buffer is all-reduced
    during the backward of the one that does; both ranks hold the same gradient, equal to one
    process accumulating every shard and micro-batch with the losses / 2."""
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_dp_worker, args=(2, _port(), out, "gloo", 2), nprocs=2, join=True)
        _check_dp(out, acc=2)


@pytest.mark.gpu
@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="RCCL needs 2 GPUs")
def test_data_parallel_trainer_nccl_matches_emulation():
    """The RCCL path (backend "nccl": GradBuckets' async all-reduces joined with the
    weight-gradient side stream), one GPU per rank."""
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_dp_worker, args=(2, _port(), out, "nccl"), nprocs=2, join=True)
        _check_dp(out)


def _nccl_one_rank_worker(rank, port, out):
    """One rank on a one-member RCCL group with the data-parallel step forced on, against a
    plain Trainer on the same GPU and batches."""
    import sys
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    importlib.import_module("mid-attribute-speaker-generation_amd.train").init_data_parallel(
        dev, rank=0, world_size=1)
    pkg = importlib.import_module("mid-attribute-speaker-generation_amd")
    M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
    tr = importlib.import_module("mid-attribute-speaker-generation_amd.train")
    pp, mc, tc, path = pkg.config.load_configs("JVS-VCTK")
    res = {}
    for dp in (True, False):
        model = M.FastSpeech2(pp, mc, path, device=dev)
        pkg.seeded.load_seeded_(model)
        model.dropout = False
        model.train()
        t = tr.Trainer(model, pp, mc, tc, data_parallel=dp)
        if dp:
            assert t.buckets is not None
            t.buckets.log = []
        losses = []
        for s in range(2):
            losses.append([float(x) for x in t.step(_shard(pkg, 0, dev, s))[0]])
        torch.cuda.synchronize()
        res[dp] = {"loss": losses, "w": model.arena().flat.cpu(),
                   "log": list(t.buckets.log) if dp else None}
    torch.save(res, f"{out}/nccl1.pt")
    dist.destroy_process_group()


@pytest.mark.gpu
def test_data_parallel_rccl_one_rank_matches_plain_step():
    """The RCCL code path on the one-GPU pool: a one-member "nccl" group with
    Trainer(data_parallel=True) -- rank-0 weight broadcast, device-side global denominators
    all-reduced, every gradient bucket all-reduced asynchronously from the weight-gradient stream
    against events of the compute streams, joined before the clip -- over 2 optimiser steps
    equals the plain single-process step (losses and weights to fp32 rounding)."""
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_nccl_one_rank_worker, args=(_port(), out), nprocs=1, join=True)
        r = torch.load(f"{out}/nccl1.pt")
    dp, plain = r[True], r[False]
    assert sorted(set(dp["log"])) == list(range(max(dp["log"]) + 1))  # every bucket went out
    for a_, b_ in zip(dp["loss"], plain["loss"]):
        for x, y in zip(a_, b_):
            assert abs(x - y) <= 1e-5 * max(abs(y), 1e-6), (a_, b_)
    w, wp = dp["w"], plain["w"]
    assert (w - wp).abs().max().item() <= 1e-6 * wp.abs().max().item()


def test_stream_reservation_check_host_logic():
    """stream_reservation_problem (the check Trainer(data_parallel=True) runs): no complaint on
    CPU devices; a CUDA device whose weight-gradient stream was never reserved, or reserved only
    after the process group existed, is reported; reserved before it, accepted.  The module's
    bookkeeping is driven directly (no GPU call)."""
    M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
    assert M.stream_reservation_problem("cpu") is None
    saved = dict(M._RESERVED_SIDE), dict(M._RESERVED_BEFORE_PG)
    try:
        M._RESERVED_SIDE.pop(7, None)
        M._RESERVED_BEFORE_PG.pop(7, None)
        msg = M.stream_reservation_problem(torch.device("cuda", 7))
        assert msg is not None and "not reserved" in msg and "init_data_parallel" in msg
        M._RESERVED_SIDE[7] = object()
        M._RESERVED_BEFORE_PG[7] = False
        msg = M.stream_reservation_problem(torch.device("cuda", 7))
        assert msg is not None and "after the process group" in msg
        M._RESERVED_BEFORE_PG[7] = True
        assert M.stream_reservation_problem(torch.device("cuda", 7)) is None
    finally:
        M._RESERVED_SIDE.clear()
        M._RESERVED_SIDE.update(saved[0])
        M._RESERVED_BEFORE_PG.clear()
        M._RESERVED_BEFORE_PG.update(saved[1])


def _unreserved_worker(rank, port, out):
    """A one-member RCCL group created with dist.init_process_group directly (the reference's
    call, train.py:67-68), no stream reservation: Trainer(data_parallel=True) must warn, and
    raise under FS2_DP_STRICT=1."""
    import sys
    import warnings
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    pkg = importlib.import_module("mid-attribute-speaker-generation_amd")
    M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
    tr = importlib.import_module("mid-attribute-speaker-generation_amd.train")
    pp, mc, tc, path = pkg.config.load_configs("JVS-VCTK")
    model = M.FastSpeech2(pp, mc, path, device=dev)
    res = {}
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        tr.Trainer(model, pp, mc, tc, data_parallel=True)
    res["warned"] = [str(x.message) for x in w if issubclass(x.category, RuntimeWarning)]
    os.environ["FS2_DP_STRICT"] = "1"
    try:
        tr.Trainer(model, pp, mc, tc, data_parallel=True)
        res["raised"] = None
    except RuntimeError as e:
        res["raised"] = str(e)
    torch.save(res, f"{out}/unres.pt")
    dist.destroy_process_group()


@pytest.mark.gpu
def test_data_parallel_warns_without_stream_reservation():
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_unreserved_worker, args=(_port(), out), nprocs=1, join=True)
        r = torch.load(f"{out}/unres.pt")
    assert any("not reserved" in m for m in r["warned"]), r
    assert r["raised"] is not None and "not reserved" in r["raised"], r


@pytest.mark.gpu
@pytest.mark.parametrize("comm", [False, True])
def test_collective_model_step_equals_plain_step(comm):
    """train.CollectiveModel (the one-GPU pricing of the N-rank collective schedule,
    scripts/dp_collective_model.py): the data-parallel step with every bucket's all-reduce and the
    denominators' all-reduce replaced by fs2_collective_standin -- issued from the weight-gradient
    stream (comm=False) or a stream of its own (comm=True) -- leaves the gradients unchanged, so
    two optimiser steps equal the plain step (to the fp32 rounding of the device-side loss
    denominators, as in the one-rank RCCL test); every bucket is issued once per step."""
    import sys
    sys.path.insert(0, REPO)
    pkg = importlib.import_module("mid-attribute-speaker-generation_amd")
    M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
    tr = importlib.import_module("mid-attribute-speaker-generation_amd.train")
    dev = torch.device("cuda", 0)
    pp, mc, tc, path = pkg.config.load_configs("JVS-VCTK")
    res = {}
    for mode in ("plain", "model"):
        torch.manual_seed(0)
        model = M.FastSpeech2(pp, mc, path, device=dev, compute_dtype=torch.bfloat16)
        model.train()
        model.dropout = False
        if mode == "plain":
            t = tr.Trainer(model, pp, mc, tc)
        else:
            t = tr.Trainer(model, pp, mc, tc, collective_model=tr.CollectiveModel(
                ranks=8, busbw_gbs=300.0, blocks=8, latency_us=5.0), bucket_bytes=16 << 20,
                comm_stream=comm)
            t.buckets.log = []
        losses = [[float(x) for x in t.step(_shard(pkg, 0, dev, s))[0]] for s in range(2)]
        torch.cuda.synchronize()
        res[mode] = (losses, model.arena().flat.cpu(),
                     list(t.buckets.log) if t.buckets is not None else None)
    for a_, b_ in zip(res["model"][0], res["plain"][0]):
        for x, y in zip(a_, b_):
            assert abs(x - y) <= 1e-5 * max(abs(y), 1e-6), (a_, b_)
    w, wp = res["model"][1], res["plain"][1]
    assert (w - wp).abs().max().item() <= 1e-6 * wp.abs().max().item()
    nb = len(t.buckets.sizes)
    assert sorted(res["model"][2]) == sorted(list(range(nb)) * 2)


_CLF_PERM = [5, 12, 0, 9, 3, 14, 7, 1, 10, 2, 15, 6, 11, 4, 13, 8]  # the global batch of 2 x 8


def _clf_pair(dev):
    G = importlib.import_module("mid-attribute-speaker-generation_amd.ge2e")
    pkg = importlib.import_module("mid-attribute-speaker-generation_amd")
    d = G.SpeechEmbedder(device=dev)
    pkg.seeded.load_seeded_(d)
    d.da_dropout = 0.0
    return d, G.GE2ELoss(dev)


def _pad_np(b, ts, tm):
    """A numpy syn_batch padded on the right to ts phonemes / tm frames with zeros (the global
    batch's collate, dataset.py:133-140) -- independent of data.pad_batch."""
    b = list(b)
    ds, dm = ts - b[5], tm - b[8]
    for i in (3, 9, 10, 11, 13):
        b[i] = np.pad(b[i], ((0, 0), (0, ds)))
    b[6] = np.pad(b[6], ((0, 0), (0, dm), (0, 0)))
    b[5], b[8] = ts, tm
    return tuple(b)


def _clf_shard(pkg, rank, dev, ts=None, pad=False):
    """Rank's shard: the equal-length default (_shard), or syn_batch(8, ts[rank]) -- padded to
    the ranks' maxima when ``pad`` (what a replica of the reference's DataParallel receives)."""
    if ts is None:
        return _shard(pkg, rank, dev, 0)
    b = pkg.data.syn_batch(8, ts[rank], seed=10 + rank)
    if pad:
        b = _pad_np(b, max(ts), 4 * max(ts))
    return pkg.data.to_device(b, dev)


def _clf_worker(rank, world, port, out, ts=None):
    import sys
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
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
    clf = _clf_pair(dev)
    grads, globs, dl = [], [], []
    clip = t.opt.clip_grad_norm_

    def capture(max_norm):
        model.join_side()
        grads.append(model.arena().grad.detach().cpu().clone())
        return clip(max_norm)

    t.opt.clip_grad_norm_ = capture
    for s in range(2):
        r = t.step(_clf_shard(pkg, rank, dev, ts), clf=clf, clf_args=(_CLF_PERM, 4 + s, 10, 1.0))
        dl.append((float(r[4][0]), int(r[4][1]), int(r[4][2])))
        globs.append(torch.cat([t.Loss.denoms, t.eLoss.denom]).cpu())
    torch.save({"g": grads, "glob": globs, "dl": dl, "w": model.arena().flat.cpu()},
               f"{out}/clf{rank}.pt")
    dist.destroy_process_group()


def _emulate_clf(globs, ts=None):
    """One process, both shards per step, as _emulate, plus the clf branch per shard with the
    speakers / metadata of the permuted global batch and the global chunk count."""
    pkg = importlib.import_module("mid-attribute-speaker-generation_amd")
    M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
    tr = importlib.import_module("mid-attribute-speaker-generation_amd.train")
    G = importlib.import_module("mid-attribute-speaker-generation_amd.ge2e")
    pp, mc, tc, path = pkg.config.load_configs("JVS-VCTK")
    model = M.FastSpeech2(pp, mc, path, device="cuda:0")
    pkg.seeded.load_seeded_(model)
    model.dropout = False
    model.train()
    t = tr.Trainer(model, pp, mc, tc)
    disc, dLoss = _clf_pair("cuda:0")
    shards = [_clf_shard(pkg, r, "cuda:0", ts, pad=True) for r in range(2)]
    gspk = torch.cat([b[2] for b in shards])
    gmeta = torch.cat([b[12] for b in shards])
    perm = torch.as_tensor(_CLF_PERM, device="cuda:0")
    grads, dls = [], []
    arena = model.arena()
    for s in range(2):
        glob = globs[s].cuda()
        parts = []
        for r in range(2):
            t.Loss.denoms, t.eLoss.denom = glob[0:2], glob[2:3]
            b = shards[r]
            out_ = model(*(b[2:12]), accents=b[13], speaker_meta=b[12])
            t.Loss(b[:12], out_[:-2])[0].backward()
            (-t.eLoss(out_[-1], out_[-2])).backward()
            mine = perm[r * 8:(r + 1) * 8]
            meta = gmeta.index_select(0, mine)
            o2 = model(gspk.index_select(0, mine), *b[3:12], accents=b[13], speaker_meta=meta)
            chunks, rep = G.chunk_mels(o2[0])
            langs = G.chunk_langs(meta, rep)
            o_r = disc(chunks)
            _, _, dloss = dLoss(o_r["embeddings"].view(chunks.shape[0], 1, -1),
                                o_r["da_lang_logits"], langs, reduction="sum")
            parts.append((dloss, langs.shape[0]))
        n_glob = sum(n for _, n in parts)
        # the two ranks' clf losses over the global chunk count (each rank backprops its own)
        for dloss, _ in parts:
            (dloss * (G.da_coefficient(4 + s, 10) / n_glob)).backward()
        model.join_side()
        dls.append(float(sum(float(d) for d, _ in parts)))
        grads.append(arena.grad.detach().cpu().clone())
        t.opt.clip_grad_norm_(t.clip)
        t.opt.step_and_update_lr()
        t.opt.zero_grad()
    return grads, dls, arena.flat.cpu()


@pytest.mark.gpu
@pytest.mark.parametrize("ts", [None, (40, 32)])
def test_data_parallel_use_clf_matches_emulation(ts):
    """``--use_clf`` under data parallelism (Trainer.step, 2 ranks on gloo, both on cuda:0):
    the global permutation of speakers / metadata across the ranks, the global chunk count, and
    the buckets all-reduced after the clf backward give the gradients, discriminator losses
    and weights of one process running both shards (sums of per-shard gradients; the emulation
    accumulates both shards in one buffer, so fp32 summation order differs: 1e-5).
    ``ts = (40, 32)``: shards of different lengths (160 vs 128 frames, so 2 vs 1 chunks of
    150 each on their own).  The reference's DataParallel replicas all see the global batch's
    max lengths, so the emulation runs each shard padded to 40 phonemes / 160 frames -- the
    PostNet statistics, the predictors' padded rows and the chunk count (2 per utterance) all
    follow from it -- and the ranks must agree on them (Trainer._agree_lengths)."""
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_clf_worker, args=(2, _port(), out, ts), nprocs=2, join=True)
        r0, r1 = torch.load(f"{out}/clf0.pt"), torch.load(f"{out}/clf1.pt")
        for g0, g1 in zip(r0["g"], r1["g"]):
            assert torch.equal(g0, g1)
        assert r0["dl"] == r1["dl"] and r0["dl"][0][2] % 16 == 0  # 16 utterances x chunks each
        if ts is not None:
            assert r0["dl"][0][2] == 16 * (4 * max(ts) // 150 + 1)
        grads, dls, w = _emulate_clf(r0["glob"], ts)
        # step 0 from the same weights: the gradients to fp32 summation order.  Step 1 starts
        # from weights one Adam step apart, and Adam's m / sqrt(v) turns the summation-order
        # noise of near-zero gradients into updates of up to lr: looser there
        for s, (g, ge) in enumerate(zip(r0["g"], grads)):
            scale = ge.abs().max().item()
            assert (g - ge).abs().max().item() <= (1e-5 if s == 0 else 2e-3) * scale, f"step {s}"
        for (d, _, _), de in zip(r0["dl"], dls):
            assert abs(d - de) <= 1e-4 * max(abs(de), 1e-6)
        assert (r0["w"] - w).abs().max().item() <= 1e-4 * w.abs().max().item()
