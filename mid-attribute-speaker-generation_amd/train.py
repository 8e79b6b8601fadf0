"""The training step of ``train.py:134-206`` (``grad_acc_step``, ``use_clf`` optional) and
its data-parallel form.

Single process: ``train_step`` is line-for-line the reference's step semantics
(forward, FastSpeech2Loss backward, negated speaker-prior log-likelihood backward,
clip_grad_norm_, ScheduledOptim.step_and_update_lr, zero_grad).

Data parallel: one process per GPU, batch sharded by utterance.
* Each rank normalises its masked means by the *global* valid counts and the GMM term by
  the global batch (one 3-float all-reduce of device-side counts before the forward, no host
  sync), so the summed gradient equals the 1-process gradient of the global batch.
* Gradients are all-reduced (sum) over RCCL in ~16 MB buckets of the flat fp32 gradient
  buffer.  The buffer is laid out in reverse backward order, every block's backward reports
  its parameters as final (``StepCtx.notify``), and a bucket's all-reduce is launched as soon
  as all of its parameters are final, so communication overlaps the rest of the backward.
  Each all-reduce is issued from the weight-gradient side stream after it waits on an event
  recorded on the main compute stream at launch time: the main chain never waits for a
  bucket (only the clip at the end of the step waits for them all).
* BatchNorm statistics stay per rank (DataParallel's per-replica semantics).
"""
import os
import warnings

import torch
import torch.distributed as dist

from . import kernels as K
from .loss import FastSpeech2Loss, SpeakerMetaEncLoss
from .optimizer import ScheduledOptim


def clf_backward(model, batch, clf, perm, step, total_step, lambd=1.0, group=None):
    """The ``--use_clf`` branch of ``train.py:168-197``: a second forward with the speakers
    (and their metadata) shuffled by ``perm`` (the reference draws it with
    ``random.sample``), the predicted mel cut into 150-frame chunks, the language
    discriminator on every chunk, and ``dloss * coef(step / total_step) / len(langs) *
    lambd`` back-propagated into the model.  ``clf = (SpeechEmbedder, GE2ELoss)``.  Returns
    ``(dloss, cross-lingual chunk count, chunk count)``.

    ``group`` (data parallel, equal shards): the reference shuffles its whole
    (``nn.DataParallel``) batch, so ``perm`` permutes the global batch of ``world x B``
    utterances, the same on every rank.  Every rank's speakers and metadata are all-gathered
    (B ints and B metadata rows per rank), a rank takes its rows of the shuffled global batch,
    and the loss is divided by the global chunk count (the BCE term sums over chunks, so the
    summed all-reduce of the ranks' gradients is the global batch's).  The returned dloss and
    counts are the global sums."""
    from . import ge2e
    disc, dLoss = clf
    dev = batch[2].device
    idx = torch.as_tensor(perm, device=dev)
    if group is None:
        speakers = batch[2].index_select(0, idx)  # (B,) ids: the gather of train.py:172
        meta = batch[12].index_select(0, idx)
    else:
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        B = batch[2].shape[0]
        if idx.numel() != world * B:
            raise ValueError(f"use_clf with data parallelism: perm must permute the global batch "
                             f"({world} x {B} utterances), got {idx.numel()}")
        spk = [torch.empty_like(batch[2]) for _ in range(world)]
        dist.all_gather(spk, batch[2].contiguous(), group=group)
        mt = [torch.empty_like(batch[12]) for _ in range(world)]
        dist.all_gather(mt, batch[12].contiguous(), group=group)
        mine = idx[rank * B:(rank + 1) * B]
        speakers = torch.cat(spk).index_select(0, mine)
        meta = torch.cat(mt).index_select(0, mine)
    output = model(speakers, *batch[3:12], accents=batch[13], speaker_meta=meta)
    chunks, rep = ge2e.chunk_mels(output[0])
    langs = ge2e.chunk_langs(meta, rep)
    langs_original = ge2e.chunk_langs(batch[12], rep)
    out_r = disc(chunks)
    _, _, dloss = dLoss(out_r["embeddings"].view(chunks.shape[0], 1, -1),
                        out_r["da_lang_logits"], langs, reduction="sum")
    cross = (langs != langs_original).sum()
    n = langs.shape[0]
    if group is None:
        scale = ge2e.da_coefficient(step, total_step) / n * lambd
        (dloss * scale).backward()
        return dloss, cross, n
    stats = torch.stack([torch.tensor(float(n), device=dev), cross.float(), dloss.detach()])
    dist.all_reduce(stats, group=group)  # global chunk count, cross-lingual chunks, dloss
    (dloss * (ge2e.da_coefficient(step, total_step) * lambd / stats[0])).backward()
    return stats[2], stats[1].long(), int(stats[0].item())


def train_step(model, optimizer, Loss, eLoss, batch, grad_clip_thresh=1.0, grad_sync=None,
               clf=None, clf_args=None, grad_acc_step=1, update=True, clf_group=None):
    """One batch of ``train.py:138-206`` -> (losses, eloss, grad norm, output).

    Both losses are back-propagated divided by ``grad_acc_step`` (``train.py:159,165``);
    with ``update`` (the reference's ``step % grad_acc_step == 0``, ``train.py:200``) the
    accumulated gradients are clipped, Adam steps and the gradients are zeroed, otherwise
    they stay accumulated and the grad norm is None.  With ``clf`` (and ``clf_args = (perm,
    step, total_step, lambd)``) the ``--use_clf`` branch runs between the losses' backward
    and the clip, and its ``(dloss, cross-lingual chunks, chunks)`` is appended."""
    output = model(*(batch[2:12]), accents=batch[13], speaker_meta=batch[12])
    losses = Loss(batch[:12], output[:-2])
    # The speaker-metadata GMM loss (train.py:162-166) goes first: its value depends on the
    # weights only, and its backward writes only the GMM head's gradients (the embedding enters
    # detached), disjoint from the FastSpeech2 loss's.  So the order changes no value, but the
    # GPU then never idles at the end of the long backward while the host issues the GMM
    # launches (about 0.1 ms per step measured in the kernel trace).
    eloss = eLoss(output[-1], output[-2])
    (-eloss / grad_acc_step if grad_acc_step != 1 else -eloss).backward()
    (losses[0] / grad_acc_step if grad_acc_step != 1 else losses[0]).backward()
    clf_out = clf_backward(model, batch, clf, *clf_args, group=clf_group) if clf is not None else None
    gnorm = None
    if update:
        if grad_sync is not None:
            grad_sync()
        gnorm = optimizer.clip_grad_norm_(grad_clip_thresh)
        optimizer.step_and_update_lr()
        optimizer.zero_grad()
    if clf_out is not None:
        return losses, eloss, gnorm, output, clf_out
    return losses, eloss, gnorm, output


def init_data_parallel(device, **kwargs):
    """``dist.init_process_group("nccl", ...)`` for the data-parallel step on ``device``.

    Reserves the step's compute streams first (model.reserve_streams: the RCCL communicator
    creates streams of its own at init), so the legacy stream, the weight-gradient stream and
    then ProcessGroupNCCL's collective stream take the first hardware queues.  Normal priority:
    a high-priority stream in the process made every kernel ~2x slower (21 vs 7.5 ms/step,
    profiles/r3_ab_experiments.txt).  Extra keyword arguments go to ``init_process_group``
    (rank, world_size, ...)."""
    from .model import reserve_streams
    reserve_streams(device)
    dist.init_process_group("nccl", device_id=device, **kwargs)


class CollectiveModel:
    """Stand-in collectives for pricing the data-parallel step at ``ranks`` ranks on ONE GPU
    (measurement only: ``scripts/dp_collective_model.py``, ``profiles/r5_dp_collective_model.txt``).

    A bucket's ring all-reduce of S bytes is replaced by ``fs2_collective_standin``:
    ``blocks`` workgroups (RCCL's channels) that read and write back 2 (n - 1) / n * S bytes of
    the bucket (values unchanged) over 2 (n - 1) / n * S / busbw + latency -- the collective's
    CU occupancy, HBM traffic and duration, without the interconnect.  Like ProcessGroupNCCL,
    which runs a collective on its own stream after that stream waits on the issuing stream,
    the stand-in runs on a stream of its own gated by an event of the issuing stream
    (``inline=True``: on the issuing stream itself, so later work there queues behind it).  The
    step's 3-float all-reduce of the loss denominators becomes a one-workgroup stand-in of
    ``latency_us`` on the main stream, and the denominators stay local, so the step's values are
    the single-GPU step's."""

    def __init__(self, ranks=8, busbw_gbs=300.0, blocks=32, latency_us=12.0, inline=False):
        self.ranks, self.busbw, self.blocks, self.lat = int(ranks), float(busbw_gbs), int(blocks), float(latency_us)
        self.inline = bool(inline)
        self.stream = None

    def wire_bytes(self, nbytes):
        return 2.0 * (self.ranks - 1) / self.ranks * nbytes

    def duration_ns(self, nbytes):
        return int((self.wire_bytes(nbytes) / (self.busbw * 1e9) + self.lat * 1e-6) * 1e9)

    def all_reduce(self, t):
        nb = t.numel() * t.element_size()
        if self.inline:
            K.lib.fs2_collective_standin(K.ptr(t), t.numel(), int(2 * self.wire_bytes(nb)),
                                         self.blocks, self.duration_ns(nb), K.stream())
            return
        if self.stream is None:
            self.stream = torch.cuda.Stream()
        self.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.stream):
            K.lib.fs2_collective_standin(K.ptr(t), t.numel(), int(2 * self.wire_bytes(nb)),
                                         self.blocks, self.duration_ns(nb), K.stream())

    def join(self):
        """The current stream waits for every stand-in collective issued so far (work.wait())."""
        if self.stream is not None:
            torch.cuda.current_stream().wait_stream(self.stream)

    def small(self, t):
        K.lib.fs2_collective_standin(K.ptr(t), t.numel(), 0, 1, int(self.lat * 1e3), K.stream())


class GradBuckets:
    """Bucketed, backward-overlapped all-reduce of the arena's flat gradient buffer."""

    def __init__(self, arena, group=None, bucket_bytes=16 << 20):
        self.arena, self.group = arena, group
        index = {id(p): i for i, p in enumerate(arena.params)}
        buckets, cur, size = [], [], 0
        for i, p in enumerate(arena.params):
            cur.append(i)
            size += p.numel() * 4
            if size >= bucket_bytes:
                buckets.append(cur)
                cur, size = [], 0
        if cur:
            buckets.append(cur)
        self.bucket_of = {pid: b for b, idxs in enumerate(buckets) for pid in
                          (id(arena.params[i]) for i in idxs)}
        self.ranges = []
        for idxs in buckets:
            last = idxs[-1]
            self.ranges.append((arena.offsets[idxs[0]],
                                arena.offsets[last] + arena.params[last].numel()))
        self.sizes = [len(idxs) for idxs in buckets]
        # producers of the gradients besides the current stream (the weight-gradient side
        # stream): a callable returning the streams.  A bucket's all-reduce is issued from the
        # last producer stream (the side stream, which trails the main chain), after it waits
        # on an event of the current stream.  A separate communication stream would need a
        # hardware queue of its own, and HIP shares 4 per priority among every stream of the
        # process (profiles/r3_ab_experiments.txt: separate / high-priority communication
        # streams measured 1.04-2.8x slower steps)
        self.producers = None
        self.standin = None  # a CollectiveModel: stand-in collectives (no process group)
        self.log = None  # optional list: bucket launches are appended (tests)
        del index
        self.reset()

    def reset(self):
        self.left = list(self.sizes)
        self.next = 0  # buckets launch strictly in index order (same order on every rank)
        self.works = []

    def _launch(self, b):
        s, e = self.ranges[b]
        if self.log is not None:
            self.log.append(b)
        cur = torch.cuda.current_stream() if self.arena.grad.is_cuda else None
        prods = [st for st in (self.producers() if self.producers else ()) if st is not None]
        if cur is None or not prods:
            if self.standin is not None:
                self.standin.all_reduce(self.arena.grad[s:e])
                return
            self.works.append(dist.all_reduce(self.arena.grad[s:e], group=self.group,
                                              async_op=True))
            return
        # the bucket's gradients are complete in stream order on the current stream and on
        # the producer streams: the issuing stream waits on an event of each of the others
        # (the main chain never waits for the collective or for the side stream here)
        issue = prods[-1]
        for st in [cur] + prods:
            if st is not issue:
                ev = torch.cuda.Event()
                ev.record(st)
                issue.wait_event(ev)
        self._issue = issue
        with torch.cuda.stream(issue):
            if self.standin is not None:
                self.standin.all_reduce(self.arena.grad[s:e])
            else:
                self.works.append(dist.all_reduce(self.arena.grad[s:e], group=self.group,
                                                  async_op=True))

    def ready(self, params):
        for p in params:
            self.left[self.bucket_of[id(p)]] -= 1
        while self.next < len(self.sizes) and self.left[self.next] == 0:
            self._launch(self.next)
            self.next += 1

    def finish(self):
        while self.next < len(self.sizes):  # includes parameters without a gradient this step
            self._launch(self.next)
            self.next += 1
        for w in self.works:
            w.wait()  # stream-ordered: the clip/Adam kernels queue behind the collectives
        if self.standin is not None:
            self.standin.join()
        if getattr(self, "_issue", None) is not None:
            torch.cuda.current_stream().wait_stream(self._issue)
            self._issue = None
        self.reset()


class Trainer:
    """Model + loss + optimiser for one rank (``world_size`` 1 = plain single-GPU).

    ``graph=True`` (single process): the first ``step`` runs eagerly and captures the whole
    step -- forward, both backwards, clip, Adam + schedule, zero_grad -- into one HIP graph;
    later steps copy the batch into the graph's static inputs and replay it.  Every per-step
    quantity the kernels read (dropout key, LR, Adam bias corrections, BN counters) lives in
    device memory, so a replay is exactly an eager step; the returned tensors are the graph's
    static outputs (overwritten by the next replay).  A batch of another shape re-captures.

    ``data_parallel`` (default: world size > 1) selects the data-parallel step -- global loss
    denominators, bucketed gradient all-reduce from the weight-gradient stream; forcing it on a
    one-rank group runs that code path on one GPU (tests/test_dp.py).  On the GPU it warns
    (raises with FS2_DP_STRICT=1) when the device's compute streams were not reserved before
    the process group existed (train.init_data_parallel does both in the right order).
    """

    def __init__(self, model, preprocess_config, model_config, train_config, current_step=0,
                 process_group=None, bucket_bytes=16 << 20, graph=False, data_parallel=None,
                 collective_model=None, comm_stream=False):
        self.model = model
        self.graph_mode = bool(graph)
        self._graph = None
        self.Loss = FastSpeech2Loss(preprocess_config, model_config)
        self.eLoss = SpeakerMetaEncLoss(preprocess_config, model_config)
        self.opt = ScheduledOptim(model, train_config, model_config, current_step)
        self.clip = train_config["optimizer"]["grad_clip_thresh"]
        # train.py:108,112: the batch counter starts at restore_step + 1; the optimiser steps
        # on the batches where it is a multiple of grad_acc_step
        self.grad_acc = int(train_config["optimizer"].get("grad_acc_step", 1))
        if self.grad_acc < 1:
            raise ValueError("grad_acc_step must be >= 1")
        self.batch_step = int(current_step) + 1
        if self.graph_mode and self.grad_acc > 1:
            # the captured step is one whole optimiser step; accumulated micro-batches (whose
            # update flag alternates) run eagerly -- say so instead of dropping the mode silently
            warnings.warn("Trainer(graph=True) with grad_acc_step > 1 runs eager steps "
                          "(HIP-graph replay captures whole optimiser steps only)", stacklevel=2)
        self.pg = process_group
        self._agree = False  # data-parallel shards padded to the ranks' maxima (_agree_lengths)
        self._host_pg = None  # its group (None: the default group, when that is gloo)
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.dp = self.world > 1 if data_parallel is None else bool(data_parallel)
        self.cm = collective_model
        if self.cm is not None:  # the data-parallel step with stand-in collectives
            self.dp = True
        if self.dp and self.cm is None and not dist.is_initialized():
            raise ValueError("data_parallel needs an initialised process group")
        self.buckets = None
        if self.cm is not None:
            arena = model.arena()
            self.buckets = GradBuckets(arena, None, bucket_bytes)
            self.buckets.standin = self.cm
            # comm_stream: issue each bucket from a stream of its own, event-gated on the main
            # stream and on the weight-gradient stream (default: from the weight-gradient stream)
            cs = torch.cuda.Stream() if comm_stream else None
            self.buckets.producers = (lambda: (model._side, cs)) if cs is not None else (lambda: (model._side,))
            model._hooks["grad"] = self.buckets.ready
        elif self.dp:
            from .model import stream_reservation_problem
            problem = stream_reservation_problem(model.encoder.position_enc.device)
            if problem is not None:
                if os.environ.get("FS2_DP_STRICT") == "1":
                    raise RuntimeError(problem)
                warnings.warn(problem, RuntimeWarning, stacklevel=2)
            arena = model.arena()
            with torch.no_grad():  # identical initial weights on every rank
                dist.broadcast(arena.flat, src=0, group=process_group)
            self.buckets = GradBuckets(arena, process_group, bucket_bytes)
            self.buckets.producers = lambda: (model._side,)
            model._hooks["grad"] = self.buckets.ready
            # host-side group for the ranks' shard lengths (_agree_lengths): gloo on CPU ints,
            # so agreeing on them never waits for the GPU
            self._agree = True
            if "gloo" in str(dist.get_backend(process_group)):
                self._host_pg = process_group
            else:
                ranks = None if process_group is None else dist.get_process_group_ranks(process_group)
                self._host_pg = dist.new_group(ranks=ranks, backend="gloo")

    def _agree_lengths(self, batch):
        """``nn.DataParallel`` semantics for the shards' padded lengths.  The reference collates
        the global batch (``dataset.py:133-140``) and ``nn.DataParallel`` (``train.py:67-68``)
        hands every replica its rows of it together with the global ``max_src_len`` /
        ``max_mel_len``.  Those lengths are visible in the outputs: the PostNet BatchNorm
        statistics run over every padded frame, the variance predictors' convs read the padded
        phoneme rows (which carry the speaker embedding), and the ``--use_clf`` chunking cuts the
        padded mel into ``max_mel_len // 150 + 1`` chunks.  So each rank pads its shard to the
        ranks' maxima (one host-side all-reduce of two ints, no GPU sync) before the step."""
        if not self._agree:
            return batch
        t = torch.tensor([int(batch[5]), int(batch[8])], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self._host_pg)
        ts, tm = int(t[0]), int(t[1])
        if ts == int(batch[5]) and tm == int(batch[8]):
            return batch
        from .data import pad_batch
        return pad_batch(batch, ts, tm)

    def _global_denominators(self, batch):
        T_dec = min(int(batch[8]), self.model.decoder.max_seq_len)
        counts = K.dp_counts(batch[4].contiguous().long(), batch[7].contiguous().long(),
                             int(batch[5]), T_dec, self.model.mel_linear.out_features)
        if self.cm is not None:
            self.cm.small(counts)  # its latency; the counts stay local
        else:
            dist.all_reduce(counts, group=self.pg)
        return counts

    def _shape_key(self, batch):
        return tuple(tuple(b.shape) if torch.is_tensor(b) else b for b in batch)

    def _graph_step(self, batch):
        key = self._shape_key(batch)
        if self._graph is not None and key == self._graph_key:
            for s, b in zip(self._static, batch):
                if torch.is_tensor(b):
                    s.copy_(b)
            self._graph.replay()
            self.opt.host_advance()
            return self._graph_out
        # eager step (this call's step), then capture the next one
        out = train_step(self.model, self.opt, self.Loss, self.eLoss, batch, self.clip)
        self._static = tuple(b.clone() if torch.is_tensor(b) else b for b in batch)
        host = (self.opt.current_step, self.opt.adam_steps,
                self.opt._optimizer.param_groups[0]["lr"])
        g = torch.cuda.CUDAGraph()
        try:  # the weight-gradient side stream joins the capture (parallel graph branches)
            with torch.cuda.graph(g):
                self._graph_out = train_step(self.model, self.opt, self.Loss, self.eLoss,
                                             self._static, self.clip)
        finally:
            # capture recorded kernels without running them: undo its host-side bookkeeping
            self.opt.current_step, self.opt.adam_steps = host[0], host[1]
            self.opt._optimizer.param_groups[0]["lr"] = host[2]
        self._graph, self._graph_key = g, key
        return out

    def step(self, batch, clf=None, clf_args=None):
        """One batch (``train.py:137-206``); the optimiser steps when the batch counter is a
        multiple of ``grad_acc_step`` (the returned grad norm is None on the other batches).
        ``clf=(SpeechEmbedder, GE2ELoss)`` with ``clf_args=(perm, step, total_step, lambd)``
        adds the ``--use_clf`` branch (eager; under data parallelism ``perm`` permutes the
        global batch and this step's gradient buckets go out after the clf backward)."""
        update = self.batch_step % self.grad_acc == 0
        self.batch_step += 1
        if self.dp:
            batch = self._agree_lengths(batch)
        acc = dict(grad_acc_step=self.grad_acc, update=update)
        if clf is not None:
            if not self.dp:
                return train_step(self.model, self.opt, self.Loss, self.eLoss, batch, self.clip,
                                  clf=clf, clf_args=clf_args, **acc)
            # data parallel: the clf backward adds to every parameter's gradient after the main
            # backward has released the buckets, so this step's buckets all go out in finish(),
            # after it (no overlap); perm permutes the global batch (clf_backward)
            glob = self._global_denominators(batch)
            self.Loss.denoms = glob[0:2]
            self.eLoss.denom = glob[2:3]
            self.model._hooks["grad"] = None
            return train_step(self.model, self.opt, self.Loss, self.eLoss, batch, self.clip,
                              grad_sync=self.buckets.finish, clf=clf, clf_args=clf_args,
                              clf_group=None if self.cm is not None else
                              (self.pg if self.pg is not None else dist.group.WORLD), **acc)
        if self.graph_mode and not self.dp and self.grad_acc == 1:
            return self._graph_step(batch)
        if self.dp:
            glob = self._global_denominators(batch)
            self.Loss.denoms = glob[0:2]
            self.eLoss.denom = glob[2:3]
            # accumulated micro-batches are summed locally; the buckets all-reduce the
            # accumulated buffer during the backward of the batch that steps (all-reduce is
            # linear, so this equals all-reducing every micro-batch)
            self.model._hooks["grad"] = self.buckets.ready if update else None
            return train_step(self.model, self.opt, self.Loss, self.eLoss, batch, self.clip,
                              grad_sync=self.buckets.finish, **acc)
        return train_step(self.model, self.opt, self.Loss, self.eLoss, batch, self.clip, **acc)
