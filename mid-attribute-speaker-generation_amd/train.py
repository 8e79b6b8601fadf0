"""The training step of ``train.py:134-206`` (``use_clf`` off, ``grad_acc_step`` 1) and its
data-parallel form.

Single process: ``train_step`` is line-for-line the reference's step semantics
(forward, FastSpeech2Loss backward, negated speaker-prior log-likelihood backward,
clip_grad_norm_, ScheduledOptim.step_and_update_lr, zero_grad).

Data parallel: one process per GPU, batch sharded by utterance.  Each rank
normalises its masked means by the *global* valid counts and the GMM term by the global
batch, so the all-reduced (summed) gradient equals the 1-process gradient of the global
batch; the sum runs over RCCL on the flat gradient buffer.  BatchNorm statistics stay
per rank (DataParallel's per-replica semantics).
"""
import torch
import torch.distributed as dist

from . import kernels as K
from .loss import FastSpeech2Loss, SpeakerMetaEncLoss
from .optimizer import ScheduledOptim


def train_step(model, optimizer, Loss, eLoss, batch, grad_clip_thresh=1.0, grad_sync=None):
    output = model(*(batch[2:12]), accents=batch[13], speaker_meta=batch[12])
    losses = Loss(batch[:12], output[:-2])
    losses[0].backward()
    eloss = eLoss(output[-1], output[-2])
    (-eloss).backward()
    if grad_sync is not None:
        grad_sync()
    gnorm = optimizer.clip_grad_norm_(grad_clip_thresh)
    optimizer.step_and_update_lr()
    optimizer.zero_grad()
    return losses, eloss, gnorm, output


class Trainer:
    """Model + loss + optimiser for one rank (``world_size`` 1 = plain single-GPU)."""

    def __init__(self, model, preprocess_config, model_config, train_config, current_step=0,
                 process_group=None):
        self.model = model
        self.Loss = FastSpeech2Loss(preprocess_config, model_config)
        self.eLoss = SpeakerMetaEncLoss(preprocess_config, model_config)
        self.opt = ScheduledOptim(model, train_config, model_config, current_step)
        self.clip = train_config["optimizer"]["grad_clip_thresh"]
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if (dist.is_initialized()) else 1
        if self.world > 1:
            with torch.no_grad():  # identical initial weights on every rank
                dist.broadcast(model.arena().flat, src=0, group=process_group)

    def _global_norm(self, batch):
        """Global denominators [mel elements, phonemes] and batch size via one tiny all-reduce."""
        mel_lens, src_lens = batch[7], batch[4]
        T_dec = min(int(batch[8]), self.model.decoder.max_seq_len)
        n_mel = self.model.mel_linear.out_features
        loc = torch.stack([mel_lens.clamp(max=T_dec).sum().float() * n_mel,
                           src_lens.sum().float(), torch.tensor(float(src_lens.numel()),
                                                                device=src_lens.device)])
        glob = loc.clone()
        dist.all_reduce(glob, group=self.pg)
        return glob

    def step(self, batch):
        if self.world > 1:
            glob = self._global_norm(batch)
            self.Loss.denoms = glob[:2].contiguous()
            self.eLoss.scale = float(batch[4].numel()) / float(glob[2].item())
            return train_step(self.model, self.opt, self.Loss, self.eLoss, batch, self.clip,
                              grad_sync=self._all_reduce)
        return train_step(self.model, self.opt, self.Loss, self.eLoss, batch, self.clip)

    def _all_reduce(self):
        dist.all_reduce(self.model.arena().grad, group=self.pg)
