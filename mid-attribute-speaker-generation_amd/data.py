"""Synthetic padded phoneme/mel batches in the reference's batch-tuple layout.

The reference's ``Dataset.reprocess`` (``dataset.py:112-172``) returns the 14-tuple
``(ids, raw_texts, speakers, texts, src_lens, max_src_len, mels, mel_lens, max_mel_len,
pitches, energies, durations, speaker_meta, accents)``; ``utils/tools.py:to_device``
(18-125) turns it into tensors.  There is no corpus on the GPU box, so ``syn_batch``
draws batches of that exact layout from a seeded generator ("SYN-B"):

* ``src_lens[0] = T_s``, the rest uniform on ``[T_s/2, T_s]``, sorted descending as
  ``collate_fn`` sorts (``dataset.py:178-180``);
* ``mel_lens = frames_per_phone * src_lens``; durations are
  ``floor(Dirichlet(1) * mel_len)`` with the remainder added to the first phonemes, so
  ``sum(durations[b]) == mel_lens[b]`` (zeros allowed, as in MFA output);
* texts on ``[1, 427]`` (0 = PAD), accents on ``[0, 3]``, speakers on ``[0, n_speakers)``,
  speaker metadata a one-hot per attribute; mels ``N(-5, 2^2)`` (log-mel range),
  pitch (f64, cast to f32 by ``to_device``) and energy (f32) ``N(0, 1)`` (already
  z-normalised, as ``ConcatDataset`` leaves them, ``dataset.py:208-209``).
"""
import numpy as np
import torch

N_SYMBOLS = 428  # len(text.symbols.symbols) in the reference (text/symbols.py:23-33)


def syn_batch(batch_size, max_src_len=128, seed=0, frames_per_phone=4, n_speakers=209,
              meta_sizes=(2, 2), n_mels=80):
    rng = np.random.default_rng(seed)
    B, Ts = batch_size, max_src_len
    src = np.concatenate([[Ts], rng.integers(Ts // 2, Ts + 1, size=B - 1)]).astype(np.int64)
    src = np.sort(src)[::-1].copy()
    mel = frames_per_phone * src
    Tm = int(mel.max())

    texts = np.zeros((B, Ts), np.int64)
    accents = np.zeros((B, Ts), np.int64)
    durations = np.zeros((B, Ts), np.int64)
    pitches = np.zeros((B, Ts), np.float64)
    energies = np.zeros((B, Ts), np.float32)
    mels = np.zeros((B, Tm, n_mels), np.float32)
    for b in range(B):
        L, M = int(src[b]), int(mel[b])
        texts[b, :L] = rng.integers(1, N_SYMBOLS, size=L)
        accents[b, :L] = rng.integers(0, 4, size=L)
        d = np.floor(rng.dirichlet(np.ones(L)) * M).astype(np.int64)
        d[: M - int(d.sum())] += 1
        durations[b, :L] = d
        pitches[b, :L] = rng.standard_normal(L)
        energies[b, :L] = rng.standard_normal(L).astype(np.float32)
        mels[b, :M] = (rng.standard_normal((M, n_mels)) * 2.0 - 5.0).astype(np.float32)
    speakers = rng.integers(0, n_speakers, size=B).astype(np.int64)
    meta = np.concatenate(
        [np.eye(n)[rng.integers(0, n, size=B)] for n in meta_sizes], axis=1)
    ids = [f"syn{seed}_{b}" for b in range(B)]
    raw = ["" for _ in range(B)]
    return (ids, raw, speakers, texts, src, int(src.max()), mels, mel.astype(np.int64),
            Tm, pitches, energies, durations, meta, accents)


def syn_batch_for(config_name, batch_size, max_src_len=128, seed=0, **kw):
    """``syn_batch`` shaped for a bundled config: speaker ids on ``[0, len(speakers.json))``
    and one one-hot per metadata attribute of ``preprocess.yaml`` (JVS-VCTK: gender +
    language, width 4; JSUT: gender, width 2; ``model/fastspeech2.py:317``)."""
    from . import config as cfg
    pp, _, _, path = cfg.load_configs(config_name)
    sizes = tuple(len(v) for v in pp["speaker_generation"]["metadata"].values())
    return syn_batch(batch_size, max_src_len, seed=seed, n_speakers=cfg.n_speakers(path),
                     meta_sizes=sizes, **kw)


def to_device(batch, device):
    """Tensor conversion with the dtypes of ``utils/tools.py:to_device`` (14-tuple branch,
    61-105): ids long, pitches/mels/meta float, energies left in their array dtype."""
    (ids, raw, speakers, texts, src_lens, max_src_len, mels, mel_lens, max_mel_len,
     pitches, energies, durations, speaker_meta, accents) = batch
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))
    return (ids, raw,
            t(speakers).long().to(device),
            t(texts).long().to(device),
            t(src_lens).to(device),
            max_src_len,
            t(mels).float().to(device),
            t(mel_lens).to(device),
            max_mel_len,
            t(pitches).float().to(device),
            t(energies).to(device),
            t(durations).long().to(device),
            t(speaker_meta).float().to(device),
            t(accents).long().to(device))


def pad_batch(batch, max_src_len, max_mel_len):
    """A device batch padded on the right to ``max_src_len`` phonemes / ``max_mel_len`` frames
    (zeros, as ``collate_fn``'s ``pad_1D`` / ``pad_2D`` pad the whole batch,
    ``dataset.py:133-140``, ``utils/tools.py:329-360``); the lengths are unchanged.  Used
    for a data-parallel shard whose own maxima are below the global batch's (see
    ``train.Trainer``)."""
    b = list(batch)
    ds, dm = int(max_src_len) - int(b[5]), int(max_mel_len) - int(b[8])
    if ds < 0 or dm < 0:
        raise ValueError("pad_batch: target lengths below the batch's own")
    F = torch.nn.functional
    if ds:
        for i in (3, 9, 10, 11, 13):  # texts, pitches, energies, durations, accents
            b[i] = F.pad(b[i], (0, ds))
        b[5] = int(max_src_len)
    if dm:
        b[6] = F.pad(b[6], (0, 0, 0, dm))  # mels (B, T, n_mel)
        b[8] = int(max_mel_len)
    return tuple(b)


def valid_frames(batch):
    return int(np.asarray(batch[7] if not torch.is_tensor(batch[7]) else batch[7].cpu()).sum())
