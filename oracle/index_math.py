"""ORACLE — TEST INFRASTRUCTURE ONLY.  numpy restatement of the integer index math on the
hot path; the HIP kernels must reproduce these bit-exactly.

* ``lr_source_map`` — LengthRegulator (``model/modules.py:167-194`` + ``utils/tools.py:363-381``):
  frame t of utterance b copies phoneme row i where cum[i-1] <= t < cum[i], cum being the
  inclusive scan of ``max(int(d), 0)`` (``int`` truncates toward zero); frames at or past
  ``mel_len`` are padding (-1 here).  ``mel_len`` is the *uncropped* total even when the
  output is cropped to ``max_len``.
* ``bucketize`` — ``torch.bucketize(v, bins, right=False)`` as used at
  ``model/modules.py:84,96``: the number of bins strictly below v, i.e. the index i with
  bins[i-1] < v <= bins[i].
"""
import numpy as np


def lr_source_map(durations, max_len=None):
    d = np.asarray(durations)
    reps = np.maximum(np.trunc(d.astype(np.float64)), 0).astype(np.int64)
    cum = np.cumsum(reps, axis=1)
    mel_len = cum[:, -1] if d.shape[1] else np.zeros(d.shape[0], np.int64)
    T = int(mel_len.max()) if max_len is None else int(max_len)
    src = np.full((d.shape[0], T), -1, np.int64)
    for b in range(d.shape[0]):
        t = np.arange(min(T, int(mel_len[b])))
        src[b, : len(t)] = np.searchsorted(cum[b], t, side="right")
    return src, mel_len.astype(np.int64)


def length_regulate(x, durations, max_len=None):
    src, mel_len = lr_source_map(durations, max_len)
    out = np.zeros((x.shape[0], src.shape[1]) + x.shape[2:], x.dtype)
    for b in range(x.shape[0]):
        ok = src[b] >= 0
        out[b, ok] = x[b, src[b, ok]]
    return out, mel_len


def bucketize(values, bins):
    v = np.asarray(values)
    bins = np.asarray(bins)
    dt = np.result_type(v.dtype, bins.dtype)
    return np.searchsorted(bins.astype(dt), v.astype(dt), side="left").astype(np.int64)


def inference_durations(log_d, d_control=1.0):
    """``model/modules.py:132-135``: clamp(round(exp(log_d) - 1) * control, 0), with
    round-half-to-even as torch.round does."""
    return np.maximum(np.round(np.exp(log_d) - 1) * d_control, 0)
