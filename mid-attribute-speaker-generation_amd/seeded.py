"""Name-seeded weights: every state-dict entry is a pure function of (key, shape).

Parity fixtures must not store a 139 MB state dict, and the reference,
the CPU oracle and the HIP path must all start from the same weights.  Each key gets its
own ``numpy.random.default_rng(crc32(key))``; the rule per key kind is below.  Frozen
tensors that the model computes itself (``position_enc``, ``*_bins``) are left alone.
"""
import zlib

import numpy as np

COMPUTED_SUFFIXES = ("position_enc", "pitch_bins", "energy_bins")


def seeded_array(key, shape):
    """fp32 array for state-dict entry ``key`` of ``shape`` (None for computed entries)."""
    if key.endswith(COMPUTED_SUFFIXES):
        return None
    shape = tuple(int(s) for s in shape)
    if key.endswith("num_batches_tracked"):
        return np.zeros(shape, np.int64)
    if key.endswith("running_mean"):
        return np.zeros(shape, np.float32)
    if key.endswith("running_var"):
        return np.ones(shape, np.float32)
    rng = np.random.default_rng(zlib.crc32(key.encode()))
    z = rng.standard_normal(shape)
    is_norm = (".layer_norm" in key) or key.split(".")[-2].isdigit() and len(shape) == 1 \
        and "postnet" in key
    if is_norm:
        a = 1.0 + 0.1 * z if key.endswith("weight") else 0.1 * z
    elif key.endswith("emb.weight") or key.endswith("embedding.weight"):
        a = 0.5 * z
        if key.endswith(("src_word_emb.weight", "src_accent_emb.weight")):
            a[0] = 0.0  # padding_idx=0 row (transformer/Models.py:56-62)
    elif len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        a = z / np.sqrt(fan_in)
    else:  # biases
        a = 0.05 * z
    return a.astype(np.float32)


def seeded_state_dict(state_dict_shapes):
    """``{key: np.ndarray}`` for an iterable of ``(key, shape)``."""
    out = {}
    for k, shape in state_dict_shapes:
        a = seeded_array(k, shape)
        if a is not None:
            out[k] = a
    return out


def load_seeded_(module):
    """Overwrite ``module``'s parameters/buffers in place with the name-seeded values."""
    import torch
    sd = module.state_dict()
    new = seeded_state_dict((k, v.shape) for k, v in sd.items())
    with torch.no_grad():
        for k, a in new.items():
            sd[k].copy_(torch.from_numpy(a))
    return module
