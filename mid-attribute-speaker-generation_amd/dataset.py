"""Preprocessed-corpus loading, batching and staging into HBM.

Host-side mirror of the reference's data path, same names, arguments and outputs:

* ``Dataset(filename, preprocess_config, train_config, sort, drop_last)`` reads the
  FastSpeech2 preprocessed layout (``dataset.py:13-110``): ``<preprocessed>/<filename>``
  metadata lines ``basename|speaker|{phones}|raw text``, ``speakers.json``
  (``speaker -> [id, meta...]``), per-utterance ``mel/ pitch/ energy/ duration/`` ``.npy``
  files and, with ``use_accent``, ``accent/<basename>.accent`` character strings.
* ``collate_fn`` (``dataset.py:175-194``): optional sort by phoneme count (``np.argsort`` of
  the negated lengths, numpy's default kind, as the reference), groups of ``batch_size``,
  tail dropped or kept; each group padded by ``reprocess`` (``dataset.py:112-172``) into the
  14-tuple (13 without accents) that ``train.py:142-145`` consumes.
* ``ConcatDataset(config_dir, datasets)`` (``dataset.py:197-211``): z-normalises pitch and
  energy with ``stats.json[2:4]`` and re-maps speaker ids through the config's
  ``speakers.json``; collates with the FIRST dataset's ``collate_fn`` (so its
  ``use_accent`` decides the tuple length for every corpus, a reference quirk).
* ``pad_1D`` / ``pad_2D`` (``utils/tools.py:329-360``) and ``to_device``
  (``utils/tools.py:18-125``, 13/14/7/8-tuples).

MI355X side: ``BatchStager`` replaces the reference's ten ``torch.from_numpy(..).to(device)``
round trips per batch (``utils/tools.py:61-105``, each a pageable host copy) with ONE packed,
pinned host buffer and ONE asynchronous host-to-device copy on a dedicated copy stream; the
device tensors are views into a single HBM staging buffer with exactly the dtypes and
shapes ``to_device`` produces.  Staging batch k+1 overlaps step k (double-buffered slots;
the compute stream waits on the copy's event only when it consumes the batch).
"""
import json
import os

import numpy as np
import torch

from .config import CONFIG_ROOT

_ACCENT_TO_ID = {"0": 0, "[": 1, "]": 2, "#": 3}  # dataset.py:22


def symbol_table():
    """The reference's symbol list (``text/symbols.py:23-33``; configs/symbols.json)."""
    with open(os.path.join(CONFIG_ROOT, "symbols.json"), encoding="utf-8") as f:
        return json.load(f)


def symbol_to_id():
    # a dict comprehension, as dataset.py:21: a repeated symbol maps to its LAST position
    return {s: i for i, s in enumerate(symbol_table())}


# ------------------------------------------------------------------ padding (utils/tools.py)
def pad_1D(inputs, PAD=0):
    """Right-pad 1-D arrays to the longest and stack (``utils/tools.py:329-339``)."""
    max_len = max(len(x) for x in inputs)
    return np.stack([np.pad(x, (0, max_len - x.shape[0]), mode="constant", constant_values=PAD)
                     for x in inputs])


def pad_2D(inputs, maxlen=None):
    """Right-pad (T, C) arrays along T and stack (``utils/tools.py:342-360``)."""
    max_len = maxlen if maxlen else max(np.shape(x)[0] for x in inputs)
    out = []
    for x in inputs:
        if np.shape(x)[0] > max_len:
            raise ValueError("not max_len")
        out.append(np.pad(x, ((0, max_len - np.shape(x)[0]), (0, 0)), mode="constant",
                          constant_values=0))
    return np.stack(out)


# ------------------------------------------------------------------ Dataset
class Dataset(torch.utils.data.Dataset):
    """``dataset.py:13-194``."""

    def __init__(self, filename, preprocess_config, train_config, sort=False, drop_last=False):
        self.dataset_name = preprocess_config["dataset"]
        self.preprocessed_path = preprocess_config["path"]["preprocessed_path"]
        self.cleaners = preprocess_config["preprocessing"]["text"]["text_cleaners"]
        self.batch_size = train_config["optimizer"]["batch_size"]
        self.symbol_to_id = symbol_to_id()
        self.use_accent = preprocess_config["preprocessing"]["accent"]["use_accent"]
        self.accent_to_id = dict(_ACCENT_TO_ID)
        self.basename, self.speaker, self.text, self.raw_text = self.process_meta(filename)
        with open(os.path.join(self.preprocessed_path, "speakers.json")) as f:
            self.speaker_map = json.load(f)
        self.speaker_meta = preprocess_config["preprocessing"]["speaker_generation"]["metadata"]
        self.sort = sort
        self.drop_last = drop_last

    def __len__(self):
        return len(self.text)

    def _npy(self, kind, speaker, basename):
        return np.load(os.path.join(self.preprocessed_path, kind,
                                    f"{speaker}-{kind}-{basename}.npy"))

    def __getitem__(self, idx):
        basename, speaker = self.basename[idx], self.speaker[idx]
        entry = self.speaker_map[speaker]
        speaker_meta = {meta: entry[i + 1] for i, meta in enumerate(self.speaker_meta)}
        phones = self.text[idx].replace("{", "").replace("}", "").split()
        phone = np.array([self.symbol_to_id[t] for t in phones])
        if self.use_accent:
            with open(os.path.join(self.preprocessed_path, "accent", basename + ".accent")) as f:
                accent = f.read()
            accent = np.array([self.accent_to_id[t] for t in accent][:len(phone)])
        else:
            accent = np.array([4] * len(phone))
        return {
            "id": basename, "speaker": entry[0], "speaker_name": speaker,
            "speaker_meta": speaker_meta, "text": phone, "raw_text": self.raw_text[idx],
            "mel": self._npy("mel", speaker, basename),
            "pitch": self._npy("pitch", speaker, basename),
            "energy": self._npy("energy", speaker, basename),
            "duration": self._npy("duration", speaker, basename),
            "accent": accent,
        }

    def process_meta(self, filename):
        name, speaker, text, raw_text = [], [], [], []
        with open(os.path.join(self.preprocessed_path, filename), "r", encoding="utf-8") as f:
            for line in f.readlines():
                n, s, t, r = line.strip("\n").split("|")
                name.append(n)
                speaker.append(s)
                text.append(t)
                raw_text.append(r)
        return name, speaker, text, raw_text

    def reprocess(self, data, idxs):
        """Pad one group into the batch tuple (``dataset.py:112-172``)."""
        pick = [data[i] for i in idxs]
        texts = [d["text"] for d in pick]
        mels = [d["mel"] for d in pick]
        # one-hot per metadata attribute, concatenated in config order (dataset.py:123-126)
        speaker_meta = np.array([
            np.concatenate([np.eye(len(self.speaker_meta[meta]))[self.speaker_meta[meta][val]]
                            for meta, val in d["speaker_meta"].items()]) for d in pick])
        text_lens = np.array([t.shape[0] for t in texts])
        mel_lens = np.array([m.shape[0] for m in mels])
        out = ([d["id"] for d in pick], [d["raw_text"] for d in pick],
               np.array([d["speaker"] for d in pick]), pad_1D(texts), text_lens,
               max(text_lens), pad_2D(mels), mel_lens, max(mel_lens),
               pad_1D([d["pitch"] for d in pick]), pad_1D([d["energy"] for d in pick]),
               pad_1D([d["duration"] for d in pick]), speaker_meta)
        if self.use_accent:
            return out + (pad_1D([d["accent"] for d in pick]),)
        return out

    def collate_fn(self, data):
        """Sort (optional), split into batch_size groups, pad each (``dataset.py:175-194``)."""
        n = len(data)
        if self.sort:
            idx_arr = np.argsort(-np.array([d["text"].shape[0] for d in data]))
        else:
            idx_arr = np.arange(n)
        cut = len(idx_arr) - (len(idx_arr) % self.batch_size)
        tail = idx_arr[cut:]
        groups = idx_arr[:cut].reshape((-1, self.batch_size)).tolist()
        if not self.drop_last and len(tail) > 0:
            groups += [tail.tolist()]
        return [self.reprocess(data, g) for g in groups]


class ConcatDataset(torch.utils.data.ConcatDataset):
    """``dataset.py:197-211``: pitch/energy z-normalised with ``stats.json[2:4]``, speaker id
    from the config's ``speakers.json``, collated by the first dataset."""

    def __init__(self, config, datasets):
        super().__init__(datasets)
        self.collate_fn = datasets[0].collate_fn
        with open(os.path.join(config, "stats.json")) as f:
            self.stats = json.load(f)
        with open(os.path.join(config, "speakers.json")) as f:
            self.speaker_map = json.load(f)

    def __getitem__(self, idx):
        sample = super().__getitem__(idx)
        sample["pitch"] = (sample["pitch"] - self.stats["pitch"][2]) / self.stats["pitch"][3]
        sample["energy"] = (sample["energy"] - self.stats["energy"][2]) / self.stats["energy"][3]
        sample["speaker"] = self.speaker_map[sample["speaker_name"]][0]
        return sample


def corpus_config(preprocess_config, corpus):
    """The per-corpus preprocess config ``train.py`` assembles (``train.py:36-41``): the
    corpus file's ``dataset``/``path`` plus the shared ``preprocessing`` section with the
    corpus's ``text`` and ``accent`` entries."""
    cfg = dict(corpus)
    pre = dict(preprocess_config)
    pre["text"] = corpus["text"]
    pre["accent"] = corpus["accent"]
    cfg["preprocessing"] = pre
    return cfg


# ------------------------------------------------------------------ to_device
def to_device(batch, device):
    """``utils/tools.py:18-125``: the 13/14-tuple training batch and the 7/8-tuple text
    batch, with the reference's dtypes (ids long, mels/pitch/meta float, energies as-is)."""
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))
    n = len(batch)
    if n in (13, 14):
        (ids, raw, speakers, texts, src_lens, max_src_len, mels, mel_lens, max_mel_len,
         pitches, energies, durations, speaker_meta) = batch[:13]
        out = (ids, raw, t(speakers).long().to(device), t(texts).long().to(device),
               t(src_lens).to(device), max_src_len, t(mels).float().to(device),
               t(mel_lens).to(device), max_mel_len, t(pitches).float().to(device),
               t(energies).to(device), t(durations).long().to(device),
               t(speaker_meta).float().to(device))
        return out + ((t(batch[13]).long().to(device),) if n == 14 else ())
    if n in (7, 8):
        ids, raw, speakers, texts, src_lens, max_src_len, speaker_meta = batch[:7]
        out = (ids, raw, t(speakers).long().to(device), t(texts).long().to(device),
               t(src_lens).to(device), max_src_len, t(speaker_meta).float().to(device))
        return out + ((t(batch[7]).long().to(device),) if n == 8 else ())
    raise ValueError(f"to_device: unsupported batch tuple of length {n}")


# ------------------------------------------------------------------ HBM staging
# tuple index -> target dtype (None: keep the array's dtype, as to_device does for energies)
_TRAIN_FIELDS = ((2, torch.int64), (3, torch.int64), (4, None), (6, torch.float32),
                 (7, None), (9, torch.float32), (10, None), (11, torch.int64),
                 (12, torch.float32), (13, torch.int64))
_NP_OF = {torch.int64: np.int64, torch.float32: np.float32}
_TORCH_OF = {np.dtype(np.int64): torch.int64, np.dtype(np.int32): torch.int32,
             np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64,
             np.dtype(np.int16): torch.int16, np.dtype(np.uint8): torch.uint8}


class BatchStager:
    """Packs collated training batches into pinned host memory and moves each with ONE
    asynchronous copy into HBM (see the module docstring).  ``stage(batch)`` returns the
    tuple ``to_device`` would return (same dtypes, shapes and values); its tensors are valid
    until ``slots`` further batches have been staged.  Consumers on the current stream are
    ordered after the copy automatically (the current stream waits on the copy event)."""

    def __init__(self, device, slots=2, copy_stream=None):
        self.device = torch.device(device)
        self.slots = slots
        self.stream = copy_stream or (torch.cuda.Stream(self.device)
                                      if self.device.type == "cuda" else None)
        self._host = [None] * slots
        self._dev = [None] * slots
        self._done = [None] * slots  # copy event of the slot's last use
        self._k = 0

    @staticmethod
    def _layout(batch):
        parts, off = [], 0
        for i, dt in _TRAIN_FIELDS[:len(batch) - 4]:
            a = np.asarray(batch[i])
            npdt = np.dtype(_NP_OF[dt]) if dt is not None else a.dtype
            off = (off + 63) // 64 * 64  # 64-B aligned sections
            parts.append((i, a, npdt, off))
            off += a.size * npdt.itemsize
        return parts, off

    def _buffers(self, slot, nbytes):
        h = self._host[slot]
        if h is None or h.numel() < nbytes:
            cap = max(nbytes, 1 << 20)
            pin = self.device.type == "cuda"
            self._host[slot] = torch.empty(cap, dtype=torch.uint8, pin_memory=pin)
            self._dev[slot] = torch.empty(cap, dtype=torch.uint8, device=self.device)
        return self._host[slot], self._dev[slot]

    def stage(self, batch):
        if len(batch) not in (13, 14):
            raise ValueError("BatchStager stages the 13/14-tuple training batch")
        slot = self._k % self.slots
        self._k += 1
        parts, nbytes = self._layout(batch)
        if self._done[slot] is not None:
            self._done[slot].synchronize()  # the host buffer's previous copy has finished
        host, dev = self._buffers(slot, nbytes)
        hv = host.numpy()
        for i, a, npdt, off in parts:
            dst = hv[off:off + a.size * npdt.itemsize].view(npdt).reshape(a.shape)
            np.copyto(dst, a, casting="unsafe")
        out = list(batch)
        if self.stream is not None:
            cur = torch.cuda.current_stream(self.device)
            # every consumer of the batch this slot held was enqueued on the compute stream
            # before this call: the copy may overwrite the slot once those have run
            used = torch.cuda.Event()
            used.record(cur)
            self.stream.wait_event(used)
            with torch.cuda.stream(self.stream):
                dev[:nbytes].copy_(host[:nbytes], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.stream)
            self._done[slot] = ev
            cur.wait_event(ev)  # consumers on the compute stream see the landed batch
        else:
            dev[:nbytes].copy_(host[:nbytes])
        for i, a, npdt, off in parts:
            n = a.size * npdt.itemsize
            out[i] = dev[off:off + n].view(_TORCH_OF[npdt]).view(a.shape)
        return tuple(out)
