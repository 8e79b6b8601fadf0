"""Seeded synthetic preprocessed corpora in the FastSpeech2 on-disk layout (test data).

Two corpora, as the JVS-VCTK configuration trains on (``train.py:33-47``): ``JA`` with
accent files (``use_accent: True``, like JSUT/JVS) and ``EN`` without (like VCTK).  Each holds
``train.txt`` (``basename|speaker|{phones}|raw``), ``speakers.json`` and per-utterance
``mel``/``pitch``/``energy``/``duration`` ``.npy`` files in the dtypes the reference's
preprocessor writes (mel (T, 80) f32, pitch f64, energy f32, duration int64;
``preprocessor/preprocessor.py:244-258,317-328``); the config directory holds ``stats.json``
and the merged ``speakers.json``.  Used by ``oracle/make_golden.py`` (g8) and the tests.
"""
import json
import os

import numpy as np

META = {"gender": {"M": 0, "F": 1}, "language": {"ja": 0, "en": 1}}
STATS = {"pitch": [-1.9, 9.1, 210.0, 45.0], "energy": [-1.3, 19.5, 30.0, 12.0]}


def _symbols():
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(here, "mid-attribute-speaker-generation_amd", "configs",
                           "symbols.json"), encoding="utf-8") as f:
        return json.load(f)


def make_corpora(root, seed=0, n_ja=13, n_en=11):
    """Write the corpora under ``root``; return ``(config_dir, [corpus_cfg_JA, corpus_cfg_EN],
    preprocess_config, train_config)`` ready for ``Dataset``/``ConcatDataset``."""
    rng = np.random.default_rng(seed)
    syms = _symbols()
    phones_ja = [s for s in syms[1:] if s.isalpha() and len(s) <= 2]  # plain letters / kana-like
    phones_en = [s for s in syms if s.startswith("@") and s[1:2].isupper()]  # ARPAbet
    speakers = {"ja": [("jsut", "F"), ("jvs001", "M"), ("jvs002", "F")],
                "en": [("p225", "F"), ("p226", "M")]}
    cfg_dir = os.path.join(root, "config")
    os.makedirs(cfg_dir, exist_ok=True)
    merged = {}
    k = 0
    for lang in ("ja", "en"):
        for name, g in speakers[lang]:
            merged[name] = [k, g, lang]
            k += 1
    with open(os.path.join(cfg_dir, "speakers.json"), "w") as f:
        json.dump(merged, f)
    with open(os.path.join(cfg_dir, "stats.json"), "w") as f:
        json.dump(STATS, f)
    corpora = []
    for tag, lang, n, use_accent, plist in (("JA", "ja", n_ja, True, phones_ja),
                                            ("EN", "en", n_en, False, phones_en)):
        pre = os.path.join(root, tag)
        for d in ("mel", "pitch", "energy", "duration", "accent"):
            os.makedirs(os.path.join(pre, d), exist_ok=True)
        local = {name: [i, g, lang] for i, (name, g) in enumerate(speakers[lang])}
        with open(os.path.join(pre, "speakers.json"), "w") as f:
            json.dump(local, f)
        lines = []
        for u in range(n):
            spk = speakers[lang][int(rng.integers(len(speakers[lang])))][0]
            base = f"{tag.lower()}_{u:03d}"
            L = int(rng.integers(3, 20))
            ph = [plist[int(i)] for i in rng.integers(0, len(plist), size=L)]
            dur = rng.integers(0, 7, size=L).astype(np.int64)
            dur[0] += 1
            T = int(dur.sum())
            np.save(os.path.join(pre, "mel", f"{spk}-mel-{base}.npy"),
                    rng.standard_normal((T, 80)).astype(np.float32))
            np.save(os.path.join(pre, "pitch", f"{spk}-pitch-{base}.npy"),
                    rng.uniform(80, 400, size=L).astype(np.float64))
            np.save(os.path.join(pre, "energy", f"{spk}-energy-{base}.npy"),
                    rng.uniform(0, 80, size=L).astype(np.float32))
            np.save(os.path.join(pre, "duration", f"{spk}-duration-{base}.npy"), dur)
            if use_accent:  # one accent char per phone (+ a few extra: truncated by Dataset)
                acc = "".join("0[]#"[int(i)] for i in rng.integers(0, 4, size=L + 2))
                with open(os.path.join(pre, "accent", base + ".accent"), "w") as f:
                    f.write(acc)
            lines.append(f"{base}|{spk}|{{{' '.join(ph)}}}|raw text {u}")
        with open(os.path.join(pre, "train.txt"), "w", encoding="utf-8") as f:
            f.write("\n".join(lines) + "\n")
        corpora.append({"dataset": tag, "path": {"preprocessed_path": pre},
                        "text": {"text_cleaners": ["english_cleaners"], "language": lang},
                        "accent": {"use_accent": use_accent}})
    pp = {"speaker_generation": {"metadata": META}}
    tc = {"optimizer": {"batch_size": 4}}
    return cfg_dir, corpora, pp, tc
