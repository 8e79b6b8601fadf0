"""Config loading for the FastSpeech2 + TacoSpawn training step.

The reference reads three YAML files plus ``stats.json`` / ``speakers.json`` from a config
directory (``train.py:296-343``, ``model/fastspeech2.py:38-49``, ``model/modules.py:41-71``).
The same layout is bundled here under ``configs/`` so nothing on the GPU box needs the
reference tree.
"""
import json
import os

import yaml

CONFIG_ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "configs")


def config_dir(name="JVS-VCTK"):
    """Path of a bundled config directory (``JVS-VCTK`` or ``JSUT``), or ``name`` itself
    when it already is a directory."""
    if os.path.isdir(name):
        return name
    return os.path.join(CONFIG_ROOT, name)


def load_configs(name="JVS-VCTK"):
    """Return ``(preprocess_config, model_config, train_config, config_path)``."""
    path = config_dir(name)
    with open(os.path.join(path, "preprocess.yaml")) as f:
        pp = yaml.safe_load(f)
    with open(os.path.join(path, "model.yaml")) as f:
        mc = yaml.safe_load(f)
    with open(os.path.join(path, "train.yaml")) as f:
        tc = yaml.safe_load(f)
    return pp, mc, tc, path


def n_speakers(config_path):
    with open(os.path.join(config_path, "speakers.json")) as f:
        return len(json.load(f))


def pitch_energy_range(config_path):
    """``(pitch_min, pitch_max, energy_min, energy_max)`` as ``model/modules.py:41-45`` reads them."""
    with open(os.path.join(config_path, "stats.json")) as f:
        stats = json.load(f)
    return stats["pitch"][0], stats["pitch"][1], stats["energy"][0], stats["energy"][1]


def meta_dim(preprocess_config):
    """Width of the speaker-metadata one-hot vector (``model/fastspeech2.py:317``)."""
    meta = preprocess_config["speaker_generation"]["metadata"]
    return sum(len(v) for v in meta.values())
