"""End-to-end inference throughput (BASELINE config 5): FastSpeech2 eval-mode forward with
predicted durations + HiFi-GAN generator, on one MI355X.

    python bench_infer.py [--batch B] [--src-len T] [--iters K] [--warmup W] [--dtype bf16|f32]

A pass = synthesize.synth_batch on one synthetic text batch resident in HBM (the 8-tuple of
synthesize.py: speakers, phoneme ids, lengths, speaker metadata, accents) -> int16 PCM per
utterance.  Prints one JSON line: generated mel-frames/s, audio samples/s and RTF (wall time
per second of generated audio, lower is better), with the vocoder's share of the pass.
Weights are name-seeded (no checkpoints ship with the reference), with the duration
predictor's output bias set so durations average ~4 frames per phoneme.
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
PKG = importlib.import_module("mid-attribute-speaker-generation_amd")
M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
HG = importlib.import_module("mid-attribute-speaker-generation_amd.hifigan")
SY = importlib.import_module("mid-attribute-speaker-generation_amd.synthesize")
DS = importlib.import_module("mid-attribute-speaker-generation_amd.dataset")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--src-len", type=int, default=128)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--dtype", default="bf16", choices=["f32", "bf16"])
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    cdt = {"f32": torch.float32, "bf16": torch.bfloat16}[args.dtype]
    pp, mc, tc, path = PKG.config.load_configs("JVS-VCTK")
    model = M.FastSpeech2(pp, mc, path, device=dev, compute_dtype=cdt)
    PKG.seeded.load_seeded_(model)
    # random weights predict ~0-1 frame per phoneme; set the duration head's output bias to
    # log(1 + 4) so predicted durations average ~4 frames per phoneme, as in the SYN-B
    # training batches (the rest of the network keeps its name-seeded weights)
    with torch.no_grad():
        model.state_dict()["variance_adaptor.duration_predictor.linear_layer.bias"].fill_(
            float(np.log(5.0)))
    model.eval()
    voc = HG.get_vocoder(device=dev, compute_dtype=cdt)
    b = PKG.data.syn_batch(args.batch, args.src_len, seed=0)
    text = (b[0], b[1], b[2], b[3], b[4], b[5], b[12], b[13])  # synthesize.py batch layout
    batch = DS.to_device(text, dev)
    hop, sr = pp["stft"]["hop_length"], pp["audio"]["sampling_rate"]
    for _ in range(args.warmup):
        SY.synth_batch(model, voc, batch)
    torch.cuda.synchronize()
    frames, t_voc = 0, 0.0
    t0 = time.perf_counter()
    for _ in range(args.iters):
        out, wavs = SY.synth_batch(model, voc, batch)
        frames += int(out[9].sum())
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # vocoder share: the same mel through the generator alone
    post = out[1]
    B, T, C = post.shape
    rows = post.reshape(B * T, C).contiguous()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.iters):
        voc.forward_rows(rows, B, T, lengths=out[9])
    torch.cuda.synchronize()
    t_voc = (time.perf_counter() - t1) / args.iters
    audio_s = frames * hop / sr
    print(json.dumps({
        "metric": "end-to-end synthesis (FastSpeech2 + HiFi-GAN), 1 MI355X",
        "mel_frames_per_s": round(frames / dt, 1),
        "samples_per_s": round(frames * hop / dt, 1),
        "rtf": round(dt / audio_s, 6), "ms_per_batch": round(dt / args.iters * 1e3, 3),
        "vocoder_ms_per_batch": round(t_voc * 1e3, 3),
        "padded_frames_per_batch": int(B * T), "valid_frames_per_batch": frames // args.iters,
        "batch": args.batch, "src_len": args.src_len, "dtype": args.dtype,
        "iters": args.iters, "warmup": args.warmup,
        "data": "synthetic phoneme batch (SYN-B text fields), name-seeded weights"}))


if __name__ == "__main__":
    main()
