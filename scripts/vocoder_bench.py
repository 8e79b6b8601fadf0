"""Vocoder alone (B=16 x 1559 frames, lengths 500): length-aware forward_rows time."""
import importlib, os, sys, torch
sys.path.insert(0, os.getcwd())
HG = importlib.import_module("mid-attribute-speaker-generation_amd.hifigan")
gen = HG.get_vocoder(device="cuda")
B, T = 16, 1559
mel = torch.randn(B * T, 80, device="cuda")
lens = torch.full((B,), 500, dtype=torch.int64, device="cuda")
for _ in range(2): gen.forward_rows(mel, B, T, lengths=lens)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(5): gen.forward_rows(mel, B, T, lengths=lens)
e.record(); torch.cuda.synchronize()
print("vocoder ms", s.elapsed_time(e) / 5, flush=True)
