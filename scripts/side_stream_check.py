"""Step time with / without the weight-gradient side stream, and the time from the last
main-stream backward kernel to the side stream's drain (HIP events)."""
import importlib, os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = importlib.import_module("mid-attribute-speaker-generation_amd")
M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
TR = importlib.import_module("mid-attribute-speaker-generation_amd.train")
dev = torch.device("cuda", 0)
pp, mc, tc, path = PKG.config.load_configs("JVS-VCTK")
batch = PKG.data.to_device(PKG.data.syn_batch(48, 128, seed=0), dev)


def run(side, main_prio=None):
    model = M.FastSpeech2(pp, mc, path, device=dev, compute_dtype=torch.bfloat16)
    model.train()
    if not side:
        model.side_stream = lambda: None
    tr = TR.Trainer(model, pp, mc, tc)
    st = torch.cuda.Stream(priority=main_prio) if main_prio is not None else torch.cuda.current_stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        for _ in range(5):
            tr.step(batch)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            tr.step(batch)
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / 20 * 1e3


print("priority range", torch.cuda.Stream.priority_range(), flush=True)
print(f"side stream on : {run(True):.3f} ms/step", flush=True)
lo, hi = torch.cuda.Stream.priority_range()
print(f"side stream on, main stream at priority {hi}: {run(True, hi):.3f} ms/step", flush=True)
print(f"side stream off: {run(False):.3f} ms/step", flush=True)
