"""PostNet BatchNorm forward/backward alone at the SYN-48 shape (24,576 rows x 512)."""
import importlib, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("mid-attribute-speaker-generation_amd.kernels")
dev = "cuda:0"
M, C = 24576, 512
z = torch.randn(M, C, device=dev)
g, b = torch.ones(C, device=dev), torch.zeros(C, device=dev)
rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
seed = torch.tensor([3], dtype=torch.int64, device=dev)


def timeit(run, n=30):
    for _ in range(3):
        run()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        run()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


out, out_t, mean, rstd = K.bn_fwd(z, g, b, rm, rv, True, 0.5, seed, 5, copy=torch.bfloat16)
print(f"bn_fwd  {timeit(lambda: K.bn_fwd(z, g, b, rm, rv, True, 0.5, seed, 5, copy=torch.bfloat16)):7.1f} us")
dout = torch.randn(M, C, device=dev)
dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
print(f"bn_bwd  {timeit(lambda: K.bn_bwd(dout, z, mean, rstd, g, b, dg, db, True, 0.5, seed, 5, copy=torch.bfloat16)):7.1f} us")
