"""PostNet BatchNorm forward/backward alone at the SYN-48 shapes (24,576 rows x 512, and the
80-channel last layer), p = 0.5 dropout and tanh as in the step."""
import importlib, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("mid-attribute-speaker-generation_amd.kernels")
dev = "cuda:0"
M = 24576
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


for C, act in ((512, True), (80, False)):
    z = torch.randn(M, C, device=dev)
    g, b = torch.ones(C, device=dev), torch.zeros(C, device=dev)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    out, out_t, mean, rstd = K.bn_fwd(z, g, b, rm, rv, act, 0.5, seed, 5, copy=torch.bfloat16)
    t = timeit(lambda: K.bn_fwd(z, g, b, rm, rv, act, 0.5, seed, 5, copy=torch.bfloat16))
    print(f"c={C:4d} bn_fwd  {t:7.1f} us")
    dout = torch.randn(M, C, device=dev)
    dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    t = timeit(lambda: K.bn_bwd(dout, z, mean, rstd, g, b, dg, db, act, 0.5, seed, 5,
                                copy=torch.bfloat16))
    print(f"c={C:4d} bn_bwd  {t:7.1f} us")
