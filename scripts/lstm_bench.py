"""One LSTM layer (N=192 sequences x 150 steps, H=256) forward / backward alone."""
import importlib, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("mid-attribute-speaker-generation_amd.kernels")
from importlib import import_module
lib = import_module("mid-attribute-speaker-generation_amd._lib").lib
dev = "cuda:0"
N, T, H, D = 192, 150, 256, 256
x = torch.randn(N * T, D, device=dev)
w_ih = torch.randn(4 * H, D, device=dev) * 0.05
w_hh = torch.randn(4 * H, H, device=dev) * 0.05
bias = torch.randn(4 * H, device=dev) * 0.05
w_hh_t = w_hh.t().contiguous()
w_ih_t = w_ih.t().contiguous()
gx = torch.empty(N * T, 4 * H, device=dev)
h = torch.empty(N * T, H, device=dev)
c = torch.empty(N * T, H, device=dev)
act = torch.empty(N * T, 4 * H, device=dev)
dh = torch.randn(N * T, H, device=dev) * 0.01
dg = torch.empty(N * T, 4 * H, device=dev)
dc = torch.empty(2 * N * H, device=dev)
dx = torch.empty(N * T, D, device=dev)
P = lambda t: t.data_ptr()


def fwd():
    lib.fs2_lstm_layer_fwd(P(x), N, T, D, H, P(w_ih), P(bias), P(w_hh), P(gx), P(h), P(c), P(act), K.stream())


def bwd():
    lib.fs2_lstm_layer_bwd(P(dh), N, T, D, H, P(w_ih_t), P(w_hh_t), P(act), P(c), P(dg), P(dc), P(dx), K.stream())


def timeit(run, n=5):
    run()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        run()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


if os.environ.get("LSTM_PROBE"):  # PMC probe: only the stacked kernels, a few launches
    L = 3
    w_ih_up = torch.randn(L - 1, 4 * H, H, device=dev) * 0.05
    w_hh3 = torch.randn(L, 4 * H, H, device=dev) * 0.05
    bias3 = torch.randn(L, 4 * H, device=dev) * 0.05
    w_ih_up_t, w_hh3_t = w_ih_up.transpose(1, 2).contiguous(), w_hh3.transpose(1, 2).contiguous()
    h3, c3 = torch.empty(L, N * T, H, device=dev), torch.empty(L, N * T, H, device=dev)
    act3, dg3 = torch.empty(L, N * T, 4 * H, device=dev), torch.empty(L, N * T, 4 * H, device=dev)
    dc3 = torch.empty(L * 2 * N * H, device=dev)
    lib.fs2_lstm_stack_fwd(P(x), N, T, D, H, L, P(w_ih), P(w_ih_up), P(w_hh3), P(bias3), P(gx),
                           P(h3), P(c3), P(act3), K.stream())
    lib.fs2_lstm_stack_bwd(P(dh), N, T, D, H, L, P(w_ih_t), P(w_ih_up_t), P(w_hh3_t), P(act3),
                           P(c3), P(dg3), P(dc3), P(dx), K.stream())
    torch.cuda.synchronize()
    sys.exit(0)

# reference: torch LSTM cell recurrence (fp32) on the same weights, for a correctness check
fwd()
torch.cuda.synchronize()
lstm = torch.nn.LSTM(D, H, batch_first=True).to(dev)
with torch.no_grad():
    lstm.weight_ih_l0.copy_(w_ih); lstm.weight_hh_l0.copy_(w_hh)
    lstm.bias_ih_l0.copy_(bias); lstm.bias_hh_l0.zero_()
xr = x.view(N, T, D).clone().requires_grad_(True)
ref, _ = lstm(xr)
print("fwd max abs err vs torch", (h.view(N, T, H) - ref.detach()).abs().max().item(), flush=True)
ref.backward(dh.view(N, T, H))
bwd()
torch.cuda.synchronize()
print("bwd dx max abs err vs torch", (dx.view(N, T, D) - xr.grad).abs().max().item(),
      "ref max", xr.grad.abs().max().item(), flush=True)
print(f"layer fwd {timeit(fwd):.3f} ms, bwd {timeit(bwd):.3f} ms", flush=True)


# the 3-layer stack: per-layer path vs the wavefront entry points
L = 3
w_ih_up = torch.randn(L - 1, 4 * H, H, device=dev) * 0.05
w_hh3 = torch.randn(L, 4 * H, H, device=dev) * 0.05
bias3 = torch.randn(L, 4 * H, device=dev) * 0.05
w_ih_up_t, w_hh3_t = w_ih_up.transpose(1, 2).contiguous(), w_hh3.transpose(1, 2).contiguous()
h3, c3 = torch.empty(L, N * T, H, device=dev), torch.empty(L, N * T, H, device=dev)
act3, dg3 = torch.empty(L, N * T, 4 * H, device=dev), torch.empty(L, N * T, 4 * H, device=dev)
dc3 = torch.empty(L * 2 * N * H, device=dev)
dh3 = torch.randn(N * T, H, device=dev) * 0.01


def sfwd():
    lib.fs2_lstm_stack_fwd(P(x), N, T, D, H, L, P(w_ih), P(w_ih_up), P(w_hh3), P(bias3), P(gx),
                           P(h3), P(c3), P(act3), K.stream())


def sbwd():
    lib.fs2_lstm_stack_bwd(P(dh3), N, T, D, H, L, P(w_ih_t), P(w_ih_up_t), P(w_hh3_t), P(act3),
                           P(c3), P(dg3), P(dc3), P(dx), K.stream())


print(f"3-layer stack (wavefront): fwd {timeit(sfwd):.3f} ms, bwd {timeit(sbwd):.3f} ms "
      f"(per-layer path: about 3x the layer times above plus 4 GEMMs)", flush=True)
