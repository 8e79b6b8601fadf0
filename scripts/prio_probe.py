"""Stream-priority probe: torch's and HIP's priority ranges on this device."""
import ctypes
import torch

print("torch priority_range", torch.cuda.Stream.priority_range())
hip = ctypes.CDLL("libamdhip64.so")
lo, hi = ctypes.c_int(), ctypes.c_int()
print("hipDeviceGetStreamPriorityRange rc", hip.hipDeviceGetStreamPriorityRange(ctypes.byref(lo), ctypes.byref(hi)),
      "least", lo.value, "greatest", hi.value)
for p in (-2, -1, 0, 1):
    s = torch.cuda.Stream(priority=p)
    print("requested", p, "got", s.priority)
