"""Per-launch-shape summary of a rocprofv3 kernel trace.

    python scripts/kshape.py <kernel_trace.csv> [steps] [top]

Groups dispatches by (kernel name, grid size) -- one template instantiation serves several
GEMM shapes, so the --stats summary averages unlike launches -- and prints total ms/step,
launches/step and the average duration of each group.  The line tagged ROOFLINE is the
launch set bench.py's `roofline` times with HIP events: conv_gemm_halo<128,128> with 1,536
workgroups is the decoder FFN Conv1d 256->1024 forward (k=9, K = 2,304), the only launch of
that kernel and grid in the step (the earlier tap-major kernel shared its grid with the k=1
data gradient of w_2, hence the widest-gap split below, kept for traces of that kernel).
"""
import csv
import sys
from collections import defaultdict

ROOF_NAME, ROOF_WGS = "conv_gemm_halo<256, 128, 2, 16, false, 8>", 768


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    groups = defaultdict(list)
    for r in csv.DictReader(open(path)):
        wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        groups[(r["Kernel_Name"], grid // max(wg, 1))].append(dur)
    total = sum(sum(v) for v in groups.values())
    print(f"kernel time {total / 1e6 / steps:.3f} ms/step over {steps} steps")
    print(f"{'ms/step':>8} {'n/step':>6} {'avg us':>8}  {'wgs':>6}  kernel")
    for (name, wgs), v in sorted(groups.items(), key=lambda kv: -sum(kv[1]))[:top]:
        tag = "  ROOFLINE" if ROOF_NAME in name and wgs == ROOF_WGS else ""
        print(f"{sum(v) / 1e6 / steps:8.3f} {len(v) / steps:6.1f} {sum(v) / len(v) / 1e3:8.1f}  "
              f"{wgs:6d}  {name[:90]}{tag}")
    roof = sorted(d for (name, wgs), v in groups.items() if ROOF_NAME in name and wgs == ROOF_WGS
                  for d in v)
    if len(roof) > 1:
        gaps = [roof[i + 1] / roof[i] for i in range(len(roof) - 1)]
        i = max(range(len(gaps)), key=gaps.__getitem__)
        if gaps[i] > 2.0:
            print(f"ROOFLINE group split at {roof[i] / 1e3:.1f} | {roof[i + 1] / 1e3:.1f} us: "
                  f"{i + 1} short launches (k=1 data gradient) dropped")
            roof = roof[i + 1:]
    if roof:
        print(f"ROOFLINE kernel: {len(roof)} launches, average {sum(roof) / len(roof) / 1e6:.4f} ms")


if __name__ == "__main__":
    main()
