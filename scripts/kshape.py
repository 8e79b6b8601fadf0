"""Per-launch-shape summary of a rocprofv3 kernel trace.

    python scripts/kshape.py <kernel_trace.csv | results.db> [steps] [top] [--stats out.csv]

Accepts the CSV kernel trace (`--output-format csv`) or the SQLite database rocprofv3 writes
by default (`-o run` -> `run_results.db`, view `kernels`).  Groups dispatches by (kernel name,
workgroup count) -- one template instantiation serves several GEMM shapes, so the --stats
summary averages unlike launches -- and prints total ms/step, launches/step and the average
duration of each group.  `--stats` also writes the per-kernel-name summary (the same columns
as rocprofv3's `kernel_stats.csv`: Name, Calls, TotalDurationNs, AverageNs, Percentage).

Lines tagged `conv_k9` are the tap-register k=9 convolutions (conv_gemm_tapreg: decoder FFN
forward and data gradient, encoder forward) of the launch set bench.py's `roofline` names (the
encoder's split-K data gradient runs on conv_gemm_halo).
"""
import csv
import sqlite3
import sys
from collections import defaultdict


def load(path):
    """[(name, workgroups, duration_ns)] in dispatch order."""
    if path.endswith(".db"):
        con = sqlite3.connect(path)
        q = ("select name, grid_x*grid_y*grid_z, workgroup_x*workgroup_y*workgroup_z, duration "
             "from kernels order by start")
        return [(n, g // max(w, 1), int(d)) for n, g, w, d in con.execute(q)]
    out = []
    for r in csv.DictReader(open(path)):
        wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        out.append((r["Kernel_Name"], grid // max(wg, 1),
                    int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    return out


def main():
    argv = list(sys.argv[1:])
    stats_out = None
    if "--stats" in argv:
        i = argv.index("--stats")
        stats_out = argv[i + 1]
        del argv[i:i + 2]
    path = argv[0]
    steps = int(argv[1]) if len(argv) > 1 else 7
    top = int(argv[2]) if len(argv) > 2 else 40
    rows = load(path)
    groups = defaultdict(list)
    for name, wgs, dur in rows:
        groups[(name, wgs)].append(dur)
    total = sum(d for _, _, d in rows)
    print(f"kernel time {total / 1e6 / steps:.3f} ms/step over {steps} steps "
          f"({len(rows) / steps:.0f} launches/step)")
    print(f"{'ms/step':>8} {'n/step':>6} {'avg us':>8}  {'wgs':>6}  kernel")
    for (name, wgs), v in sorted(groups.items(), key=lambda kv: -sum(kv[1]))[:top]:
        tag = "  conv_k9" if "conv_gemm_tapreg<" in name and ", 9, " in name else ""
        print(f"{sum(v) / 1e6 / steps:8.3f} {len(v) / steps:6.1f} {sum(v) / len(v) / 1e3:8.1f}  "
              f"{wgs:6d}  {name[:100]}{tag}")
    if stats_out:
        by_name = defaultdict(list)
        for name, _, dur in rows:
            by_name[name].append(dur)
        with open(stats_out, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
            for name, v in sorted(by_name.items(), key=lambda kv: -sum(kv[1])):
                w.writerow([name, len(v), sum(v), f"{sum(v) / len(v):.1f}",
                            f"{100.0 * sum(v) / total:.3f}"])


if __name__ == "__main__":
    main()
