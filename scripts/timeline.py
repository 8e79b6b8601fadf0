"""GPU busy/idle anatomy of a rocprofv3 kernel trace of bench.py: per training step (steps end
at adam_kernel), the union of kernel intervals over all streams, the idle time, the share of
time with 2+ kernels in flight, and the largest idle gaps with their neighbours.

    python scripts/timeline.py <kernel_trace.csv> [skip_steps]
"""
import csv
import sys


def main():
    rows = []
    for r in csv.DictReader(open(sys.argv[1])):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70]))
    rows.sort()
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    ends = [e for s, e, n in rows if "adam_kernel" in n]
    bounds = []
    prev = rows[0][0]
    for e in ends:
        bounds.append((prev, e))
        prev = e
    for i, (b0, b1) in enumerate(bounds[skip:], start=skip):
        ks = [(s, e, n) for s, e, n in rows if s >= b0 and e <= b1]
        if not ks:
            continue
        ev = sorted([(s, 1) for s, e, n in ks] + [(e, -1) for s, e, n in ks])
        busy = multi = 0
        depth, last = 0, ev[0][0]
        for t, d in ev:
            if depth >= 1:
                busy += t - last
            if depth >= 2:
                multi += t - last
            depth += d
            last = t
        wall = ks[-1][1] - ks[0][0]
        gaps = []
        cur_end = ks[0][1]
        prevn = ks[0][2]
        for s, e, n in ks[1:]:
            if s > cur_end:
                gaps.append((s - cur_end, prevn, n))
            if e > cur_end:
                cur_end, prevn = e, n
        gaps.sort(reverse=True)
        print(f"step {i}: wall {wall / 1e3:.1f} us, busy {busy / 1e3:.1f} us, idle {(wall - busy) / 1e3:.1f} us "
              f"in {len(gaps)} gaps, 2+ kernels {multi / 1e3:.1f} us, kernels {len(ks)}, "
              f"sum of kernel times {sum(e - s for s, e, n in ks) / 1e3:.1f} us")
        for g, a, b in gaps[:8]:
            print(f"     gap {g / 1e3:6.1f} us  after {a[:55]}  before {b[:55]}")
        hist = {}
        for g, a, b in gaps:
            k = "<2us" if g < 2000 else "2-5us" if g < 5000 else "5-20us" if g < 20000 else ">20us"
            hist[k] = hist.get(k, 0) + g
        print("     idle by gap size:", {k: round(v / 1e3, 1) for k, v in hist.items()})


if __name__ == "__main__":
    main()
