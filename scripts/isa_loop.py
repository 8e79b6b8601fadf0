"""Compact listing of a kernel's memory / MFMA / sync skeleton from a device .s file
(runs of MFMAs, ds_reads and LDS-DMA loads collapsed), to check a k-loop's schedule.

    hipcc -O3 -std=c++17 --offload-arch=gfx950 --offload-device-only -S x.hip -o x.s
    python scripts/isa_loop.py x.s <mangled-name substring>
"""
import sys

KEEP = ("v_mfma", "ds_read", "ds_write", "s_barrier", "s_waitcnt", "global_load", "buffer_load",
        "s_cbranch", "s_branch", "global_store", "s_setprio", "s_endpgm")


def main():
    path, key = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, ln in enumerate(lines) if ln.startswith("_Z") and key in ln and ln.split(":")[0].endswith(key.split()[-1]) or (ln.startswith("_Z") and ln.split(":")[0] == key))
    out, prev, n, last = [], None, 0, None

    def flush():
        if prev:
            out.append(f"{last}  x{n}" if n > 1 else last)

    for ln in lines[start + 1:]:
        t = ln.strip()
        if t.startswith(".Lfunc_end"):
            break
        if t.startswith(".LBB"):
            flush()
            prev, n, last = None, 0, None
            out.append(t)
            continue
        if not t or t[0] in ";.":
            continue
        op = t.split()[0]
        if not op.startswith(KEEP):
            continue
        fam = op if not op.startswith(("v_mfma", "ds_read", "global_load_lds")) else op.split("_b")[0]
        if fam == prev and op.startswith(("v_mfma", "ds_read", "global_load_lds")):
            n += 1
        else:
            flush()
            prev, n, last = fam, 1, t[:70]
    flush()
    print("\n".join(out))


if __name__ == "__main__":
    main()
