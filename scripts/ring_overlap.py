"""Overlap of socket I/O, staging copies and kernels in a device-ring all-reduce, from one rocprofv3 run:

    PCCL_ROCTX_IO=1 rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --output-format csv -d DIR -o ring \\
        -- python3 bench.py --quick --steps 2 --warmup 1
    python scripts/ring_overlap.py DIR/ring > profiles/<name>.md

Inside the window of the large all-reduces (roctx ranges "pccl all_reduce ... bytes >= 256 MiB") it takes the union
over all threads / queues of: H2D staging copies (copy engine), the fused reduce kernels (k_reduce_copy), D2H blit
kernels (step-0 payload), socket sends and receives (roctx "send" / "recv" ranges, PCCL_ROCTX_IO=1), and reports the
busy fraction of each and of their pairwise intersections: the pipeline overlaps when sends / receives run while copies
and kernels run.
"""
import csv
import glob
import sys


def intervals_union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def length(u):
    return sum(e - s for s, e in u)


def intersect(a, b):
    i = j = 0
    out = []
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if e > s:
            out.append([s, e])
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def rows(path):
    files = glob.glob(path)
    if not files:
        return []
    with open(files[0]) as f:
        return list(csv.DictReader(f))


def main(prefix):
    marks = rows(prefix + "_marker_api_trace.csv")
    kern = rows(prefix + "_kernel_trace.csv")
    copies = rows(prefix + "_memory_copy_trace.csv")
    ops = []
    for r in marks:
        name = r["Function"]
        if name.startswith("pccl all_reduce") and "bytes" in name:
            nbytes = int(name.rsplit("bytes", 1)[1].split()[0])
            if nbytes >= (256 << 20):
                ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    if not ops:
        print("no large all-reduce ranges found")
        return
    win_u = intervals_union(ops)  # time covered by at least one large op (gaps between ops excluded)
    cat = {"H2D copies": [], "reduce kernels": [], "D2H blit kernels": [], "socket sends": [], "socket receives": []}
    for r in copies:
        if "HOST_TO_DEVICE" in r.get("Direction", "") + r.get("Kind", ""):
            cat["H2D copies"].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for r in kern:
        n = r["Kernel_Name"]
        iv = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
        if "reduce" in n:
            cat["reduce kernels"].append(iv)
        elif "copyBuffer" in n:
            cat["D2H blit kernels"].append(iv)
    for r in marks:
        if r["Function"] in ("send", "recv"):
            key = "socket sends" if r["Function"] == "send" else "socket receives"
            cat[key].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    win = length(win_u)
    u = {k: intersect(intervals_union(v), win_u) for k, v in cat.items()}
    print(f"# Device-ring overlap: {len(ops)} op ranges (all peers), {win / 1e6:.1f} ms inside ops\n")
    print("| activity | intervals | busy (union) | share of window |")
    print("|---|---:|---:|---:|")
    for k, v in u.items():
        print(f"| {k} | {len(cat[k])} | {length(v) / 1e6:.1f} ms | {100 * length(v) / win:.0f}% |")
    print("\n| overlap (both busy at once) | ms | share of window |")
    print("|---|---:|---:|")
    keys = list(u)
    for i in range(len(keys)):
        for j in range(i + 1, len(keys)):
            ov = length(intersect(u[keys[i]], u[keys[j]]))
            print(f"| {keys[i]} & {keys[j]} | {ov / 1e6:.1f} | {100 * ov / win:.0f}% |")
    gpu = intervals_union([iv for k in ("H2D copies", "reduce kernels", "D2H blit kernels") for iv in u[k]])
    net = intervals_union(u["socket sends"] + u["socket receives"])
    both = length(intersect(gpu, net))
    print(f"\nGPU/PCIe work (copies or kernels) busy {100 * length(gpu) / win:.0f}% of the window, socket I/O busy "
          f"{100 * length(net) / win:.0f}%, both at once {100 * both / win:.0f}%.")


if __name__ == "__main__":
    main(sys.argv[1])
