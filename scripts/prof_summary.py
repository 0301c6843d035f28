"""Summarise a rocprofv3 rocpd database (``--kernel-trace --stats`` output) into a compact markdown table.

usage: python scripts/prof_summary.py gpurun_out/prof/bench_results.db > profiles/<name>.md
"""
import re
import sqlite3
import sys


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name) if not name.startswith("void at::") else name.split("<")[0]
    return name.replace("void ", "")[:110]


def main(path: str) -> None:
    c = sqlite3.connect(f"file:{path}?mode=ro", uri=True)  # never creates a database
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    print(f"# rocprofv3 kernel summary: `{path.split('/')[-1]}`\n")
    print("| kernel | calls | total (us) | avg (us) | % |")
    print("|---|---:|---:|---:|---:|")
    for name, calls, tot, avg, pct in rows[:25]:
        print(f"| `{short(name)}` | {calls} | {tot / 1e3 if tot > 1e6 else tot:.1f} | {avg / 1e3 if avg > 1e6 else avg:.1f} | {pct:.1f} |")
    try:
        q = ("select name, count(*), sum(end-start), avg(end-start), max(grid_x), max(workgroup_x), max(vgpr_count), "
             "max(sgpr_count), max(lds_size) from kernels group by name order by sum(end-start) desc limit 12")
        print("\n| kernel | calls | total (us) | avg (us) | grid (threads) | wg | VGPR | SGPR | LDS |")
        print("|---|---:|---:|---:|---:|---:|---:|---:|---:|")
        for name, n, tot, avg, gx, wg, vg, sg, lds in c.execute(q):
            print(f"| `{short(name)}` | {n} | {tot / 1e3:.1f} | {avg / 1e3:.1f} | {gx} | {wg} | {vg} | {sg} | {lds} |")
    except sqlite3.Error as e:  # older schema
        print(f"\n(kernels view unavailable: {e})")
    try:
        q = "select count(*), sum(end-start), sum(size) from memory_copies"
        n, tot, size = next(c.execute(q))
        if n:
            print(f"\nmemory copies: {n} calls, {tot / 1e3:.1f} us, {size / 2**20:.1f} MiB")
    except sqlite3.Error:
        pass


if __name__ == "__main__":
    if len(sys.argv) != 2 or sys.argv[1].startswith("-"):
        sys.exit(__doc__)
    main(sys.argv[1])
