"""Per-step breakdown of the quantized device ring from PCCL_TRACE_OPS=1 stderr (lane 0, which runs on the op thread).

    python profiles/scripts_archive/quant_trace_breakdown.py qtrace.err [--world 8] [--last-ops 3]

Marks per step g (0 .. 2(W-1)-1): q<g> own payload quantized and published (reduce-scatter steps and the all-gather's
first step), f<g> first received piece consumed, rs<g> / ag<g-(W-1)> step complete. Prints, per step, the median over
peers and ops of: prev-end -> q (metadata fold + quantize launch), q (or prev-end) -> f (waiting for the upstream's
first piece), f -> end (rest of the step's receive), and the whole step.
"""
import argparse
import re
import statistics


def parse(path):
    ops = []
    for ln in open(path, errors="replace"):
        if "[pccl-trace]" not in ln or " ok " not in ln:
            continue
        head, _, rest = ln.partition(" ok ")
        tag = int(re.search(r"tag (\d+)", head).group(1))
        marks = dict((m.group(1), float(m.group(2))) for m in re.finditer(r"(\w+) ([\d.]+)us", rest))
        ops.append((tag, marks))
    return ops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--last-ops", type=int, default=3)
    a = ap.parse_args()
    ops = parse(a.path)
    tags = sorted({t for t, _ in ops})[-a.last_ops:]
    W = a.world
    n = 2 * (W - 1)
    rows = {g: {"meta": [], "wait": [], "rest": [], "step": []} for g in range(n)}
    totals = []
    for t, m in ops:
        if t not in tags:
            continue
        prev = m.get("commence", 0.0)
        start = prev
        for g in range(n):
            end = m.get(f"rs{g}" if g < W - 1 else f"ag{g - (W - 1)}")
            if end is None:
                break
            q, f = m.get(f"q{g}"), m.get(f"f{g}")
            if q is not None:
                rows[g]["meta"].append(q - prev)
            if f is not None:
                rows[g]["wait"].append(f - (q if q is not None else prev))
                rows[g]["rest"].append(end - f)
            rows[g]["step"].append(end - prev)
            prev = end
        totals.append(prev - start)
    med = lambda v: statistics.median(v) if v else float("nan")  # noqa: E731
    print(f"ops {tags}, {len(totals)} peer-op traces, commence -> last step: median {med(totals) / 1e3:.1f} ms")
    print("| step | kind | end -> q (ms) | -> first piece (ms) | first piece -> end (ms) | step (ms) |")
    print("|---:|---|---:|---:|---:|---:|")
    for g in range(n):
        r = rows[g]
        print(f"| {g} | {'RS' if g < W - 1 else 'AG'} | {med(r['meta']) / 1e3:.2f} | {med(r['wait']) / 1e3:.2f} | "
              f"{med(r['rest']) / 1e3:.2f} | {med(r['step']) / 1e3:.2f} |")


if __name__ == "__main__":
    main()
