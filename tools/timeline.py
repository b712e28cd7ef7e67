"""Per-launch timeline of one step from a rocprofv3 --kernel-trace CSV (kernel_trace.csv).

    python tools/timeline.py <kernel_trace.csv> [--marker adam_kernel] [--step -2] [--top 0]

A step ends at each launch whose name contains --marker; --step picks which step (Python index
over the steps found, default the second to last).  Prints every launch of that step in start
order: start offset, duration, gap since the previous launch on the same queue, queue, grid, name;
then the step's wall time, the busy time (union of launch intervals) and the per-kernel totals."""
import argparse
import csv
from collections import defaultdict


def col(row, *names):
    for n in names:
        if n in row:
            return row[n]
    raise KeyError(names)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--marker", default="adam_kernel")
    ap.add_argument("--step", type=int, default=-2)
    ap.add_argument("--top", type=int, default=0, help="print only the N longest launches")
    a = ap.parse_args()
    with open(a.csv) as f:
        rows = list(csv.DictReader(f))
    ev = []
    for r in rows:
        name = col(r, "Kernel_Name", "Name")
        t0 = int(col(r, "Start_Timestamp", "Begin_Ns"))
        t1 = int(col(r, "End_Timestamp", "End_Ns"))
        q = col(r, "Queue_Id", "Stream_Id")
        g = "x".join(str(r.get(k, "")) for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))
        ev.append((t0, t1, q, g, name.split("(")[0].replace("void ", "")[:80]))
    ev.sort()
    ends = [i for i, e in enumerate(ev) if a.marker in e[4]]
    if len(ends) < 2:
        raise SystemExit(f"fewer than two '{a.marker}' launches")
    bounds = list(zip([-1] + ends[:-1], ends))
    lo, hi = bounds[a.step]
    step = ev[lo + 1: hi + 1]
    base = step[0][0]
    last_end = defaultdict(lambda: None)
    lines = []
    for t0, t1, q, g, name in step:
        gap = (t0 - last_end[q]) / 1e3 if last_end[q] is not None else 0.0
        last_end[q] = t1
        lines.append(((t1 - t0), f"{(t0 - base) / 1e3:9.1f} {(t1 - t0) / 1e3:8.1f} {gap:7.1f} "
                                 f"{q:>4} {g:>16}  {name}"))
    hdr = f"{'start_us':>9} {'dur_us':>8} {'gap_us':>7} {'q':>4} {'grid':>16}  kernel"
    print(hdr)
    sel = sorted(lines, key=lambda x: -x[0])[:a.top] if a.top else lines
    for _, s in sel:
        print(s)
    wall = (max(e[1] for e in step) - base) / 1e3
    busy, cur0, cur1 = 0, None, None
    for t0, t1, *_ in step:
        if cur1 is None or t0 > cur1:
            if cur1 is not None:
                busy += cur1 - cur0
            cur0, cur1 = t0, t1
        else:
            cur1 = max(cur1, t1)
    busy += cur1 - cur0
    tot = defaultdict(lambda: [0, 0.0])
    for t0, t1, q, g, name in step:
        tot[name][0] += 1
        tot[name][1] += (t1 - t0) / 1e3
    print(f"\nstep: {len(step)} launches, wall {wall:.1f} us, busy (union) {busy / 1e3:.1f} us, "
          f"idle {wall - busy / 1e3:.1f} us")
    for name, (n, us) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"{n:5d} {us:10.1f} us  {name}")


if __name__ == "__main__":
    main()
