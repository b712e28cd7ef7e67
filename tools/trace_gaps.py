"""Idle-gap analysis of one VGP training step from a rocprofv3 --kernel-trace CSV: the step is the
run of kernels between two Adam updates; reports span, GPU-busy union, biggest gaps, per-queue
busy time and the top kernels by time."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"])
            for r in rows)
ends = [i for i, k in enumerate(ks) if "adam" in k[2].lower()]
starts = [ends[i] for i in range(1, len(ends)) if ends[i] - ends[i - 1] > 1]
s0, s1 = starts[-2] + 1, starts[-1]
step = ks[s0:s1 + 2]
t0, t1 = step[0][0], max(e for _, e, _, _ in step)
busy, cs, ce = 0, None, None
for s, e, _, _ in step:
    if ce is None or s > ce:
        if ce is not None:
            busy += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
print(f"step span {(t1 - t0) / 1e6:.3f} ms, GPU busy (union) {busy / 1e6:.3f} ms, kernels {len(step)}")
gaps, pe, pn = [], step[0][1], step[0][2]
for s, e, n, _ in step[1:]:
    if s > pe:
        gaps.append(((s - pe) / 1e3, pn[:60], n[:60]))
    if e > pe:
        pe, pn = e, n
gaps.sort(reverse=True)
for g in gaps[:12]:
    print(f"gap {g[0]:8.1f} us  after {g[1]}  ->  {g[2]}")
print(f"sum of gaps {sum(g[0] for g in gaps):.1f} us over {len(gaps)} gaps")
q = collections.defaultdict(float)
kt = collections.defaultdict(lambda: [0.0, 0])
for s, e, n, qq in step:
    q[qq] += (e - s) / 1e6
    key = n.split("(")[0][:70]
    kt[key][0] += (e - s) / 1e6
    kt[key][1] += 1
print("per-queue busy ms", dict(q))
for k, (t, c) in sorted(kt.items(), key=lambda kv: -kv[1][0])[:14]:
    print(f"  {t:7.3f} ms  {c:4d}x  {k}")
