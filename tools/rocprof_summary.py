"""Summarise a rocprofv3 --kernel-trace --stats result (kernel_stats.csv or results .db) into a
plain-text table for profiles/."""
import csv
import sqlite3
import sys


def rows_from(path, top):
    if path.endswith(".csv"):
        with open(path) as f:
            r = list(csv.DictReader(f))
        return [(x["Name"], int(x["Calls"]), float(x["TotalDurationNs"]) / 1e3,
                 float(x["AverageNs"]) / 1e3, float(x["Percentage"])) for x in r[:top]]
    c = sqlite3.connect(path)
    return [(n, calls, tot, avg, pct) for n, calls, tot, avg, pct in
            c.execute("select name, total_calls, total_duration, average, percentage "
                      "from top_kernels limit ?", (top,))]


def main(path, out=None, top=15):
    lines = [f"# rocprofv3 --kernel-trace --stats summary of {path.split('/')[-1]}",
             f"{'calls':>7} {'total_ms':>11} {'avg_us':>10} {'pct':>6}  kernel"]
    for name, calls, tot_us, avg_us, pct in rows_from(path, int(top)):
        short = name.split("(")[0][:90]
        lines.append(f"{calls:>7} {tot_us / 1e3:>11.3f} {avg_us:>10.3f} {pct:>6.2f}  {short}")
    text = "\n".join(lines) + "\n"
    if out:
        with open(out, "w") as f:
            f.write(text)
    print(text)


if __name__ == "__main__":
    main(*sys.argv[1:4])
