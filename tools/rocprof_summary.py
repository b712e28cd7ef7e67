"""Summarise a rocprofv3 results database (kernel-trace) into a plain-text table for profiles/."""
import sqlite3
import sys


def main(db, out=None, top=15):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage "
                          "from top_kernels limit ?", (top,)))
    lines = [f"# rocprofv3 --kernel-trace --stats summary of {db.split('/')[-1]}",
             f"{'calls':>7} {'total_ms':>11} {'avg_us':>10} {'pct':>6}  kernel"]
    for name, calls, tot, avg, pct in rows:
        short = name.split("(")[0][:90]
        lines.append(f"{calls:>7} {tot / 1e3:>11.3f} {avg:>10.3f} {pct:>6.2f}  {short}")
    text = "\n".join(lines) + "\n"
    if out:
        with open(out, "w") as f:
            f.write(text)
    print(text)


if __name__ == "__main__":
    main(*sys.argv[1:3])
