#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--stats`` kernel_stats.csv into a markdown table (for profiles/)."""
import csv
import sys


def _rows_from_db(path):
    """rocprofv3 7.x writes a rocpd SQLite database; its ``top_kernels`` view has µs totals."""
    import sqlite3
    c = sqlite3.connect(path)
    return [{"Name": n, "TotalDurationNs": t * 1e3, "Calls": k}
            for n, k, t in c.execute("select name, total_calls, total_duration from top_kernels")]


def main(path, title="", steps=None, top=40):
    rows = _rows_from_db(path) if path.endswith(".db") else list(csv.DictReader(open(path)))
    key_t = next(k for k in rows[0] if "TotalDuration" in k)
    key_c = next(k for k in rows[0] if k.lower() == "calls")
    tot = sum(float(r[key_t]) for r in rows)
    print(f"# {title}\n")
    print(f"Total kernel time: {tot / 1e6:.1f} ms" + (f" over {steps} steps ({tot / 1e6 / steps:.1f} ms/step)" if steps else ""))
    print("\n| ms total | % | calls | avg us | kernel |\n|---|---|---|---|---|")
    for r in sorted(rows, key=lambda r: -float(r[key_t]))[:top]:
        t = float(r[key_t])
        n = int(r[key_c])
        print(f"| {t / 1e6:.2f} | {100 * t / tot:.1f} | {n} | {t / 1e3 / max(n, 1):.1f} | `{r['Name'][:100]}` |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "", int(sys.argv[3]) if len(sys.argv) > 3 else None)
