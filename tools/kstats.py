"""Summarise a rocprofv3 results database (kernel name -> calls, total/avg us)."""
import sqlite3
import sys


def main(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, count(*), sum(end-start), avg(end-start) from kernels group by {name} "
                     "order by sum(end-start) desc").fetchall()
    tot = sum(r[2] for r in rows)
    print(f"{'kernel':80s} {'calls':>7s} {'total_ms':>10s} {'avg_us':>10s} {'pct':>6s}")
    for n, k, s, a in rows:
        print(f"{n[:80]:80s} {k:7d} {s/1e6:10.3f} {a/1e3:10.2f} {100*s/tot:6.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
