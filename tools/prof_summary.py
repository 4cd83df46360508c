#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats database (run_results.db) into
the per-kernel table committed under profiles/ (calls, total/avg/min/max us, %)."""
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    with open(out, "w") as f:
        f.write("| kernel | calls | total us | avg us | min us | max us | % |\n|---|---|---|---|---|---|---|\n")
        for name, n, s, a, lo, hi in rows:
            short = name.split("(")[0]
            f.write("| %s | %d | %.1f | %.2f | %.2f | %.2f | %.1f |\n" % (short, n, s / 1e3, a / 1e3, lo / 1e3, hi / 1e3,
                                                                        100.0 * s / tot))
    print(open(out).read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
