"""Kernel statistics (name, calls, total/average ns, %) out of a rocprofv3
SQLite output (rocpd *_results.db), as CSV -- the same columns as the
--stats kernel_stats.csv of the csv output format."""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    rows = c.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
        for r in rows:
            w.writerow(r)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
