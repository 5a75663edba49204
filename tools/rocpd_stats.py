# SPDX-License-Identifier: BSD-3-Clause
"""The kernel statistics of a rocprofv3 --kernel-trace --stats run written
as a rocpd database (ROCm 7's default output), as CSV: rocprofv3's own
top_kernels view (name, calls, total and average duration in
microseconds, percentage).

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db > profiles/x_kernel_stats.csv
"""
import csv
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
    for name, calls, total, avg, pct in db.execute(
            "select name, total_calls, total_duration, average, percentage from top_kernels"):
        w.writerow([name, calls, round(float(total), 3), round(float(avg), 3), round(float(pct), 3)])


if __name__ == "__main__":
    main()
