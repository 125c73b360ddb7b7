"""Export the kernel dispatches of a rocprofv3 SQLite result (``run_results.db``, the default
output format of this ROCm) to the ``kernel_trace.csv`` columns ``tools/analyze_trace.py`` reads:
Kernel_Name, Start_Timestamp, End_Timestamp, Stream_Id, Grid_Size_X/Y/Z, Workgroup_Size_X."""
import csv
import sqlite3
import sys


def main(db: str, out: str) -> None:
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, stream_id, grid_x, grid_y, grid_z, workgroup_x "
                     "from kernels order by start").fetchall()
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Stream_Id", "Grid_Size_X",
                    "Grid_Size_Y", "Grid_Size_Z", "Workgroup_Size_X"])
        w.writerows(rows)
    print(f"{len(rows)} dispatches -> {out}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
