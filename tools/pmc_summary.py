"""Per-dispatch PMC values of one kernel from rocprofv3 rocpd databases.

    python tools/pmc_summary.py KERNEL_SUBSTR db1 [db2 ...]
Prints one row per (db, dispatch) with every counter collected for it.
"""
import sqlite3
import sys


def main(sub, paths):
    for p in paths:
        c = sqlite3.connect(p)
        rows = c.execute("select dispatch_id, duration, counter_name, sum(counter_value) from pmc_events "
                         "where name like ? group by dispatch_id, counter_name order by dispatch_id",
                         (f"%{sub}%",)).fetchall()
        by = {}
        for d, dur, name, val in rows:
            by.setdefault((d, dur), {})[name] = val
        for (d, dur), vals in by.items():
            print(p.split("/")[-2], f"dispatch={d}", f"dur_us={dur / 1e3:.1f}",
                  " ".join(f"{k}={v:.6g}" for k, v in sorted(vals.items())))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
