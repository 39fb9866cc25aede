"""Per-dispatch PMC values of one kernel from rocprofv3 rocpd databases.

    python tools/pmc_summary.py KERNEL_SUBSTR db1 [db2 ...]
Prints one row per (db, dispatch) with every counter collected for it, then
per db the totals over those dispatches and, where the counters allow, the
derived rates: MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMDs x CUs x
GRBM_GUI_ACTIVE / 8 XCDs)), the effective clock (GRBM_GUI_ACTIVE / 8 / kernel
time, MI355X_MICROARCH.md DVFS item) and non-MFMA VALU per MFMA.
"""
CUS = 256
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
        tot, tdur = {}, 0.0
        for (d, dur), vals in by.items():
            print(p.split("/")[-2], f"dispatch={d}", f"dur_us={dur / 1e3:.1f}",
                  " ".join(f"{k}={v:.6g}" for k, v in sorted(vals.items())))
            tdur += dur
            for k, v in vals.items():
                tot[k] = tot.get(k, 0.0) + v
        if not tot:
            continue
        der = []
        if "GRBM_GUI_ACTIVE" in tot:
            gui = tot["GRBM_GUI_ACTIVE"] / 8
            der.append(f"clock_GHz={gui / tdur:.3f}")
            if "SQ_VALU_MFMA_BUSY_CYCLES" in tot:
                der.append(f"mfma_busy={tot['SQ_VALU_MFMA_BUSY_CYCLES'] / (4 * CUS * gui):.4f}")
        if "SQ_INSTS_MFMA" in tot and "SQ_INSTS_VALU" in tot:
            if tot['SQ_INSTS_MFMA'] > 0:
                der.append(f"nonmfma_valu_per_mfma={(tot['SQ_INSTS_VALU'] - tot['SQ_INSTS_MFMA']) / tot['SQ_INSTS_MFMA']:.3f}")
        print(p.split("/")[-2], "TOTAL", f"dispatches={len(by)}", f"dur_us={tdur / 1e3:.1f}",
              " ".join(f"{k}={v:.6g}" for k, v in sorted(tot.items())), *der)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
