"""Summarise a rocprofv3 rocpd database (kernel trace) into a per-kernel table.

    python tools/rocpd_summary.py gpurun_out/prof_r01/bench_results.db > profiles/r01_kernel_stats.md
"""
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    rows = c.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
        "max(vgpr_count), max(accum_vgpr_count), max(sgpr_count), max(lds_size), max(grid_x), max(workgroup_x) "
        "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    print(f"# rocprofv3 --kernel-trace --stats summary: `{path}`\n")
    print("| kernel | calls | total ms | avg us | min us | max us | % | VGPR | AGPR | SGPR | LDS B | grid | wg |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|---|")
    for name, n, tot, avg, mn, mx, v, a, s, lds, gx, wx in rows:
        short = name.replace("(anonymous namespace)::", "").split("(")[0]
        print(f"| `{short}` | {n} | {tot / 1e6:.3f} | {avg / 1e3:.1f} | {mn / 1e3:.1f} | {mx / 1e3:.1f} | "
              f"{100 * tot / total:.2f} | {v} | {a} | {s} | {lds} | {gx} | {wx} |")
    print("\nDispatches of the top kernel (us):",
          ", ".join(f"{d / 1e3:.1f}" for (d,) in c.execute(
              "select duration from kernels where name = ? order by start", (rows[0][0],))))


if __name__ == "__main__":
    main(sys.argv[1])
