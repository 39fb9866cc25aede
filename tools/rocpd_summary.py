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
    # the bench line's headline kernel (cfg3 f32 rollout), whatever its rank in
    # the table: its dispatches in launch order are warmup, TIMED, next rollout,
    # then the radii lines' warmup + rollout pairs (bench.py)
    head = [(n, d) for n, d in c.execute("select name, duration from kernels order by start")
            if "chain_rollout_kernel" in n and "CoreF32T<2, 4, false, true>" in n.replace("(anonymous namespace)::", "")]
    if head:
        print("\nDispatches of the headline kernel `chain_rollout_kernel<CoreF32T<2, 4, false, true>, 4>` "
              "in launch order (us; bench.py: warmup, timed, next rollout, then the radii's warmup + rollout pairs):",
              ", ".join(f"{d / 1e3:.1f}" for _, d in head))


if __name__ == "__main__":
    main(sys.argv[1])
