"""Per-step kernel timeline of the training bench from a rocprofv3 kernel
trace (tools/gpu_ab.sh trainks): steps start at each chain_train_fwd_kernel
dispatch; steps with the same kernel sequence are grouped (the bench's arms
differ in their optimizer kernels), and per group every position's median
duration and the median gap before it (the previous dispatch's end to this
one's start: drain, launch, or a host wait) are printed, so that the gaps of
a step are attributed to the kernel boundaries that hold them.

    python tools/train_timeline.py RUN_results.db
"""
import re
import sqlite3
import statistics
import sys


def short(name):
    n = re.sub(r"\(.*", "", name)
    n = re.sub(r"<.*", "", n)
    return n.split("::")[-1][:40]


def main(db):
    rows = sqlite3.connect(db).execute("select name, start, end from kernels order by start").fetchall()
    steps, cur = [], []
    for n, s, e in rows:
        if "chain_train_fwd_kernel" in n and cur:
            steps.append(cur)
            cur = []
        if cur or "chain_train_fwd_kernel" in n:
            cur.append((short(n), s, e))
    groups = {}
    for i, st in enumerate(steps[:-1]):
        nxt = steps[i + 1][0][1]  # the step ends where the next one's forward starts
        groups.setdefault(tuple(k for k, _, _ in st), []).append((st, nxt))
    for sig, lst in sorted(groups.items(), key=lambda kv: -len(kv[1])):
        if len(lst) < 5:
            continue
        span = statistics.median((nxt - st[0][1]) / 1e3 for st, nxt in lst)
        busy = statistics.median(sum(e - s for _, s, e in st) / 1e3 for st, _ in lst)
        print(f"## {len(lst)} steps of {len(sig)} dispatches: median step {span:.1f} us, kernels {busy:.1f} us, "
              f"gaps {span - busy:.1f} us\n")
        print("| # | kernel | median us | median gap before us |")
        print("|---|---|---|---|")
        for p, k in enumerate(sig):
            d = statistics.median((st[p][2] - st[p][1]) / 1e3 for st, _ in lst)
            g = statistics.median(((st[p][1] - st[p - 1][2]) if p else 0) / 1e3 for st, _ in lst)
            print(f"| {p} | {k} | {d:.1f} | {g:.1f} |")
        g_end = statistics.median((nxt - st[-1][2]) / 1e3 for st, nxt in lst)
        print(f"| - | (to the next step's forward) | | {g_end:.1f} |\n")


if __name__ == "__main__":
    main(sys.argv[1])
