"""cfg4 step attribution table from a tools/gpu_ab.sh cfg4tl run of the shipped
library and the cumulative timing-only builds under build/d5 (VERDICT r05
item 1): per build the ms per step of the random-weight L = 0 rollout (the
step's fixed part), of L = 4 and of the W1_r2 workload, averaged over the
repetitions; each row's cost is the drop from the row above, so the rows sum
to the shipped figure by construction and the last row is what no switch
removes.  Markdown on stdout.

    python tools/cfg4_attrib.py TAG [timeline.json [stripped_timeline.json]]

stripped_timeline.json: the lane timeline of the last cumulative build
(tools/cfg4_timeline.py under rocprofv3, HYBRIDFLUX_LIB = that build): what
no switch removes, split into the kernels that still run and the gaps.
"""
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LABELS = {
    "noropiece": "readout epilogue (z = P(i) + Q(i+1) sums, ReLU, w2 dots)",
    "noromfma": "readout MFMAs ([W_a ; W_b] h, 65.5 kFLOP per cell)",
    "noinmfma": "input-layer MFMAs",
    "nofeat": "feature loads + flux stores",
    "nosync": "ring: LDS-DMA issue, its waits, the ring barriers",
    "noseam": "seam trade (publish, reads, waits)",
    "nofvstep": "FV + spectral Poisson kernel (fv_step_fft_kernel)",
    "nods": "weight-fragment ds_reads (4 x b128 per unit per wave)",
    "nofinish": "readout cross-lane sums (readout_finish)",
    "noloc": "stream-cell locate arithmetic (IC, segment cell)",
    "nopark": "park round trip of the L = 0 hand-off",
    "noinput": "input-layer VALU (bf16 hi/lo split, ReLU, packs)",
}


def main(tag, tl=None, strip=None):
    rows = {}
    # tools/gpu_ab.sh cfg4tl names its outputs ab_cfg4tl_<tag>_*, tools/gpu_cfg4_timeline.sh tl_<tag>_*
    files = glob.glob(os.path.join(ROOT, "gpurun_out", f"ab_cfg4tl_{tag}_*.json")) + \
        [f for f in glob.glob(os.path.join(ROOT, "gpurun_out", f"tl_{tag}_*.json"))
         if re.match(rf"tl_{re.escape(tag)}_lib.+_\d+\.json$", os.path.basename(f))]
    for f in files:
        m = re.match(rf"(?:ab_cfg4tl|tl)_{re.escape(tag)}_(.+)_(\d+)\.json$", os.path.basename(f))
        if not m:
            continue
        d = json.load(open(f))
        g = {x["name"]: x["ms_per_step"] for x in d["groups"]}
        rows.setdefault(m.group(1), []).append(g)
    avg = {k: {n: sum(r[n] for r in v) / len(v) for n in v[0]} for k, v in rows.items()}
    chain = sorted((k for k in avg if k.startswith("lib_")), key=lambda k: k.count("+"))
    order = ["libhybridflux"] + chain
    names = ("rand_L0", "rand_L4", "W1_r2")
    print(f"# cfg4 step attribution ({tag}): 4096 ICs x 1024 cells, bf16, T = 30, hf_run's 3 lanes\n")
    print("ms per step (HIP events over 3 back-to-back rollouts after 0.5 s of the same work, "
          f"mean of {len(rows['libhybridflux'])} alternated runs on one box; builds: tools/build_diag5.sh, "
          "timing-only HF_DIAG_* switches, results wrong by construction).  Cumulative: each row removes "
          "one more piece; its cost is the drop from the row above.\n")
    print("| build (cumulative) | removed | L = 0 ms | cost (L = 0) | share of the L = 0 step | L = 4 ms | cost (L = 4) | W1_r2 ms |")
    print("|---|---|---|---|---|---|---|---|")
    base = avg["libhybridflux"]
    prev = base
    for k in order:
        a = avg[k]
        last = k.split("+")[-1].replace("lib_", "") if k != "libhybridflux" else None
        c0 = prev["rand_L0"] - a["rand_L0"] if last else 0.0
        c4 = prev["rand_L4"] - a["rand_L4"] if last else 0.0
        print(f"| {'shipped' if not last else '+ ' + last} | {LABELS.get(last, '-') if last else '-'} | "
              f"{a['rand_L0']:.4f} | {c0:.4f} | {100 * c0 / base['rand_L0']:.1f} % | {a['rand_L4']:.4f} | "
              f"{c4:.4f} | {a['W1_r2']:.4f} |")
        prev = a
    print(f"| left | what no switch removes | {prev['rand_L0']:.4f} | | {100 * prev['rand_L0'] / base['rand_L0']:.1f} % | "
          f"{prev['rand_L4']:.4f} | | {prev['W1_r2']:.4f} |")
    if strip:
        # the best (lowest L = 0) cumulative build: the trace was taken of it
        best = min(order[1:], key=lambda k: avg[k]["rand_L0"])
        r = {x["group"]: x for x in json.load(open(strip))["rows"]}["rand_L0"]
        print(f"\nWhat no switch removes, from the kernel trace of `{best}` at L = 0 (ms per step; HIP-event "
              f"step of that build {avg[best]['rand_L0']:.4f}):\n")
        print("| piece | ms per step | share of the shipped L = 0 step |")
        print("|---|---|---|")
        for name, v in (("flux kernels' skeleton (grid dispatch, wave start, loop control and barriers with "
                         "every piece removed; the three lanes' dispatches overlap)", r["flux_union_ms_per_step"]),
                        ("other kernels exposed", r["exposed_other_ms_per_step"]),
                        ("nothing running", r["idle_ms_per_step"])):
            print(f"| {name} | {v:.4f} | {100 * v / base['rand_L0']:.1f} % |")
        rest = avg[best]["rand_L0"] - r["span_ms_per_step"]
        print(f"| unattributed (that build's HIP-event step less the traced span) | {rest:.4f} | "
              f"{100 * rest / base['rand_L0']:.1f} % |")
    if tl:
        t = json.load(open(tl))
        print("\nLane timeline (rocprofv3 --kernel-trace of the same run, tools/cfg4_timeline.py analyze), ms per step:\n")
        print("| group | wall span | flux kernels' union | sum of flux kernel durations | FV kernels exposed "
              "(no flux kernel running) | other kernels exposed | nothing running |")
        print("|---|---|---|---|---|---|---|")
        for r in t["rows"]:
            print(f"| {r['group']} | {r['span_ms_per_step']} | {r['flux_union_ms_per_step']} | "
                  f"{r['flux_sum_ms_per_step']} | {r['exposed_fv_ms_per_step']} | "
                  f"{r['exposed_other_ms_per_step']} | {r['idle_ms_per_step']} |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None, sys.argv[3] if len(sys.argv) > 3 else None)
