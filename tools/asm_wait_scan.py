"""Static scan of the library's device code for load-latency hazards the
compiler introduces: per kernel, the global/buffer loads (not LDS-DMA) waited
with s_waitcnt vmcnt(0) within three instructions of their issue, the
compiler-inserted vmcnt(0) waits inside loops (inline-asm waits excluded: a
vmcnt(0) also waits out the ring's hidden LDS-DMA), and scratch (spill) ops.

    python tools/asm_wait_scan.py [file.hip ...]     (default: every csrc/*.hip)

Compiles each file for gfx950 with the Makefile's flags (device code only, -S)
into /tmp and prints one line per kernel that has MFMAs or any hazard.
"""
import glob
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "gnn-plasma-flux_amd", "csrc")
FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "--offload-arch=gfx950",
         "-I" + os.path.join(ROOT, "include"), "--cuda-device-only", "-S"]
K32 = ["-mllvm", "-amdgpu-mfma-vgpr-form", "-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]  # Makefile: K32 cores


def scan(path, out_dir="/tmp"):
    """{kernel symbol: {loads, waited_at_issue, loop_vmcnt0, scratch, mfma}} of one .hip file."""
    out = os.path.join(out_dir, os.path.basename(path) + ".s")
    extra = K32 if os.path.basename(path) in ("chain_k32.hip", "chain_bf16.hip") else []
    subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *extra, path, "-o", out], check=True, cwd=CSRC,
                   stderr=subprocess.DEVNULL)
    lines = open(out).read().split("\n")
    kern, stats, in_loop = None, {}, False
    for i, ln in enumerate(lines):
        m = re.match(r"^(_Z\S+):", ln)
        if m:
            kern = m.group(1)
            stats[kern] = {"loads": 0, "waited_at_issue": 0, "loop_vmcnt0": 0, "scratch": 0, "mfma": 0}
            continue
        if kern is None:
            continue
        st = stats[kern]
        if re.match(r"^\.LBB|^; %bb", ln):
            in_loop = "Loop" in ln
        if ("global_load" in ln or "buffer_load" in ln) and " lds" not in ln:
            st["loads"] += 1
            if any("s_waitcnt" in lines[j] and "vmcnt(0)" in lines[j] for j in range(i + 1, min(i + 4, len(lines)))):
                st["waited_at_issue"] += 1
        if "s_waitcnt" in ln and "vmcnt(0)" in ln and "ASMSTART" not in lines[i - 1] and in_loop:
            st["loop_vmcnt0"] += 1
        if "scratch_" in ln:
            st["scratch"] += 1
        if "v_mfma" in ln:
            st["mfma"] += 1
    return stats


if __name__ == "__main__":
    for p in sys.argv[1:] or sorted(glob.glob(os.path.join(CSRC, "*.hip"))):
        for k, st in scan(os.path.abspath(p)).items():
            if st["mfma"] or st["waited_at_issue"] or st["loop_vmcnt0"] or st["scratch"]:
                print(os.path.basename(p), k[:100], " ".join(f"{a}={b}" for a, b in st.items()))
