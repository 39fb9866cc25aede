"""Turn the FETCH_SIZE / WRITE_SIZE rocprofv3 passes of `bench.py` into the
per-launch HBM traffic that bench.py reports as roofline.traffic.

    python tools/pmc_traffic.py TAG_A STEPS_A TAG_B STEPS_B ICS NX TRAJ(0|1) > profiles/pmc_traffic.json

Two passes at different step counts (tools/gpu_pmc_traffic.sh runs both: TAG_A STEPS_A, then TAG_B
STEPS_B) separate a fixed part (state, weight stream, launch) from a per-step
part (trajectory and metric writes), so bench.py can state the traffic of a
launch of any --steps: traffic(K) = fixed_bytes + per_step_bytes * K.

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are
in KiB; on gfx950 FETCH_SIZE reports half the bytes of wide (16 B/lane)
coalesced reads, so it is doubled; WRITE_SIZE is exact for 16-B/lane stores.
The timed launch is the LAST dispatch of the rollout kernel in each pass.

The record is bound to the library it was measured on: "build" is the src:
hash that bench.py printed in both passes (their logs
gpurun_out/pmc_{fetch,write}_<tag>.log), and bench.py reports the traffic
only while the loaded library carries that same hash.
"""
import json
import sqlite3
import sys
from glob import glob

KERNEL = "CoreF32T<2, 4, false, true>, 4>"   # the headline (f32) kernel; bench times alt precisions after it


def last_value(db, counter):
    c = sqlite3.connect(db)
    rows = c.execute("select dispatch_id, sum(counter_value), max(duration) from pmc_events where instr(name, ?) > 0 "
                     "and counter_name = ? group by dispatch_id order by dispatch_id",
                     (KERNEL, counter)).fetchall()
    return rows[-1]


def bench_build(tag):
    """The src: hash of the library bench.py ran in each pass of `tag` (the JSON
    line of its log); every pass must name the same one."""
    builds = set()
    for kind in ("fetch", "write"):
        with open(f"gpurun_out/pmc_{kind}_{tag}.log") as f:
            for ln in f:
                if ln.startswith("{"):
                    builds.add(json.loads(ln)["build"].split("src:")[-1].split(" flags:")[0])
    assert len(builds) == 1, builds
    return builds.pop()


def traffic(tag):
    # databases under /tmp on the box (tools/gpu_pmc_traffic.sh), or gpurun_out/ (older passes)
    db = lambda kind: (glob(f"/tmp/pmc_{kind}_{tag}/*.db") + glob(f"gpurun_out/pmc_{kind}_{tag}/*.db"))[0]  # noqa: E731
    f = last_value(db("fetch"), "FETCH_SIZE")
    w = last_value(db("write"), "WRITE_SIZE")
    return 2 * f[1] * 1024, w[1] * 1024, f[2] / 1e3


def main(tag_a, steps_a, tag_b, steps_b, ics, nx, traj):
    ka, kb = int(steps_a), int(steps_b)
    fa, wa, da = traffic(tag_a)
    fb, wb, db = traffic(tag_b)
    build = bench_build(tag_a)
    assert bench_build(tag_b) == build
    per_step = ((fb + wb) - (fa + wa)) / (kb - ka)
    fixed = (fa + wa) - per_step * ka
    print(json.dumps({"kernel": KERNEL, "build": build, "ics_per_gpu": int(ics), "nx": int(nx), "traj": bool(int(traj)),
                      "fixed_bytes": fixed, "per_step_bytes": per_step,
                      "passes": {str(ka): {"fetch_bytes": fa, "write_bytes": wa, "dispatch_us": da},
                                 str(kb): {"fetch_bytes": fb, "write_bytes": wb, "dispatch_us": db}},
                      "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py at {ka} and {kb} steps "
                                f"({tag_a}, {tag_b}); FETCH_SIZE x2 (gfx950 wide-load correction), KiB -> B; "
                                "linear in steps", "algorithmic_bytes_model": "12 B x B x nx x (K+1) trajectory + 24 B x B x nx "
                                "state in/out + 16 B x B x (K+1) metrics"}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:8])
