"""Turn the FETCH_SIZE / WRITE_SIZE rocprofv3 passes of `bench.py` into the
per-launch HBM traffic that bench.py reports as roofline.traffic.

    python tools/pmc_traffic.py TAG STEPS ICS NX TRAJ(0|1) > profiles/pmc_traffic.json

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are
in KiB; on gfx950 FETCH_SIZE reports half the bytes of wide (16 B/lane)
coalesced reads, so it is doubled; WRITE_SIZE is exact for 16-B/lane stores.
The timed launch is the LAST dispatch of the rollout kernel in each pass.
"""
import json
import sqlite3
import sys
from glob import glob

KERNEL = "CoreF32, 4>"   # the headline (f32) kernel; bench times alt precisions after it


def last_value(db, counter):
    c = sqlite3.connect(db)
    rows = c.execute("select dispatch_id, sum(counter_value), max(duration) from pmc_events where instr(name, ?) > 0 "
                     "and counter_name = ? group by dispatch_id order by dispatch_id",
                     (KERNEL, counter)).fetchall()
    return rows[-1]


def main(tag, steps, ics, nx, traj):
    f = last_value(glob(f"gpurun_out/pmc_fetch_{tag}/*.db")[0], "FETCH_SIZE")
    w = last_value(glob(f"gpurun_out/pmc_write_{tag}/*.db")[0], "WRITE_SIZE")
    fetch = 2 * f[1] * 1024
    write = w[1] * 1024
    print(json.dumps({"kernel": KERNEL, "steps": int(steps), "ics_per_gpu": int(ics), "nx": int(nx),
                      "traj": bool(int(traj)), "fetch_bytes": fetch, "write_bytes": write,
                      "traffic_bytes": fetch + write, "dispatch_us": f[2] / 1e3,
                      "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py ({tag}); "
                                "FETCH_SIZE x2 (gfx950 wide-load correction), KiB -> B"}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:6])
