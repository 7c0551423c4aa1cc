"""Summarise rocprofv3 --pmc passes (one directory per pass, as tools/gpu_pmc.sh writes them)
into per-kernel averages, with HBM bytes corrected as /opt/skills/guides/MI355X_MICROARCH.md
(§HBM) prescribes: FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the
bytes of a wide coalesced streaming read, so it is doubled (calibrated in the same workload by
the 134 MB torch copy, whose doubled FETCH_SIZE equals its byte count).

Usage: python tools/pmc_summary.py gpurun_out/pmc2 > profiles/r01/pmc_summary.json
"""
import collections
import csv
import glob
import json
import os
import sys


MIN_CLOCK_NS = 50_000  # shorter dispatches report no clock (r02 printed 7.4 GHz for a 3 us kernel)


def main(d):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    clk = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "*", "*_counter_collection.csv"))):
        acc = collections.defaultdict(float)
        meta = {}
        for r in csv.DictReader(open(f)):
            k = (r["Dispatch_Id"], r["Kernel_Name"], r["Counter_Name"])
            acc[k] += float(r["Counter_Value"])
            meta[r["Dispatch_Id"]] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
        for (disp, kname, cname), v in acc.items():
            per[kname][cname].append(v)
            if cname == "GRBM_GUI_ACTIVE":
                t0, t1 = meta[disp]
                # GHz (sum over 8 XCDs / ns), only for dispatches long enough that the counter
                # window (which extends past a short kernel's timestamps) does not dominate
                if t1 - t0 >= MIN_CLOCK_NS:
                    clk[kname].append(v / 8 / (t1 - t0))
    out = {}
    for kname, cs in per.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        e = {"counters_avg": avg}
        if "FETCH_SIZE" in avg:
            e["hbm_read_bytes"] = avg["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in avg:
            e["hbm_write_bytes"] = avg["WRITE_SIZE"] * 1024
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            e["hbm_bytes_per_launch"] = e["hbm_read_bytes"] + e["hbm_write_bytes"]
        # VALU-busy fraction (the gfx94x derived VALUBusy, which ROCm 7.2 applies to gfx950 too:
        # SQ_ACTIVE_INST_VALU x 4 / SIMDs / GRBM_GUI_ACTIVE, GRBM summed over the 8 XCDs) and the
        # SQ-busy fraction (SQ_BUSY_CYCLES over the same GPU-active cycles, 32 SQs per XCD)
        if "SQ_ACTIVE_INST_VALU" in avg and avg.get("GRBM_GUI_ACTIVE"):
            gui = avg["GRBM_GUI_ACTIVE"] / 8
            e["valu_busy_frac"] = avg["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / gui
            if "SQ_BUSY_CYCLES" in avg:
                e["sq_busy_frac"] = avg["SQ_BUSY_CYCLES"] / 256 / gui
        if clk.get(kname):
            e["effective_clock_GHz"] = sum(clk[kname]) / len(clk[kname])
        elif "GRBM_GUI_ACTIVE" in avg:
            e["effective_clock_GHz"] = None
            e["clock_note"] = "dispatch shorter than %d us: no clock derived" % (MIN_CLOCK_NS // 1000)
        out[kname] = e
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
