"""Correlate tools/replay_timeline.py's per-transition host timestamps with the rocprofv3
kernel trace of the same run (tools/ only): python3 tools/timeline_analyze.py OUT
For each transition: the tally kernel (pz_vote_words*) that started after the flush began,
its dispatch delay after the launch call returned, its duration, and the host's notice delay
after the kernel ended (all µs, medians over the replay's transitions)."""
import csv
import glob
import json
import sys

import numpy as np


def main(out):
    tl = np.array(json.load(open(out + "/timeline.json"))["transitions"], dtype=np.int64)
    rows = []
    for path in glob.glob(out + "/tl/**/*kernel_trace.csv", recursive=True):
        rows += list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows
                if r["Kernel_Name"].startswith("pz_vote_words"))
    starts = np.array([k[0] for k in ks])
    res = []
    for t0, t1, t2, t3 in tl:
        i = int(np.searchsorted(starts, t0))
        if i >= len(ks):
            continue
        s, e, _ = ks[i]
        if s > t3:  # no tally kernel inside this transition's window
            continue
        res.append((t1 - t0, s - t1, e - s, t3 - e, t3 - t1, t2 - t1))
    r = np.array(res, dtype=np.float64) / 1e3
    names = ["flush host (launch call)", "dispatch delay (launch returned -> kernel start)", "tally kernel",
             "notice delay (kernel end -> host saw the totals)", "launch returned -> totals seen",
             "epoch pack + launches (host, overlapped)"]
    print("%d transitions matched of %d" % (len(r), len(tl)))
    for j, n in enumerate(names):
        print("  %-52s median %7.2f  p10 %7.2f  p90 %7.2f us" % (n, np.median(r[:, j]), np.percentile(r[:, j], 10),
                                                                np.percentile(r[:, j], 90)))


if __name__ == "__main__":
    main(sys.argv[1])
