"""One line per leg of a bench.py output (the last JSON line of the file given)."""
import json
import sys


def main(path):
    d = json.loads(open(path).read().strip().splitlines()[-1])
    r = d["roofline"]
    print("hash %.3f G/s frac %.3f kernel_ms %.4f" % (d["value"] / 1e9, r["frac"], r["kernel_ms"]))
    for k in ("epoch", "epoch_1m_single_gpu", "wire", "attcheck", "wire_att"):
        if k in d:
            v, r = d[k], d[k]["roofline"]
            print("%-20s %.4g %s ms/step %.4f frac %.3f device_ms %.4f" % (
                k, v["value"], v["unit"], v["ms_per_step"], r["frac"], r["step_device_ms"]))
    if "replay" in d:
        print("replay %.0f blocks/s parity: %s" % (d["replay"]["value"], str(d["replay"].get("parity"))[-12:]))


if __name__ == "__main__":
    main(sys.argv[1])
