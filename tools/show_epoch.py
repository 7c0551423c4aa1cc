"""Print the epoch objects of a bench line (tools/ session helper): python tools/show_epoch.py LOG"""
import json
import sys

line = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")][-1]
e = line.get("epoch", {})
for k in ("value", "roofline"):
    print(k, json.dumps(e.get(k)))
print("single_instance", json.dumps(e.get("single_instance")))
print("cold", json.dumps(e.get("cold")))
print("1m cold", json.dumps(line.get("epoch_1m_single_gpu", {}).get("cold")))
