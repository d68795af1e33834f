"""One line per tools/ab_run.sh run (development tool)."""
import collections
import csv
import glob
import json
import re
import sys

mode, path = sys.argv[1], sys.argv[2]
tag = path.rstrip("/").split("/")[-1]


def short(name):
    base = re.sub(r"^(void )?qf::", "", name.split("(")[0])
    m = re.match(r"(\w+)<(.*)>$", base)
    if m and "bsort_fast" in m.group(1):  # keep the configuration
        return "bsort_fast<" + m.group(2).replace(" ", "") + ">"
    return base.split("<")[0][-24:]


if mode == "kbench":
    f = glob.glob(f"{path}/**/run_kernel_stats.csv", recursive=True)[0]
    t = {short(r["Name"]): round(float(r["AverageNs"]) / 1e3, 1) for r in csv.DictReader(open(f))
         if "qf::" in r["Name"] and "synth" not in r["Name"] and "copy" not in r["Name"]}
    print(tag, t, flush=True)
elif mode == "kstats":
    f = glob.glob(f"{path}/**/run_kernel_stats.csv", recursive=True)[0]
    log = open(sys.argv[3]).read()
    dg = re.findall(r"ok ([0-9a-f]{16})", log)
    t = {}
    for r in csv.DictReader(open(f)):
        if any(k in r["Name"] for k in ("sort", "join", "fuse_large")):
            t[short(r["Name"])] = round(float(r["AverageNs"]) / 1e3, 1)
    print(tag, dg, t, flush=True)
elif mode == "pmc":
    f = glob.glob(f"{path}/**/run_counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        if any(k in r["Kernel_Name"] for k in ("sort", "join")):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        print(tag, k, {c[3:]: "%.3e" % (sum(v) / len(v)) for c, v in sorted(cs.items())},
              flush=True)
elif mode == "bench":
    d = json.load(open(path))
    r = d["roofline"]
    print(tag, d["ms_per_step"], "fuse", r["kernel_ms"], "frac", r["frac"],
          "parity", d["parity_vs_oracle"]["bit_exact"], "U", d["config"]["mean_union"], flush=True)
