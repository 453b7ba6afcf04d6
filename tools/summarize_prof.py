"""Summarise a gpu_check.sh run into committed profile files.

python tools/summarize_prof.py gpurun_out/<tag> profiles/<round>_<name> [--steps 25]

Writes
  <prefix>_kernel_stats.csv      rocprofv3 --kernel-trace --stats summary (copied as is)
  <prefix>_per_step.txt          per-kernel average duration and time per step
  <prefix>_pmc_traffic.txt       per-kernel HBM bytes per launch from separate FETCH_SIZE and
                                 WRITE_SIZE passes, gfx950-corrected as MI355X_MICROARCH.md §HBM
                                 prescribes: bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
and updates profiles/traffic.json (kernel-name key -> bytes per launch) that bench.py reads.
"""
from __future__ import annotations

import collections
import csv
import json
import os
import shutil
import sys


def kernel_stats(run: str):
    for root, _, files in os.walk(os.path.join(run, "prof")):
        for f in files:
            if f.endswith("kernel_stats.csv"):
                return os.path.join(root, f)
    raise SystemExit("no kernel_stats.csv under " + run)


def pmc(run: str, counter: str):
    path = None
    for root, _, files in os.walk(os.path.join(run, f"pmc_{counter}")):
        for f in files:
            if f.endswith("counter_collection.csv"):
                path = os.path.join(root, f)
    if path is None:
        return {}
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    run, prefix = sys.argv[1], sys.argv[2]
    steps = 25
    # --workload W: traffic.json keys "W:<kernel>" (kernels shared by workloads of other sizes)
    wl = sys.argv[sys.argv.index("--workload") + 1] if "--workload" in sys.argv else None
    if "--steps" in sys.argv:
        steps = int(sys.argv[sys.argv.index("--steps") + 1])
    ks = kernel_stats(run)
    shutil.copy(ks, prefix + "_kernel_stats.csv")
    rows = list(csv.DictReader(open(ks)))
    lines = [f"{'kernel':100s} {'calls':>6} {'avg_us':>9} {'us/step':>9}"]
    total = 0.0
    for r in rows:
        if "spin_kernel" in r["Name"]:
            continue
        per_step = float(r["TotalDurationNs"]) / 1e3 / steps
        total += per_step
        lines.append(f"{r['Name'][:100]:100s} {r['Calls']:>6} {float(r['AverageNs']) / 1e3:9.2f} "
                     f"{per_step:9.2f}")
    lines.append(f"total kernel time per step (us, {steps} profiled steps incl. warmup): "
                 f"{total:.1f}")
    open(prefix + "_per_step.txt", "w").write("\n".join(lines) + "\n")
    fetch, write = pmc(run, "FETCH_SIZE"), pmc(run, "WRITE_SIZE")
    if fetch:
        tl = [f"{'kernel':100s} {'FETCH_KB':>11} {'WRITE_KB':>11} {'hbm_MB':>9}",
              "hbm bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950: FETCH_SIZE counts half of "
              "a 16-B/lane stream)"]
        traffic_path = os.path.join(os.path.dirname(prefix) or ".", "traffic.json")
        traffic = json.load(open(traffic_path)) if os.path.exists(traffic_path) else {}
        for k in sorted(fetch, key=lambda k: -fetch[k]):
            w = write.get(k, 0.0)
            b = (2 * fetch[k] + w) * 1024
            tl.append(f"{k[:100]:100s} {fetch[k]:11.1f} {w:11.1f} {b / 1e6:9.2f}")
            traffic[f"{wl}:{k}" if wl else k] = {"bytes_per_launch": b, "source": os.path.basename(prefix) +
                          "_pmc_traffic.txt"}
        open(prefix + "_pmc_traffic.txt", "w").write("\n".join(tl) + "\n")
        json.dump(traffic, open(traffic_path, "w"), indent=1, sort_keys=True)
    print(open(prefix + "_per_step.txt").read())


if __name__ == "__main__":
    main()
