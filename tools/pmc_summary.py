"""Condense rocprofv3 CSV output (gpurun_out/prof_*) into committed summaries under profiles/.

profiles/<tag>_kernel_stats.csv   rocprofv3 --stats kernel summary of the bench command
profiles/<tag>_pmc.json           per-launch FETCH_SIZE / WRITE_SIZE of the trace kernel
profiles/pmc_traffic.json         bytes per trace launch per config, read by bench.py ("traffic")

HBM bytes per launch = 2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024: FETCH_SIZE counts 64 B per 128-B
fabric read on gfx950 (MI355X_MICROARCH.md, HBM section), WRITE_SIZE is exact for wide stores.
"""
import argparse
import csv
import glob
import json
import os
import shutil
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))



def is_frame_kernel(name: str) -> bool:
    """The timed frame kernel: k_trace_frame*<MODE, STATS=false, ...> (the STATS=true launch is the
    untimed counter pass)."""
    if "k_trace_frame" not in name or "<" not in name:
        return False
    args = [a.strip() for a in name.split("<", 1)[1].split(">", 1)[0].split(",")]
    return len(args) > 1 and args[1] == "false"

def find(pattern):
    hits = sorted(glob.glob(os.path.join(ROOT, "gpurun_out", pattern), recursive=True))
    return hits[0] if hits else None


def counter_per_launch(path, name):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") == name and is_frame_kernel(row.get("Kernel_Name", "")):
                vals.append(float(row["Counter_Value"]))
    return statistics.median(vals) if vals else None, len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r01")
    ap.add_argument("--config", default="C2")
    a = ap.parse_args()
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    stats = find("prof_kt/**/*kernel_stats.csv")
    if stats:
        shutil.copy(stats, os.path.join(ROOT, "profiles", f"{a.tag}_{a.config}_kernel_stats.csv"))
    out = {"config": a.config}
    for key, pat in (("FETCH_SIZE", "prof_fetch/**/*counter_collection.csv"),
                     ("WRITE_SIZE", "prof_write/**/*counter_collection.csv")):
        p = find(pat)
        if p:
            v, n = counter_per_launch(p, key)
            out[key] = v
            out[key + "_launches"] = n
    if out.get("FETCH_SIZE") is not None and out.get("WRITE_SIZE") is not None:
        out["hbm_bytes_per_launch"] = 2 * out["FETCH_SIZE"] * 1024 + out["WRITE_SIZE"] * 1024
        tpath = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        t = {}
        if os.path.exists(tpath):
            with open(tpath) as f:
                t = json.load(f)
        t[a.config] = {"bytes_per_launch": out["hbm_bytes_per_launch"], "source": f"profiles/{a.tag}_{a.config}_pmc.json"}
        with open(tpath, "w") as f:
            json.dump(t, f, indent=1)
    with open(os.path.join(ROOT, "profiles", f"{a.tag}_{a.config}_pmc.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
