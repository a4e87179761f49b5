#!/usr/bin/env python3
"""Roofline inputs from rocprofv3, and a re-derivation of bench.py's roofline fields.

  summarize --tag r02 --config C2
      reads the passes tools/profile_round.sh left under gpurun_out/prof_<tag>_<config>_* and writes
        profiles/<tag>_<config>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary of the bench
        profiles/<tag>_<config>_pmc.json           per-launch counters of the frame kernel + derived fields
        profiles/roofline_inputs.json[config]      what bench.py reads: HBM bytes and issue fractions
  check <bench.json | BENCH_rNN.json>
      recomputes every roofline field of a bench line from its own counters and profiles/, and
      fails on any disagreement.

Derivations (MI355X_MICROARCH.md):
  HBM bytes per launch = 2 x FETCH_SIZE x 1 KiB + WRITE_SIZE x 1 KiB  (gfx950 FETCH_SIZE counts
      64 B per 128-B fabric read; WRITE_SIZE is exact for wide stores); FETCH and WRITE in separate
      passes (TCC slots).
  cycles per XCD = GRBM_GUI_ACTIVE / 8 (the counter sums the 8 XCDs).
  SALU issue fraction = SQ_INSTS_SALU / (256 CUs x cycles per XCD): one scalar instruction per CU per
      cycle.
  VALU issue fraction = SQ_INSTS_VALU / (1024 SIMDs x cycles per XCD / 2): a wave64 VALU instruction
      occupies a SIMD32 for 2 cycles.
  Fetched bytes (bench.py) = 128 B x node fetches + 48 B x triangle fetches + 64 B x instance fetches
      + 108 B x primary rays + 4 B x pixels; packet-schedule fetches are counted once per wave.
"""
import argparse
import csv
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

N_CU, N_SIMD, N_XCD = 256, 1024, 8
L2_PEAK_GBS, HBM_PEAK_GBS = 34500.0, 8000.0


def is_frame_kernel(name: str) -> bool:
    """k_trace_frame*<MODE, STATS=false, ...>: the timed frame kernel, not the counter pass."""
    if "k_trace_frame" not in name or "<" not in name:
        return False
    args = [a.strip() for a in name.split("<", 1)[1].split(">", 1)[0].split(",")]
    return len(args) > 1 and args[1] == "false"


def counters(paths):
    vals = {}
    for p in paths:
        with open(p) as f:
            for row in csv.DictReader(f):
                if is_frame_kernel(row.get("Kernel_Name", "")):
                    vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    return {k: statistics.median(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def kernel_stats(path):
    with open(path) as f:
        for row in csv.DictReader(f):
            if is_frame_kernel(row["Name"]):
                return row["Name"], float(row["AverageNs"]), int(row["Calls"])
    return None, None, None


def summarize(tag, config):
    base = os.path.join(ROOT, "gpurun_out")
    out = {"config": config, "tag": tag}
    kt = sorted(glob.glob(f"{base}/prof_{tag}_{config}_kt/**/*kernel_stats.csv", recursive=True))
    if kt:
        dst = os.path.join(ROOT, "profiles", f"{tag}_{config}_kernel_stats.csv")
        shutil.copy(kt[0], dst)
        name, avg_ns, calls = kernel_stats(kt[0])
        out.update(kernel=name, kernel_avg_ns=avg_ns, kernel_calls=calls,
                   kernel_stats=os.path.relpath(dst, ROOT))
    paths = sorted(glob.glob(f"{base}/prof_{tag}_{config}_pmc*/**/*counter_collection.csv", recursive=True))
    med, n = counters(paths)
    out["counters"] = med
    out["launches"] = n
    sha = os.path.join(base, f"prof_{tag}_libsha.txt")
    if os.path.exists(sha):
        out["lib_sha"] = open(sha).read().split()[0][:16]
    if "FETCH_SIZE" in med and "WRITE_SIZE" in med:
        out["hbm_bytes_per_launch"] = 2 * med["FETCH_SIZE"] * 1024 + med["WRITE_SIZE"] * 1024
    g = med.get("GRBM_GUI_ACTIVE")
    if g and "SQ_INSTS_SALU" in med and "SQ_INSTS_VALU" in med:
        cyc = g / N_XCD
        out["issue"] = {
            "cycles_per_xcd": round(cyc, 1),
            "salu_per_launch": med["SQ_INSTS_SALU"], "valu_per_launch": med["SQ_INSTS_VALU"],
            "smem_per_launch": med.get("SQ_INSTS_SMEM"),
            "salu_frac": round(med["SQ_INSTS_SALU"] / (N_CU * cyc), 4),
            "valu_frac": round(med["SQ_INSTS_VALU"] / (N_SIMD * cyc / 2), 4),
            "wait_inst_frac": (round(med["SQ_WAIT_INST_ANY"] / med["SQ_WAVE_CYCLES"], 4)
                               if med.get("SQ_WAVE_CYCLES") and "SQ_WAIT_INST_ANY" in med else None),
            "source": f"profiles/{tag}_{config}_pmc.json",
        }
    with open(os.path.join(ROOT, "profiles", f"{tag}_{config}_pmc.json"), "w") as f:
        json.dump(out, f, indent=1)
    ipath = os.path.join(ROOT, "profiles", "roofline_inputs.json")
    inputs = {}
    if os.path.exists(ipath):
        with open(ipath) as f:
            inputs = json.load(f)
    entry = {"source": f"profiles/{tag}_{config}_pmc.json", "lib_sha": out.get("lib_sha")}
    if "hbm_bytes_per_launch" in out:
        entry["hbm_bytes_per_launch"] = out["hbm_bytes_per_launch"]
    if "issue" in out:
        entry["issue"] = {k: out["issue"][k] for k in ("salu_frac", "valu_frac", "salu_per_launch", "valu_per_launch",
                                                       "cycles_per_xcd", "wait_inst_frac")}
    if "kernel_avg_ns" in out:
        entry["rocprof_kernel_avg_ms"] = round(out["kernel_avg_ns"] / 1e6, 5)
    inputs[config] = entry
    with open(ipath, "w") as f:
        json.dump(inputs, f, indent=1)
    print(json.dumps(out, indent=1))


def load_line(path):
    with open(path) as f:
        txt = f.read()
    try:
        d = json.loads(txt)
    except ValueError:
        d = json.loads([ln for ln in txt.splitlines() if ln.startswith("{")][-1])
    if "parsed" in d:  # driver record BENCH_rNN.json
        d = d["parsed"]
    return d


def check(path):
    """Recomputes every roofline field of a bench line and enforces the pairing: `frac` is the
    `bound` pipe's fraction, `bound` the largest fraction, achieved / peak == frac for the top-level pipe and every
    pipe under `pipes`, `l2_frac` the fetched bytes over the L2 roof, `logical_bytes` SURVEY §8(d)'s per-lane model."""
    import bench
    from realtimeraytracing_gradproject_amd import scenes
    d = load_line(path)
    rf = d["roofline"]
    name = d["config"]["workload"].split(":", 1)[0]
    spec = scenes.config(name)
    pixels = spec.width * spec.height
    st = {"node_fetches": rf["node_fetches"], "tri_fetches": rf["tri_fetches"],
          "instance_fetches": rf["instance_fetches"], "primary_rays": d["config"]["primary_rays"],
          "aabb_tests": rf["aabb_tests"], "tri_tests": rf["tri_tests"]}
    b = bench.fetched_bytes(st, pixels)
    ach = b / (rf["kernel_ms"] * 1e-3) / 1e9
    problems = []
    if b != rf["bytes_per_launch"]:
        problems.append(f"bytes_per_launch {rf['bytes_per_launch']} != {b}")
    pipes = rf.get("pipes", {})
    l2 = pipes.get("l2", {})
    if abs(l2.get("achieved", -1) - ach) > 0.05 + 1e-3 * ach:  # kernel_ms is rounded to 4 decimals in the line
        problems.append(f"l2 achieved {l2.get('achieved')} != {ach:.1f}")
    if abs(rf.get("l2_frac", -1) - ach / L2_PEAK_GBS) > 1e-3:
        problems.append(f"l2_frac {rf.get('l2_frac')} != {ach / L2_PEAK_GBS:.4f}")
    fr = dict(rf.get("fracs", {}))
    if not fr or rf["bound"] != max(fr, key=fr.get):
        problems.append(f"bound {rf['bound']} is not the largest fraction {fr}")
    elif abs(rf["frac"] - fr[rf["bound"]]) > 1e-4:
        problems.append(f"frac {rf['frac']} is not the bound pipe's {fr[rf['bound']]}")
    top = pipes.get(rf["bound"], {})
    if (rf["achieved"], rf["peak"], rf["unit"]) != (top.get("achieved"), top.get("peak"), top.get("unit")):
        problems.append(f"achieved / peak / unit are not the bound pipe's ({top})")
    for k, v in pipes.items():
        if v["peak"] and abs(v["achieved"] / v["peak"] - v["frac"]) > 2e-3 * max(1.0, v["frac"]):
            problems.append(f"pipe {k}: achieved / peak {v['achieved'] / v['peak']:.4f} != frac {v['frac']}")
    if rf["frac"] > 1:
        problems.append("frac > 1")
    prof = bench.load_profile(name) or {}
    if prof.get("hbm_bytes_per_launch") != rf.get("traffic"):
        problems.append(f"traffic {rf.get('traffic')} != profiles {prof.get('hbm_bytes_per_launch')}")
    if "issue" in rf:
        for k in ("salu_frac", "valu_frac"):
            if rf["issue"][k] != prof["issue"][k]:
                problems.append(f"issue.{k} {rf['issue'][k]} != profiles {prof['issue'][k]}")
            if pipes.get(k[:4], {}).get("frac") != round(prof["issue"][k], 4):
                problems.append(f"pipes.{k[:4]}.frac != profiles issue.{k}")
    lb = bench.logical_bytes(st, pixels)
    if rf.get("logical_bytes", {}).get("bytes_per_launch") != lb:
        problems.append(f"logical_bytes {rf.get('logical_bytes')} != {lb}")
    rk = prof.get("rocprof_kernel_avg_ms")
    agree = None if not rk else round(rf["kernel_ms"] / rk, 3)
    print(json.dumps({"bench": path, "config": name, "bytes_per_launch": b, "achieved_GBs": round(ach, 1),
                      "l2_frac": round(ach / L2_PEAK_GBS, 4), "bound": rf["bound"], "frac": rf["frac"], "fracs": fr,
                      "logical_bytes": lb, "bench_kernel_ms_over_rocprof": agree, "problems": problems}, indent=1))
    return 1 if problems else 0


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("summarize")
    s.add_argument("--tag", required=True)
    s.add_argument("--config", default="C2")
    c = sub.add_parser("check")
    c.add_argument("bench")
    a = ap.parse_args()
    if a.cmd == "summarize":
        summarize(a.tag, a.config)
        return 0
    return check(a.bench)


if __name__ == "__main__":
    sys.exit(main())
