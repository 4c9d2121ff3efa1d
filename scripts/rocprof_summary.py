#!/usr/bin/env python3
"""Summarise the rocprofv3 databases written by scripts/gpu_profile_round.sh.

For each kernel-trace run: per-kernel calls / total / average / min / max duration (the
--stats view) from the rocpd SQLite output.  For the PMC passes: per-dispatch FETCH_SIZE and
WRITE_SIZE of md_rollout_kernel, with the gfx950 correction of MI355X_MICROARCH.md (FETCH_SIZE
reports half the bytes of wide coalesced reads: doubled; WRITE_SIZE taken as is), averaged
per launch -> traffic.json.

Usage: python scripts/rocprof_summary.py gpurun_out/prof_r01
"""
import glob
import json
import os
import sqlite3
import sys

KERNEL = "md_rollout_kernel"


def dbs(d):
    return sorted(glob.glob(os.path.join(d, "**", "*.db"), recursive=True))


def kernel_stats(path):
    cur = sqlite3.connect(path).cursor()
    rows = list(cur.execute("select name, duration, grid_x, workgroup_x from kernels"))
    out = {}
    for name, dur, gx, wx in rows:
        e = out.setdefault(name, {"calls": 0, "total_ns": 0, "min_ns": None, "max_ns": 0, "workgroups": set()})
        e["calls"] += 1
        e["total_ns"] += dur
        e["min_ns"] = dur if e["min_ns"] is None else min(e["min_ns"], dur)
        e["max_ns"] = max(e["max_ns"], dur)
        e["workgroups"].add(gx // max(1, wx))
    for e in out.values():
        e["avg_ns"] = e["total_ns"] / e["calls"]
        e["workgroups"] = sorted(e["workgroups"])
    return out


def pmc(path, counter, kernel):
    cur = sqlite3.connect(path).cursor()
    rows = list(cur.execute("select kernel_name, value, dispatch_id from counters_collection where counter_name = ?",
                            (counter,)))
    per = {}
    for name, val, disp in rows:
        if kernel in name:
            per[disp] = per.get(disp, 0.0) + float(val)  # KB, summed over any per-XCD instances
    return [per[k] for k in sorted(per)]


def traffic_of(d, suffix, kernel, lines):
    traffic = {}
    for sub, counter in (("pmc_fetch" + suffix, "FETCH_SIZE"), ("pmc_write" + suffix, "WRITE_SIZE")):
        for path in dbs(os.path.join(d, sub)):
            vals = pmc(path, counter, kernel)
            traffic[counter] = vals
            lines.append(f"== {counter} per {kernel} dispatch (KB, raw): {[round(v, 1) for v in vals]}")
    if not traffic.get("FETCH_SIZE") or not traffic.get("WRITE_SIZE"):
        return None
    f = traffic["FETCH_SIZE"]
    w = traffic["WRITE_SIZE"]
    fetch_b = 2.0 * 1024.0 * sum(f) / len(f)   # gfx950: FETCH_SIZE counts half of wide reads
    write_b = 1024.0 * sum(w) / max(1, len(w))
    out = {"kernel": kernel, "launches": len(f), "fetch_bytes_per_launch": fetch_b,
           "write_bytes_per_launch": write_b, "hbm_bytes_per_launch": fetch_b + write_b,
           "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); WRITE_SIZE as is; "
                         "access widths other than 16 B/lane are uncalibrated"}
    lines.append(f"== traffic per {kernel} launch: " + json.dumps(out))
    return out


def main():
    d = sys.argv[1]
    report = {}
    lines = []
    for sub in ("single", "batch"):
        for path in dbs(os.path.join(d, sub)):
            st = kernel_stats(path)
            report[sub] = {k: {kk: vv for kk, vv in v.items()} for k, v in st.items()}
            lines.append(f"== {sub}: {path}")
            lines.append(f"{'kernel':60s} {'calls':>6s} {'total_ms':>10s} {'avg_us':>10s} {'min_us':>10s} {'max_us':>10s} workgroups")
            for k, v in sorted(st.items(), key=lambda kv: -kv[1]["total_ns"]):
                lines.append(f"{k[:60]:60s} {v['calls']:6d} {v['total_ns'] / 1e6:10.3f} {v['avg_ns'] / 1e3:10.1f} "
                             f"{v['min_ns'] / 1e3:10.1f} {v['max_ns'] / 1e3:10.1f} {v['workgroups']}")
    single = traffic_of(d, "", KERNEL, lines)
    batch = traffic_of(d, "_batch", "md_queue_kernel", lines)
    if single is not None:
        out = dict(single)
        if batch is not None:
            out["batch"] = batch
        with open(os.path.join(d, "traffic.json"), "w") as fo:
            json.dump(out, fo, indent=1)
    with open(os.path.join(d, "summary.txt"), "w") as fo:
        fo.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
