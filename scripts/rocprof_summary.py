#!/usr/bin/env python3
"""Summarise the rocprofv3 databases written by scripts/gpu_profile_round.sh.

* kernel-trace runs (single/, batch/): per-kernel calls / total / average / min / max duration
  (the --stats view) from the rocpd SQLite output;
* PMC passes (pmc_<group>_<workload>/): per-dispatch counter values of the workload's main
  kernel (md_rollout_kernel for the single graph, the degree-cost graph and the N = 18 000
  testReal-sized cases; md_wq_kernel for the batch and C5, with their tail launches:
  md_queue_kernel for the last MD_WQPARK graphs, md_rollout_kernel for the last MD_QPARK),
  averaged per launch.

Derived per launch (written to traffic.json, which bench.py reads when its `src_hash` equals the
hash of the kernel sources being benchmarked):
* HBM traffic: FETCH_SIZE x 2 (gfx950: FETCH_SIZE counts half the bytes of wide coalesced
  reads, MI355X_MICROARCH.md HBM section) + WRITE_SIZE;
* MFMA busy: SQ_VALU_MFMA_BUSY_CYCLES / (kernel cycles x 256 CUs x 4 SIMDs), kernel cycles =
  GRBM_GUI_ACTIVE / 8 (rocprofv3 sums it over the 8 XCDs); and the executed MFMA rate
  SQ_INSTS_VALU_MFMA_MOPS_F32 x 512 FLOP / kernel-trace duration against the 157.3 TFLOP/s
  fp32 matrix peak (executed, not algorithmic, flops);
* wave-state split: SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES;
* LDS bank conflicts: SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE.

Usage: python scripts/rocprof_summary.py gpurun_out/prof_r02
       python scripts/rocprof_summary.py --merge traffic.json traffic_a.json traffic_b.json
"""
import glob
import json
import os
import sqlite3
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
KERNELS = {"single": "md_rollout_kernel", "batch": "md_wq_kernel", "c5": "md_wq_kernel",
           "degree": "md_rollout_kernel", "real_degree": "md_rollout_kernel", "real_unit": "md_rollout_kernel"}
TAILS = ("md_queue_kernel", "md_rollout_kernel")  # a batch launch's tail hand-offs, in order
CUS, SIMDS, XCDS, PEAK_TF = 256, 4, 8, 157.3


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


def pmc(path, kernel):
    """{counter: [per-dispatch value (summed over instances)]} for dispatches of `kernel`."""
    cur = sqlite3.connect(path).cursor()
    rows = list(cur.execute("select kernel_name, counter_name, value, dispatch_id from counters_collection"))
    per = {}
    for name, cname, val, disp in rows:
        if kernel in name:
            d = per.setdefault(cname, {})
            d[disp] = d.get(disp, 0.0) + float(val)
    return {c: [v[k] for k in sorted(v)] for c, v in per.items()}


def mean(x):
    return sum(x) / len(x) if x else None


def workload(d, w, lines):
    kernel = KERNELS[w]
    out = {"kernel": kernel}
    for path in dbs(os.path.join(d, w)):
        st = kernel_stats(path)
        lines.append(f"== {w}: kernel trace {os.path.relpath(path, d)}")
        lines.append(f"{'kernel':60s} {'calls':>6s} {'total_ms':>10s} {'avg_us':>10s} {'min_us':>10s} {'max_us':>10s} workgroups")
        for k, v in sorted(st.items(), key=lambda kv: -kv[1]["total_ns"]):
            lines.append(f"{k[:60]:60s} {v['calls']:6d} {v['total_ns'] / 1e6:10.3f} {v['avg_ns'] / 1e3:10.1f} "
                         f"{v['min_ns'] / 1e3:10.1f} {v['max_ns'] / 1e3:10.1f} {v['workgroups']}")
            if kernel in k:
                out["avg_ns"] = v["avg_ns"]
    vals = {}
    for group in ("fetch", "write", "sq1", "sq2", "sq3"):
        for path in dbs(os.path.join(d, f"pmc_{group}_{w}")):
            for c, v in pmc(path, kernel).items():
                vals[c] = v
                lines.append(f"== {w} {c} per {kernel} dispatch (raw): {[round(x, 1) for x in v]}")
    # (C5 is profiled with --c5-shard-graphs 0, gpu_profile_round.sh: every md_wq_kernel
    # dispatch of that run is a 4096-graph launch, so all of them are kept -- no filtering by
    # duration or traffic, which would also drop short relaunches of the same run)
    m = {c: mean(v) for c, v in vals.items()}
    if w in ("batch", "c5"):
        # the tail launches of each batch rollout (md_queue_kernel: the graphs the wave-item
        # kernel parks; md_rollout_kernel: the last ones the queue hands to the lock-step
        # kernel): their traffic per dispatch, averaged over both, so bench.py can report the
        # traffic of a whole batch step (main + tails)
        tb, nd = 0.0, 0
        for tk in TAILS:
            tv = {}
            for group in ("fetch", "write"):
                for path in dbs(os.path.join(d, f"pmc_{group}_{w}")):
                    for c, v in pmc(path, tk).items():
                        tv[c] = v
                        lines.append(f"== {w} {c} per {tk} (tail) dispatch (raw): {[round(x, 1) for x in v]}")
            if tv.get("FETCH_SIZE") and tv.get("WRITE_SIZE") and len(tv["FETCH_SIZE"]) == len(tv["WRITE_SIZE"]):
                tb += sum(2.0 * 1024.0 * f + 1024.0 * x for f, x in zip(tv["FETCH_SIZE"], tv["WRITE_SIZE"]))
                nd += len(tv["FETCH_SIZE"])
        if nd:
            out["tail_hbm_bytes_per_launch"] = tb / nd
            out["tail_dispatches"] = nd
    if m.get("FETCH_SIZE") is not None and m.get("WRITE_SIZE") is not None:
        out["fetch_bytes_per_launch"] = 2.0 * 1024.0 * m["FETCH_SIZE"]
        out["write_bytes_per_launch"] = 1024.0 * m["WRITE_SIZE"]
        out["hbm_bytes_per_launch"] = out["fetch_bytes_per_launch"] + out["write_bytes_per_launch"]
        out["correction"] = ("FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); WRITE_SIZE as is; access "
                             "widths other than 16 B/lane are uncalibrated")
    if m.get("SQ_VALU_MFMA_BUSY_CYCLES") is not None and m.get("GRBM_GUI_ACTIVE"):
        cyc = m["GRBM_GUI_ACTIVE"] / XCDS
        busy = {"mfma_busy_frac": m["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * CUS * SIMDS),
                "kernel_cycles": cyc,
                "mfma_busy_cycles": m["SQ_VALU_MFMA_BUSY_CYCLES"],
                "mfma_f32_insts": m.get("SQ_INSTS_VALU_MFMA_F32"),
                "mfma_f32_flops_executed": (m.get("SQ_INSTS_VALU_MFMA_MOPS_F32") or 0.0) * 512.0}
        if out.get("avg_ns"):
            busy["clock_ghz"] = cyc / out["avg_ns"]
            tf = busy["mfma_f32_flops_executed"] / (out["avg_ns"] * 1e-9) / 1e12
            busy["mfma_executed_tflops"] = tf
            busy["mfma_executed_frac_of_peak"] = tf / PEAK_TF
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if m.get(c) is not None:
                    busy[c.lower() + "_frac"] = m[c] / wc
        if m.get("SQ_LDS_IDX_ACTIVE"):
            busy["lds_bank_conflict_frac"] = (m.get("SQ_LDS_BANK_CONFLICT") or 0.0) / m["SQ_LDS_IDX_ACTIVE"]
        for c in ("SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_VALU", "SQ_INSTS_SALU",
                  "SQ_VALU_MFMA_COEXEC_CYCLES", "SQ_BUSY_CYCLES", "SQ_INSTS_FLAT", "SQ_INSTS_SMEM",
                  "SQ_INSTS_BRANCH", "SQ_WAVES"):
            if m.get(c) is not None:
                busy[c.lower()] = m[c]
        out["mfma_busy"] = busy
    lines.append(f"== {w} per-launch summary: " + json.dumps(out))
    return out


def merge(dst, parts):
    """traffic.json of a round profiled in parts (gpu_profile_round.sh PART=...): the first part
    holding the single graph gives the top-level fields, every part its nested workloads."""
    out = {}
    for p in parts:
        with open(p) as f:
            t = json.load(f)
        nested = {k: v for k, v in t.items() if k in KERNELS}
        top = {k: v for k, v in t.items() if k not in KERNELS}
        if "avg_ns" in top or not out:
            out.update(top)
        out.update(nested)
    with open(dst, "w") as fo:
        json.dump(out, fo, indent=1)


def main():
    import bench
    if sys.argv[1] == "--merge":  # rocprof_summary.py --merge out.json part_a.json part_b.json ...
        merge(sys.argv[2], sys.argv[3:])
        return
    d = sys.argv[1]
    lines = [f"kernel sources hash {bench.kernel_src_hash()}"]
    report = {w: workload(d, w, lines) for w in KERNELS if os.path.isdir(os.path.join(d, w))}
    out = dict(report.get("single", {}))
    for w in KERNELS:
        if w != "single" and w in report:
            out[w] = report[w]
    out["src_hash"] = bench.kernel_src_hash()
    out["source"] = f"rocprofv3 PMC passes, {os.path.basename(os.path.normpath(d))} (scripts/gpu_profile_round.sh)"
    with open(os.path.join(d, "traffic.json"), "w") as fo:
        json.dump(out, fo, indent=1)
    with open(os.path.join(d, "summary.txt"), "w") as fo:
        fo.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
