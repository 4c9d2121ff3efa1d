"""Host logic of the profile summary (scripts/rocprof_summary.py): parts of a round profiled in
separate gpurun calls merge into one traffic.json (the part holding the single graph gives the
top-level fields), and the C5 workload keeps only its 4096-graph launches' dispatches."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import rocprof_summary as rs  # noqa: E402


def test_merge_parts(tmp_path):
    a = {"kernel": "md_rollout_kernel", "avg_ns": 3.9e6, "hbm_bytes_per_launch": 5.5e8, "src_hash": "h",
         "batch": {"avg_ns": 2.5e7}, "c5": {"avg_ns": 3.8e8}}
    b = {"src_hash": "h", "real_degree": {"avg_ns": 5.2e7}, "real_unit": {"avg_ns": 3.1e7}}
    pa, pb, out = tmp_path / "a.json", tmp_path / "b.json", tmp_path / "t.json"
    pa.write_text(json.dumps(a))
    pb.write_text(json.dumps(b))
    rs.merge(str(out), [str(pb), str(pa)])
    t = json.loads(out.read_text())
    assert t["avg_ns"] == 3.9e6 and t["hbm_bytes_per_launch"] == 5.5e8 and t["src_hash"] == "h"
    assert set(t) >= {"batch", "c5", "real_degree", "real_unit"}
