"""The round-profile tooling bench.py prices its roofline from (tools/profile_final.sh): the f64
document with the lane pass (lane-weighted FLOPs), the Durand-Kerner per-pass grouping of a merged
round, and bench.py's choice of the PMC document profiled on its own tree.  CPU only: synthetic
counter files in rocprofv3's CSV shapes."""
import csv
import importlib.util
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tool(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "tools", name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _write(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)


def test_pmc_f64_lane_weighting(tmp_path, monkeypatch):
    f64 = tmp_path / "f64.csv"
    _write(f64, [
        {"kernel": "normalize_kernel", "dispatches": 2, "SQ_INSTS_VALU_FMA_F64": 0, "SQ_INSTS_VALU_MUL_F64": 0,
         "SQ_INSTS_VALU_ADD_F64": 0, "SQ_INSTS_VALU_TRANS_F64": 0, "SQ_INSTS_VALU": 10, "SQ_WAVES": 1},
        {"kernel": "ransac_dk_kernel", "dispatches": 6, "SQ_INSTS_VALU_FMA_F64": 100, "SQ_INSTS_VALU_MUL_F64": 10,
         "SQ_INSTS_VALU_ADD_F64": 20, "SQ_INSTS_VALU_TRANS_F64": 0, "SQ_INSTS_VALU": 200, "SQ_WAVES": 4},
    ])
    lanes = tmp_path / "lanes.csv"
    _write(lanes, [{"kernel": "ransac_dk_kernel", "dispatches": 6, "SQ_ACTIVE_INST_VALU": 200,
                    "SQ_THREAD_CYCLES_VALU": 200 * 64 * 0.75, "SQ_INSTS_VALU": 200, "SQ_WAVES": 4}])
    monkeypatch.setenv("DVO_PMC_LANES", str(lanes))
    monkeypatch.setenv("DVO_PMC_TREE", json.dumps({"git": "abc", "source_hash": "0123"}))
    monkeypatch.setenv("DVO_PMC_STREAMS", "1")
    out = tmp_path / "f64.json"
    _tool("pmc_f64").main(str(f64), str(out), 3072)
    doc = json.load(open(out))
    k = doc["kernels"]["ransac_dk_kernel"]
    # 6 dispatches over 2 launches (normalize_kernel): 3 per launch
    assert k["f64_wave_insts"] == pytest.approx(3 * 130)
    assert k["f64_flops_full_wave"] == pytest.approx(3 * 64 * (2 * 100 + 10 + 20))
    assert k["valu_lane_util"] == pytest.approx(0.75)
    assert k["f64_flops_lane_weighted"] == pytest.approx(0.75 * k["f64_flops_full_wave"])
    assert doc["tree"] == {"git": "abc", "source_hash": "0123"} and doc["config"]["batch"] == 3072


def test_dk_passes_groups_merged_rounds(tmp_path):
    dk = "dvo::ransac_dk_kernel(dvo::GeomArgs, int, int, int)"
    pmc, trace, lanes = [], [], []
    for i in range(6):  # two merged rounds x three passes
        for c, v in (("SQ_INSTS_VALU_FMA_F64", 10 * (i % 3 + 1)), ("SQ_WAVES", 8)):
            pmc.append({"Dispatch_Id": i, "Kernel_Name": dk, "Counter_Name": c, "Counter_Value": v})
        for c, v in (("SQ_ACTIVE_INST_VALU", 100), ("SQ_THREAD_CYCLES_VALU", 100 * 64 * (0.5 + 0.1 * (i % 3)))):
            lanes.append({"Dispatch_Id": i, "Kernel_Name": dk, "Counter_Name": c, "Counter_Value": v})
        trace.append({"Dispatch_Id": i, "Kernel_Name": dk, "Start_Timestamp": 0, "End_Timestamp": 1000 * (i % 3 + 1)})
    for name, rows in (("pmc", pmc), ("trace", trace), ("lanes", lanes)):
        _write(tmp_path / f"{name}.csv", rows)
    out = tmp_path / "dk.json"
    _tool("dk_passes").main(str(tmp_path / "pmc.csv"), str(tmp_path / "trace.csv"), str(out),
                            str(tmp_path / "lanes.csv"))
    rows = json.load(open(out))["passes"]
    assert [r["pass"] for r in rows] == [0, 1, 2]
    assert [r["dispatches"] for r in rows] == [2, 2, 2]
    assert [r["f64_wave_insts"] for r in rows] == [10, 20, 30]
    assert [round(r["valu_lane_util"], 6) for r in rows] == [0.5, 0.6, 0.7]
    for r in rows:
        assert r["issue_frac_lane_weighted"] == pytest.approx(r["issue_frac"] * r["valu_lane_util"])


def test_bench_prefers_this_trees_document(tmp_path, monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    from droplet_visual_odometry_amd.build import source_hash
    prof = tmp_path / "profiles"
    prof.mkdir()
    cfg = {"width": 1280, "height": 720, "nfeatures": 2000, "batch": 3072}
    here = {"config": cfg, "kernels": {}, "tree": {"git": "x", "source_hash": source_hash()}}
    other = {"config": cfg, "kernels": {}, "tree": {"git": "y", "source_hash": "not-this-tree"}}
    json.dump(here, open(prof / "r05a_pmc_traffic.json", "w"))
    json.dump(other, open(prof / "r05b_pmc_traffic.json", "w"))  # newer by name, another tree
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    path, doc = bench.pmc_doc(bench.PMC_TRAFFIC_GLOB, 1280, 720, 2000)
    assert os.path.basename(path) == "r05a_pmc_traffic.json"
    assert bench.pmc_tree(doc)["this_tree"] is True
    assert bench.pmc_tree(other)["this_tree"] is False
    os.remove(prof / "r05a_pmc_traffic.json")  # no document of this tree: the newest one
    path, _ = bench.pmc_doc(bench.PMC_TRAFFIC_GLOB, 1280, 720, 2000)
    assert os.path.basename(path) == "r05b_pmc_traffic.json"
