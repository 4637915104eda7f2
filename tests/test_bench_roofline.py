"""bench.py's graded roofline (VALU issue) uses PMC counters only when they were collected for
the kernel sources being timed, and for the same workload; otherwise it reports frac = null
with the reason.  CPU-only: a stand-in for the package supplies the source hash."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


class FakeRtm:
    """lib: the hash baked into the loaded library (rt_build_hash); src: the sources on disk."""
    def __init__(self, lib, src=None):
        self.lib, self.src = lib, src if src is not None else lib

    def library_build_hash(self):
        return self.lib

    def kernel_source_hash(self):
        return self.src


def _counters(tmp_path, h, workload="scenes[1, 8]_1920x1080x4"):
    os.makedirs(tmp_path / "profiles", exist_ok=True)
    c = {"source_hash": h, "workload": workload,
         "scenes": {"1": {"SQ_INSTS_VALU": 2.0e8, "hbm_bytes": 1.6e7},
                    "8": {"SQ_INSTS_VALU": 3.6e8, "hbm_bytes": 3.2e7}}}
    with open(tmp_path / "profiles" / "counters_bench.json", "w") as f:
        json.dump(c, f)


def _args():
    return argparse.Namespace(kernel=0, workload="bench")


def test_roofline_uses_matching_counters(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "SCENES", (1, 8))
    _counters(tmp_path, "abc123")
    kms = {1: 0.27, 8: 0.50}
    r = bench.valu_roofline(FakeRtm("abc123"), kms, _args(), 1, 1.9e13)
    rate = (2.0e8 + 3.6e8) / (0.77e-3)
    assert r["bound"] == "valu" and abs(r["frac"] - rate / bench.VALU_PEAK) < 1e-3
    assert r["frac"] <= 1.0 and r["traffic"] == round(1.6e7 + 3.2e7)      # per step: both launches
    assert abs(r["algorithmic_frac"] - 1.9e13 / bench.HBM_PEAK) < 1e-3
    # per scene over its own launches' duration, or over its own step alone when the legs measured it
    assert abs(r["per_scene_valu_frac"]["8"] - 3.6e8 / 0.50e-3 / bench.VALU_PEAK) < 1e-3
    r = bench.valu_roofline(FakeRtm("abc123"), kms, _args(), 1, 1.9e13, step_ms=0.51,
                            scene_ms={"1": {"ms_per_step": 0.18}, "8": {"ms_per_step": 0.33}})
    assert abs(r["frac"] - (2.0e8 + 3.6e8) / 0.51e-3 / bench.VALU_PEAK) < 1e-3
    assert abs(r["per_scene_valu_frac"]["8"] - 3.6e8 / 0.33e-3 / bench.VALU_PEAK) < 1e-3


def test_roofline_refuses_other_sources(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "SCENES", (1, 8))
    _counters(tmp_path, "old0000")
    r = bench.valu_roofline(FakeRtm("new1111"), {1: 0.27, 8: 0.5}, _args(), 1, 1.0e13)
    assert r["frac"] is None and r["achieved"] is None and "refused" in r["counters"]


def test_roofline_refuses_other_workload(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "SCENES", (1, 8))
    _counters(tmp_path, "abc123", workload="scenes[4]_4096x4096x16")
    r = bench.valu_roofline(FakeRtm("abc123"), {1: 0.27, 8: 0.5}, _args(), 1, 1.0e13)
    assert r["frac"] is None and "refused" in r["counters"]


def test_roofline_missing_counters(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    r = bench.valu_roofline(FakeRtm("abc123"), {1: 0.27, 8: 0.5}, _args(), 1, 1.0e13)
    assert r["frac"] is None and "missing" in r["counters"]


def test_roofline_refuses_stale_library(tmp_path, monkeypatch):
    """Counters collected for the sources on disk do not grade a library built from other
    sources (a stale prebuilt librt_tracer.so): the LOADED library's baked hash decides."""
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "SCENES", (1, 8))
    _counters(tmp_path, "fresh22")
    r = bench.valu_roofline(FakeRtm(lib="stale11", src="fresh22"), {1: 0.27, 8: 0.5}, _args(), 1, 1.0e13)
    assert r["frac"] is None and "refused" in r["counters"] and "stale11" in r["counters"]
