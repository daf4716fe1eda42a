"""The bench line's evidence fields, checked on CPU with stand-ins for the
device buffers: the erase-and-rebuild check fails a rebuild that writes
nothing, the PMC traffic carries its source file and library hash, and
cpu_baseline.value is the faster of its affinity and cgroup-quota legs."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


class FakeBuf:
    def __init__(self):
        self.data = bytearray(b"\x01" * 64)

    def checksum(self):
        return hash(bytes(self.data))


class FakeCtx:
    def sync(self):
        pass


def test_erase_check_detects_a_rebuild_that_writes_nothing():
    buf = FakeBuf()
    want = buf.checksum()

    def erase():
        buf.data[8:16] = b"\x00" * 8

    def good():
        buf.data[8:16] = b"\x01" * 8

    wl = bench.Workload("t", "m", {}, [], [buf], "k", 1, erase=[("good", erase, good), ("noop", erase, lambda: None)])
    out = bench.erase_checks(wl, FakeCtx(), want)
    assert out == {"good": True, "noop": False}
    # an erase that destroys nothing cannot vouch for its rebuild either
    buf.data[:] = b"\x01" * 64
    wl.erase = [("vacuous", lambda: None, good)]
    assert bench.erase_checks(wl, FakeCtx(), want) == {"vacuous": False}


def test_traffic_carries_its_source(monkeypatch):
    class A:
        chunk, layout = 1 << 20, "auto"

    t, src = bench.load_traffic(A, "rs10_4", 60129542144)
    assert t and abs(t / 60129542144 - 1) < 0.01
    assert src["file"].startswith("profiles/") and os.path.exists(os.path.join(ROOT, src["file"]))
    assert "lib_sha16" in src and src["dispatches"] >= 1
    assert src["same_library"] == (src["lib_sha16"] == bench.lib_sha16())
    # a pass measured on another build is reported as such, not hidden
    monkeypatch.setattr(bench, "lib_sha16", lambda: "0" * 16)
    t2, src2 = bench.load_traffic(A, "rs10_4", 60129542144)
    assert t2 == t and src2["same_library"] is False
    A.chunk = 12345
    assert bench.load_traffic(A, "rs10_4", 1) == (None, None)


def test_pmc_summaries_are_labelled_passes():
    """Every PMC file bench.py quotes as `traffic` is a labelled pass
    (tools/pmc_label.py) stamped with the library it measured, labels every
    dispatch with the op bench.py filters on, and the roofline workloads are
    covered.  Whether the stamp is this build's library is reported in the
    bench line (`same_library`), not asserted here: the .so is a build
    artefact, not tracked source."""
    import warnings

    h = bench.lib_sha16()
    files = {v[0]: v[1] for v in bench.PMC_SUMMARIES.values()}
    assert {w for w, _, _ in bench.PMC_SUMMARIES} >= {"rs10_4", "decode_full", "write14", "repair12", "files", "mixed16"}
    for name, op in files.items():
        with open(os.path.join(ROOT, "profiles", name)) as f:
            doc = json.load(f)
        assert len(doc["lib_sha16"]) == 16 and int(doc["lib_sha16"], 16) >= 0, name
        if doc["lib_sha16"] != h:
            warnings.warn(f"{name} was measured on libnxec {doc['lib_sha16']}, this build is {h}")
        ops = op if isinstance(op, tuple) else (op,)
        assert doc["dispatches"] and all(d["op"] == ops[0] or d["op"].startswith(ops[1:])
                                         for d in doc["dispatches"]), name


def test_lib_hash_is_sixteen_hex_digits():
    h = bench.lib_sha16()
    assert len(h) == 16 and int(h, 16) >= 0


def test_cpu_baseline_reports_the_faster_leg(monkeypatch):
    """cpu_baseline with the timing legs stubbed: the quota leg is faster here,
    so it becomes `value` (and `cores`), both legs stay in the line."""
    import numpy as np

    calls = []

    def fake_legs(threads, ns, legs, min_s):
        calls.append(threads)
        return 1, [1e-6 if threads == 3 else 4e-6] * len(legs)  # 3 threads: 4x faster

    class Args:
        cpu_threads, cpu_stripes, cpu_seconds, cpu_ref_stripes = 12, 12, 0.0, 1

    monkeypatch.setattr(bench, "_cpu_legs", fake_legs)
    monkeypatch.setattr(bench, "_host_info", lambda: {"affinity": 12, "cgroup_cpu_quota": 3.0})
    from nexoedge_amd import nxec

    import oracle
    monkeypatch.setattr(bench, "nxec", nxec)
    monkeypatch.setattr(oracle, "ref_available", lambda: False)
    monkeypatch.setattr(oracle, "fill_bytes", lambda n, seed: np.zeros(n, dtype=np.uint8))
    out = bench.cpu_baseline(Args, 14, 10, 64)
    assert out["value_leg"] == "at_cgroup_quota" and out["cores"] == 3
    assert out["value"] == out["at_cgroup_quota"]["value"] > out["at_affinity"]["value"]
    json.dumps(out)
