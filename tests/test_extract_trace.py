"""MDX_EXTRACT_TRACE (extract._Timeline) on the CPU: spans are recorded only
when the variable names a file, written as JSON at dump(), and summarised by
tools/extract_trace.py."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _extract():
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd import extract
    return extract


def test_timeline_off_records_nothing(monkeypatch, tmp_path):
    monkeypatch.delenv("MDX_EXTRACT_TRACE", raising=False)
    tl = _extract()._Timeline()
    t0 = tl.now()
    assert tl.add("device pass", 0, t0) >= t0
    tl.dump()
    assert tl.events == [] and not list(tmp_path.iterdir())


def test_timeline_dump_and_summary(monkeypatch, tmp_path):
    path = tmp_path / "trace.json"
    monkeypatch.setenv("MDX_EXTRACT_TRACE", str(path))
    tl = _extract()._Timeline()
    for k in range(3):
        t0 = tl.now()
        t1 = tl.add("device pass", k, t0)
        t2 = tl.add("instance selection", k, t1)
        tl.add("writer hand-off", k, t2)
    tl.dump()
    doc = json.loads(path.read_text())
    assert [e["phase"] for e in doc["events"]][:3] == ["device pass", "instance selection", "writer hand-off"]
    assert all(e["end_s"] >= e["start_s"] for e in doc["events"]) and doc["total_s"] >= 0
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "extract_trace.py"), str(path)],
                         capture_output=True, text=True, check=True).stdout
    assert "3 chunks" in out and "worker busy" in out
