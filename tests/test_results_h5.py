"""The h5py branch of the result writer (results.open_results ->
results_00.h5), run with the image's real h5py 3.3.0 under
/opt/conda/bin/python3.9 (tests/_h5_writer_run.py), against the file the
REFERENCE's own create_extract_h5 + write_extracted_chunk_to_h5 write for the
same inputs (M/io/result.py:14-130; tests/golden/make_golden_results_tree.py):
the same dataset tree, and per dataset the same dtype, shape, compression
filter, 'description' attribute and values.  One value differs by design:
metadata/extraction/extract_version names the extractor that wrote the file.
The parameters carry no click help texts on either side (the CLI is out of
scope; the golden stubs click_param_annot).

Also the rank-0 writer of a sharded session (chunks arriving out of order,
TSV rows in per-rank part files, a stale part file of a failed earlier run
present): its results_00.h5 and keypoints_00.tsv equal the one-process
files."""
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

TESTS = os.path.dirname(os.path.abspath(__file__))
PY39 = "/opt/conda/bin/python3.9"
sys.path.insert(0, TESTS)
import _h5tree  # noqa: E402


def _have_h5py() -> bool:
    if not os.path.exists(PY39):
        return False
    return subprocess.run([PY39, "-c", "import h5py"], capture_output=True).returncode == 0


pytestmark = pytest.mark.skipif(not _have_h5py(), reason="no interpreter with h5py in this image")

VERSION_KEY = "metadata/extraction/extract_version"


@pytest.fixture(scope="module")
def written(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("h5w"))
    r = subprocess.run([PY39, os.path.join(TESTS, "_h5_writer_run.py"), d], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return d


def _compare(got, want):
    ga, gm = got
    wa, wm = want
    wm = {k: v for k, v in wm.items() if k != "__inputs__"}
    assert sorted(gm) == sorted(wm), (set(gm) ^ set(wm))
    for k, w in wm.items():
        g = gm[k]
        for field in ("dtype", "shape", "compression", "empty", "attrs"):
            assert g[field] == w[field], (k, field, g[field], w[field])
        if w["empty"] or k == VERSION_KEY:
            continue
        a, b = ga["d/" + k], wa["d/" + k]
        assert a.dtype == b.dtype and a.shape == b.shape, k
        assert np.array_equal(a, b, equal_nan=a.dtype.kind == "f"), k


def test_h5_tree_equals_reference_writer(written):
    want = _h5tree.load(os.path.join(TESTS, "golden", "ref_results_tree.npz"))
    got = _h5tree.load(os.path.join(written, "one.npz"))
    _compare(got, want)
    assert bytes(got[0]["d/" + VERSION_KEY]).startswith(b"moseq2-detectron-extract")
    # the reference writer's TSV bytes for the same chunks (ref_results.npz)
    g = np.load(os.path.join(TESTS, "golden", "ref_results.npz"))
    with open(os.path.join(written, "one", "keypoints_00.tsv"), "rb") as fh:
        assert fh.read() == bytes(g["tsv"])


def test_sharded_writer_h5_equals_one_process(written):
    one = _h5tree.load(os.path.join(written, "one.npz"))
    shard = _h5tree.load(os.path.join(written, "shard.npz"))
    # uuid and every other value identical (the same status dict is passed)
    _compare(shard, ({**one[0]}, {**one[1]}))
    for k in one[0]:
        assert np.array_equal(one[0][k], shard[0][k], equal_nan=one[0][k].dtype.kind == "f"), k
    with open(os.path.join(written, "one", "keypoints_00.tsv"), "rb") as a, \
            open(os.path.join(written, "shard", "keypoints_00.tsv"), "rb") as b:
        assert a.read() == b.read()
    # every part file (this run's and the stale one) is gone
    assert not [f for f in os.listdir(os.path.join(written, "shard")) if ".part" in f]


def test_runner_needs_no_reference():
    """The runner and the tree helper read only tests/ (the reference is not
    on the GPU box): no path under /root/reference is named in them."""
    for f in ("_h5_writer_run.py", "_h5tree.py"):
        with open(os.path.join(TESTS, f)) as fh:
            assert "/root/reference" not in fh.read(), f
    assert shutil.which(PY39) or os.path.exists(PY39)
