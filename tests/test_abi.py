"""CPU-side checks of the C ABI: the library builds/loads and exports every
entry point include/mdx.h declares (no device work without a GPU)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    names = []
    for fn in sorted(os.listdir(os.path.join(ROOT, "include"))):
        if fn.endswith(".h"):
            src = open(os.path.join(ROOT, "include", fn)).read()
            src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
            names += re.findall(r"\b(mdx_[a-z0-9_]+)\s*\(", src)
    return sorted(set(names))


def test_header_declares_entry_points():
    names = _declared()
    assert "mdx_prep_frames" in names and "mdx_crop_rotate" in names


def test_library_exports_every_declared_symbol(mdx):
    import ctypes
    from moseq2_detectron_extract_amd import _build, _lib
    if not os.path.exists(_lib.LIB_PATH):
        _build.build()
    L = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in _declared() if not hasattr(L, n)]
    assert not missing, missing
    # every declared symbol has a Python signature (so ctypes calls are typed)
    assert not [n for n in _declared() if n not in _lib.SIGNATURES]


def test_host_only_entry_points(mdx):
    import numpy as np
    from moseq2_detectron_extract_amd import proc
    from oracle import frameops as O
    for vmin, vmax in [(0, 100), (10, 80), (0.5, 99.5)]:
        np.testing.assert_array_equal(proc.scale_lut(vmin, vmax), O.scale_lut(vmin, vmax))
    assert mdx.lib().mdx_version().decode().startswith("mdx")


def test_inpaint_workspace_is_sparse(mdx):
    """The inpaint workspace of a 423 x 511 extract frame (512 x 424 ROI crop)
    stays under 1 MB per frame at batch 32 and 1024 (sparse per-frame slots
    plus one shared full-size slot), with room for about 4 % of the frame's
    pixels per frame in the sparse slot."""
    from moseq2_detectron_extract_amd._lib import call
    H, W = 423, 511
    for n in (32, 1024):
        per_frame = call("mdx_inpaint_workspace_bytes", n, H, W) / n
        assert per_frame < (1 << 20) * (1.5 if n == 32 else 1.0), (n, per_frame)
    slope = (call("mdx_inpaint_workspace_bytes", 1024, H, W) - call("mdx_inpaint_workspace_bytes", 32, H, W)) / 992
    assert slope < 1e6
    cap = call("mdx_inpaint_sparse_capacity", H, W)
    assert 0.04 * H * W <= cap <= 0.05 * H * W
    assert call("mdx_inpaint_workspace_bytes", 0, H, W) == 0


def test_no_gpu_means_loud_failure(mdx):
    import numpy as np
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from moseq2_detectron_extract_amd import MdxError, proc
    with pytest.raises(MdxError):
        proc.clean_frames(np.zeros((1, 8, 8), np.uint8), iters_tail=1)


@pytest.mark.parametrize("m", [2, 4, 6])
def test_winograd_weight_transform_host(mdx, m):
    """mdx_winograd_weights (a host function): U = G g G^T for F(m x m, 3x3),
    checked by running one m x m output tile through the transform algebra in
    fp64 (Y = A^T [U . (B^T d B)] A, B^T / A^T the kernels' matrices, Lavin's
    points; F(6,3): 0, +-1, +-2, +-1/2) against the direct 3x3 correlation;
    and the policy-6 tile choice per map size."""
    import ctypes
    import numpy as np
    from moseq2_detectron_extract_amd._lib import call
    BT = {2: [[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]],
          4: [[4, 0, -5, 0, 1, 0], [0, -4, -4, 1, 1, 0], [0, 4, -4, -1, 1, 0], [0, -2, -1, 2, 1, 0],
              [0, 2, -1, -2, 1, 0], [0, 4, 0, -5, 0, 1]],
          6: [[1, 0, -5.25, 0, 5.25, 0, -1, 0], [0, 1, 1, -4.25, -4.25, 1, 1, 0], [0, -1, 1, 4.25, -4.25, -1, 1, 0],
              [0, .5, .25, -2.5, -1.25, 2, 1, 0], [0, -.5, .25, 2.5, -1.25, -2, 1, 0], [0, 2, 4, -2.5, -5, .5, 1, 0],
              [0, -2, 4, 2.5, -5, -.5, 1, 0], [0, -1, 0, 5.25, 0, -5.25, 0, 1]]}[m]
    AT = {2: [[1, 1, 1, 0], [0, 1, -1, -1]],
          4: [[1, 1, 1, 1, 1, 0], [0, 1, -1, 2, -2, 0], [0, 1, 1, 4, 4, 0], [0, 1, -1, 8, -8, 1]],
          6: [[1, 1, 1, 1, 1, 1, 1, 0], [0, 1, -1, 2, -2, .5, -.5, 0], [0, 1, 1, 4, 4, .25, .25, 0],
              [0, 1, -1, 8, -8, .125, -.125, 0], [0, 1, 1, 16, 16, .0625, .0625, 0],
              [0, 1, -1, 32, -32, .03125, -.03125, 1]]}[m]
    BT, AT = np.array(BT, float), np.array(AT, float)
    a, Cout, Cin = m + 2, 3, 5
    rng = np.random.default_rng(m)
    w = rng.standard_normal((Cout, Cin, 3, 3)).astype(np.float32)
    U = np.empty((a * a, Cout, Cin), np.float32)
    call("mdx_winograd_weights", w.ctypes.data_as(ctypes.c_void_p), Cout, Cin, m, U.ctypes.data_as(ctypes.c_void_p))
    U = U.reshape(a, a, Cout, Cin).astype(np.float64)
    d = rng.standard_normal((Cin, a, a))
    V = np.einsum("ij,cjk,lk->ilc", BT, d, BT)
    Y = np.einsum("ij,jko,lk->oil", AT, np.einsum("jkoc,jkc->jko", U, V), AT)
    want = np.array([[[np.sum(w[o].astype(np.float64) * d[:, y:y + 3, x:x + 3]) for x in range(m)]
                      for y in range(m)] for o in range(Cout)])
    np.testing.assert_allclose(Y, want, rtol=0, atol=1e-5 * np.abs(want).max())
    assert call("mdx_winograd_tile", 112, 128, 6) == 6 and call("mdx_winograd_tile", 56, 64, 6) == 6
    assert call("mdx_winograd_tile", 28, 32, 6) == 4 and call("mdx_winograd_tile", 7, 7, 6) == 4
    assert call("mdx_winograd_tile", 112, 128, 4) == 4 and call("mdx_winograd_tile", 5, 5, 2) == 2


def test_policy_struct_matches_header():
    """_lib.POLICY_FIELDS is include/mdx.h's mdx_policy, field for field."""
    import re
    from moseq2_detectron_extract_amd._lib import POLICY_FIELDS
    hdr = open(os.path.join(ROOT, "include", "mdx.h")).read()
    body = hdr[hdr.index("typedef struct mdx_policy {"):hdr.index("} mdx_policy;")]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    fields = [f.strip() for decl in re.findall(r"\bint\s+([^;]+);", body) for f in decl.split(",")]
    assert tuple(fields) == POLICY_FIELDS


def test_policy_per_thread_and_validated(mdx):
    """mdx_policy_set / get: the calling thread's policy (another thread keeps
    the library defaults), validated fields, restored by policy_scope."""
    import threading
    from moseq2_detectron_extract_amd._lib import MdxError, knob, policy, policy_defaults, policy_scope, set_policy
    d = policy_defaults()
    assert d["winograd"] == 6 and d["fp32_split"] == 0 and d["single_stage"] == 4 and d["roi_mode"] == 4
    assert policy() == d
    seen = {}
    with policy_scope(winograd=4, roi_mode=7):
        assert policy()["winograd"] == 4 and policy()["roi_mode"] == 7
        t = threading.Thread(target=lambda: seen.update(policy()))
        t.start()
        t.join()
        assert knob("winograd", 2) == 4 and policy()["winograd"] == 2
    assert seen == d          # the other thread: its own (default) policy
    assert policy() == d      # restored
    for bad in ({"winograd": 3}, {"fp32_split": 5}, {"roi_mode": 9}, {"narrow_kmax": -1}):
        with pytest.raises(MdxError):
            set_policy(**bad)
    assert policy() == d
    with pytest.raises(KeyError):
        set_policy(no_such_field=1)
