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


def test_winograd_fused_pack_and_policy_host(mdx):
    """mdx_winograd_pack_f4 (host): the consumer B-fragment layout of the fused
    F(4,3) kernel -- piece (channel block, K-step, point) of 64 lanes x 4, lane
    (n = l & 15, k-pair kp = l >> 4) holding U at (n, 2 kp), (n, 2 kp + 1),
    (n + 16, 2 kp), (n + 16, 2 kp + 1); a permutation of U (same multiset of
    values).  Policy: off by default, eligibility needs Cin % 8 == 0 and
    Cout % 32 == 0, shape errors are refused."""
    import ctypes
    import numpy as np
    from moseq2_detectron_extract_amd._lib import MdxError, call
    Cout, Cin = 64, 16
    U = np.random.default_rng(3).standard_normal((36, Cout, Cin)).astype(np.float32)
    Up = np.empty_like(U)
    call("mdx_winograd_pack_f4", U.ctypes.data_as(ctypes.c_void_p), Cout, Cin, Up.ctypes.data_as(ctypes.c_void_p))
    KS = Cin // 8
    pieces = Up.reshape(Cout // 32, KS, 36, 64, 4)
    for nb, ks, xi, lane in [(0, 0, 0, 0), (1, 1, 35, 63), (0, 1, 17, 21), (1, 0, 5, 40)]:
        n, kp = lane & 15, lane >> 4
        want = [U[xi, nb * 32 + n + 16 * (e >> 1), ks * 8 + 2 * kp + (e & 1)] for e in range(4)]
        np.testing.assert_array_equal(pieces[nb, ks, xi, lane], want)
    np.testing.assert_array_equal(np.sort(Up, axis=None), np.sort(U, axis=None))
    with pytest.raises(MdxError):
        call("mdx_winograd_pack_f4", U.ctypes.data_as(ctypes.c_void_p), 48, Cin, Up.ctypes.data_as(ctypes.c_void_p))
    assert call("mdx_winograd_fused_eligible", 32, 112, 128, 256, 256) == 0  # default policy: off
    old = call("mdx_conv_set_winograd_fused", 2, 0)
    try:
        assert call("mdx_winograd_fused_eligible", 32, 112, 128, 256, 256) == 1
        assert call("mdx_winograd_fused_eligible", 32, 112, 128, 260, 256) == 0  # Cin % 8
        assert call("mdx_winograd_fused_eligible", 32, 112, 128, 256, 48) == 0   # Cout % 32
        call("mdx_conv_set_winograd_fused", 1, 384)
        assert call("mdx_winograd_fused_eligible", 32, 112, 128, 256, 256) == 1  # 896 blocks x 8
        assert call("mdx_winograd_fused_eligible", 32, 7, 8, 256, 256) == 0      # 4 blocks x 8 < 384
    finally:
        call("mdx_conv_set_winograd_fused", old, 384)
