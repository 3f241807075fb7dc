"""Pin the CPU oracle against fixtures produced by the reference itself
(tests/golden/make_golden.py imports M/proc/proc.py and M/proc/roi.py)."""
import numpy as np

from oracle import frameops as O


def test_scale_lut_matches_reference(golden):
    for k in range(5):
        vmin, vmax = golden[f"scale_vmin_{k}"].item(), golden[f"scale_vmax_{k}"].item()
        lut = O.scale_lut(vmin, vmax)
        x = golden[f"scale_in_{k}"]
        np.testing.assert_array_equal(lut[x], golden[f"scale_out_{k}"])


def test_scale_fp64_quirk():
    # the float64 path maps 100 -> 254 for (0, 100); fp32 would give 255
    assert O.scale_lut(0, 100)[100] == 254


def _prep_tags(golden):
    return sorted({k[len("prep_out_"):] for k in golden if k.startswith("prep_out_")})


def test_prep_matches_reference(golden):
    tags = _prep_tags(golden)
    assert len(tags) == 6
    for tag in tags:
        vmin = float(golden[f"prep_vmin_{tag}"]); vmax = float(golden[f"prep_vmax_{tag}"])
        out, _ = O.prep_raw_frames(golden[f"prep_raw_{tag}"], golden[f"prep_bg_{tag}"], golden[f"prep_roi_{tag}"],
                                   None if np.isnan(vmin) else vmin, None if np.isnan(vmax) else vmax,
                                   fix_invalid_pixels=False)
        np.testing.assert_array_equal(out, golden[f"prep_out_{tag}"], err_msg=tag)


def test_invalid_mask_and_bbox_match_reference(golden):
    for k in range(2):
        raw = golden[f"invalid_raw_{k}"]
        tag = f"{k}_0_100"
        _, inv = O.prep_raw_frames(raw, golden[f"prep_bg_{tag}"], golden[f"prep_roi_{tag}"], 0, 100,
                                   fix_invalid_pixels=False)
        np.testing.assert_array_equal(inv, golden[f"invalid_roi_out_{k}"])
        np.testing.assert_array_equal(O.get_bbox(golden[f"prep_roi_{tag}"]), golden[f"bbox_{k}"])


def test_ellipse_strel_rows():
    # SURVEY A17 literal rows of cv2.getStructuringElement(MORPH_ELLIPSE, (9, 9))
    rows = ["000010000", "011111110", "011111110", "111111111", "111111111", "111111111",
            "011111110", "011111110", "000010000"]
    want = np.array([[int(c) for c in r] for r in rows], np.uint8)
    np.testing.assert_array_equal(O.ellipse_strel((9, 9)), want)
