"""Eye-tracking front end, CPU side.

* The CPU oracle of the network (oracle/ritnet_oracle.py) with the
  reference's own checkpoint, fed through this build's preprocessing
  (gamma table, OpenCV-CLAHE restatement, normalisation, transpose), must
  reproduce the segmentation the reference saved (eye_seg_pred.png, decoded
  into tests/golden/eye_pins.npz by tools/make_eye_golden.py) -- this pins
  both the preprocessing and the network restatement to the reference's own
  output.  It needs /root/reference (the checkpoint is not copied into this
  repository) and is skipped elsewhere.
* Preprocessing pins and properties that need no reference.
* The fovea mapping of SURVEY §8(d) config 3.
"""
import os

import numpy as np
import pytest

import ritnet_oracle as R

REF = "/root/reference"
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "eye_pins.npz")


def _E():
    from gaussian_splatting_with_eye_tracking_amd import eye_tracking as E
    return E


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "RITnet", "best_model.pkl")),
                    reason="needs the reference's RITnet checkpoint (this container only)")
@pytest.mark.timeout(600)
def test_oracle_with_reference_checkpoint_reproduces_saved_prediction():
    import torch
    E = _E()
    g = np.load(GOLD)
    sd = torch.load(os.path.join(REF, "RITnet", "best_model.pkl"), map_location="cpu", weights_only=True)
    lab = R.labels(R.forward(sd, E.preprocess(g["eye"])))
    assert lab.shape == g["labels"].shape == (640, 400)
    agree = float((lab == g["labels"]).mean())
    assert agree >= 0.9999, agree          # observed: 1.0 (identical label histograms)
    np.testing.assert_array_equal(np.bincount(lab.ravel(), minlength=4), np.bincount(g["labels"].ravel(), minlength=4))
    # the ground truth is a different thing (annotation); record the model's agreement with it
    assert float((lab.T == g["label_gt"]).mean()) > 0.85


def test_clahe_regression_and_properties():
    E = _E()
    g = np.load(GOLD)
    np.testing.assert_array_equal(E.clahe(E.apply_gamma(g["eye"])), g["clahe"])
    flat = np.full((80, 64), 97, np.uint8)           # one grey level everywhere
    out = E.clahe(flat)
    assert out.dtype == np.uint8 and out.shape == flat.shape
    assert len(np.unique(out)) == 1                  # a constant image stays constant
    dark = np.zeros((64, 64), np.uint8)
    dark[::2, ::2] = 255                             # two levels: the LUT keeps their order
    d = E.clahe(dark)
    assert (d[::2, ::2] > d[1::2, 1::2]).all()


def test_preprocess_layout_and_range():
    E = _E()
    g = np.load(GOLD)
    x = E.preprocess(g["eye"])
    assert x.shape == (640, 400) and x.dtype == np.float32 and x.flags.c_contiguous
    assert float(x.min()) >= -1.0 and float(x.max()) <= 1.0
    np.testing.assert_array_equal(x, ((g["clahe"].astype(np.float32) / np.float32(255)) - np.float32(0.5))
                                  .__truediv__(np.float32(0.5)).T)


def test_gamma_table_truncates():
    E = _E()
    t = E.gamma_table()
    v = np.arange(256, dtype=np.uint8)
    np.testing.assert_array_equal(E.apply_gamma(v), np.floor(t).astype(np.uint8))


def test_fovea_mapping_config3():
    E = _E()
    fx, fy = E.fovea_center((361.74, 248.19), (640, 400), (1920, 1080))
    assert abs(fx - 1085.22) < 0.01 and abs(fy - 670.113) < 0.01


def test_saved_prediction_pupil_centroid():
    """The pupil (label 3) of the reference's saved prediction, in the eye
    image's orientation (x along its 640 columns), next to the ground truth's
    (361.74, 248.19) quoted by SURVEY §8(d)."""
    g = np.load(GOLD)
    ys, xs = np.nonzero(g["labels"].T == 3)
    cx, cy = xs.mean(), ys.mean()
    gy, gx = np.nonzero(g["label_gt"] == 3)
    assert abs(gx.mean() - 361.74) < 0.01 and abs(gy.mean() - 248.19) < 0.01
    # the model's pupil vs the annotation: observed (358.24, 229.81) vs (361.74, 248.19)
    assert abs(cx - 358.235) < 0.01 and abs(cy - 229.810) < 0.01
    assert np.hypot(cx - gx.mean(), cy - gy.mean()) < 25.0
