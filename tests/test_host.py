"""Host-side helpers against the oracle (CPU only, no GPU calls)."""
import numpy as np
import pytest

from oracle import ref_post
from ycx.detect import yolo_correct_boxes


@pytest.mark.parametrize('letterbox', [True, False])
@pytest.mark.parametrize('image_hw', [(512, 773), (640, 640), (1080, 1920), (333, 17)])
def test_yolo_correct_boxes_matches_oracle(letterbox, image_hw):
    """The host yolo_correct_boxes (detect.py:147-165) reproduces the reference's
    numpy arithmetic bit for bit, including the in-place float32 scaling of the
    caller's box_wh."""
    rng = np.random.default_rng(sum(image_hw) + letterbox)
    xy = rng.random((257, 2), dtype=np.float32)
    wh = rng.random((257, 2), dtype=np.float32) * np.float32(0.5)
    wh_a, wh_b = wh.copy(), wh.copy()
    got = yolo_correct_boxes(xy.copy(), wh_a, (640, 640), np.array(image_hw), letterbox)
    want = ref_post.yolo_correct_boxes(xy.copy(), wh_b, (640, 640), np.array(image_hw), letterbox)
    assert got.dtype == want.dtype and got.shape == want.shape == (257, 4)
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(wh_a, wh_b)  # the same in-place side effect on the caller's array


def test_target_box_record():
    """utils/target_box.py:8-38 API: corner fields, accessors, printable record;
    the palette of utils/helper_cv.py:60-64."""
    from ycx.utils.target_box import TargetBox, colors_for
    tb = TargetBox([3, 4, 50, 60], 0.75, 'dog', (255, 0, 0))
    assert (tb.left, tb.top, tb.right, tb.bottom) == (3, 4, 50, 60)
    assert tb.get_topleft() == (3, 4) and tb.get_bottomright() == (50, 60)
    text = str(tb)
    assert text.startswith('-' * 20 + 'TargetBox') and 'dog' in text and '0.75' in text
    assert colors_for(3) == [(255, 0, 0), (0, 255, 0), (0, 0, 255)]
    assert colors_for(1) == [(255, 0, 0)]



def test_decoded_flip_report_attribution():
    """helpers.decoded_flip_report (the fp16 C1 predict attribution): identical decoded
    tensors give no flips; a score swap between two overlapping boxes flips both keep
    decisions and is attributed to the swap; a score moved across conf_thres is a
    membership flip next to the threshold."""
    import torch
    from helpers import decoded_flip_report
    d = torch.tensor([[0.50, 0.50, 0.20, 0.20, 0.90, 0.90],    # row 0: kept
                      [0.51, 0.50, 0.20, 0.20, 0.89, 0.90],    # row 1: suppressed by 0
                      [0.10, 0.10, 0.05, 0.05, 0.60, 0.50],    # row 2: score 0.30, at conf
                      [0.90, 0.90, 0.05, 0.05, 0.80, 0.80]])   # row 3: alone
    r = decoded_flip_report(d, d, 1, 0.3, 0.3)
    assert r['keep_flips'] == 0 and r['member_flips'] == 0 and r['unexplained_flips'] == 0
    e = d.clone()
    e[1, 4] = 0.91  # row 1 now outranks row 0: the kept box changes (two flips, one class)
    e[2, 4] = 0.599  # score 0.2995: below conf on the device side only
    r = decoded_flip_report(e, d, 1, 0.3, 0.3)
    assert r['keep_flips'] == 3 and r['member_flips'] == 1 and r['member_far'] == 0, r
    assert r['unexplained_flips'] == 0 and r['flip_classes'] == 1, r
