"""Image-side steps on the GPU:
ycx_letterbox vs the CPU restatement (bit-exact fp32), ycx_correct_boxes vs the
reference's numpy yolo_correct_boxes (bit-exact), headless predict()."""
import numpy as np
import pytest
import torch
import yaml

from helpers import ANCHORS, MASK, rel_err
from oracle import ref_letterbox
from ycx.utils.target_box import TargetBox
from ycx.detect import correct_boxes_device, predict, yolo_correct_boxes
from ycx.utils.letterbox import letterbox_geometry, letterbox_gpu

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('hw', [(512, 773), (640, 640), (900, 300), (3, 5), (1080, 1920), (480, 640)])
def test_letterbox_matches_restatement(device, hw):
    g = np.random.default_rng(hw[0] * 7 + hw[1])
    img = g.integers(0, 256, size=(*hw, 3), dtype=np.uint8)
    want = ref_letterbox.letterbox_tensor(img, (640, 640))
    got = letterbox_gpu(img, (640, 640), device=device).cpu().numpy()
    assert got.shape == want.shape
    np.testing.assert_array_equal(got, want)
    assert letterbox_geometry(*hw) == ref_letterbox.letterbox_geometry(*hw)


def test_letterbox_into_batch_slot(device):
    imgs = [np.full((100, 200, 3), v, dtype=np.uint8) for v in (0, 255)]
    batch = torch.zeros((2, 3, 320, 320), device=device)
    for i, im in enumerate(imgs):
        letterbox_gpu(im, (320, 320), out=batch[i])
    b = batch.cpu().numpy()
    for i, im in enumerate(imgs):
        np.testing.assert_array_equal(b[i], ref_letterbox.letterbox_tensor(im, (320, 320)))


def test_letterbox_batch_matches_restatement(device):
    """ycx_letterbox_batch (one launch for a whole batch, bench.py --image-in) ==
    the CPU restatement image by image, bit for bit."""
    from ycx.utils.letterbox import letterbox_batch_gpu
    g = np.random.default_rng(5)
    imgs = g.integers(0, 256, size=(5, 512, 773, 3), dtype=np.uint8)
    out = torch.full((5, 3, 640, 640), -1.0, device=device)
    letterbox_batch_gpu(torch.from_numpy(imgs).to(device), out)
    got = out.cpu().numpy()
    for i in range(5):
        np.testing.assert_array_equal(got[i], ref_letterbox.letterbox_tensor(imgs[i], (640, 640)))


@pytest.mark.parametrize('letterbox_image', [True, False])
@pytest.mark.parametrize('image_hw', [(512, 773), (1080, 1920), (640, 640), (333, 777)])
def test_correct_boxes_matches_numpy(device, letterbox_image, image_hw):
    g = np.random.default_rng(sum(image_hw))
    n, max_det = 3, 50
    dets = np.zeros((n, max_det, 7), dtype=np.float32)
    xy = g.random((n, max_det, 2), dtype=np.float32)
    wh = g.random((n, max_det, 2), dtype=np.float32) * 0.3
    dets[..., 0:2], dets[..., 2:4] = xy, xy + wh
    dets[..., 4:7] = g.random((n, max_det, 3), dtype=np.float32)
    counts = np.array([0, 17, 60], dtype=np.int32)  # empty, partial, more than max_det
    got = correct_boxes_device(torch.from_numpy(dets).to(device), torch.from_numpy(counts).to(device), (640, 640),
                               np.array(image_hw), letterbox_image).cpu().numpy()
    for i in range(n):
        k = min(int(counts[i]), max_det)
        o = dets[i, :k].copy()
        box_xy, box_wh = (o[:, 0:2] + o[:, 2:4]) / 2, o[:, 2:4] - o[:, 0:2]
        o[:, :4] = yolo_correct_boxes(box_xy, box_wh, (640, 640), np.array(image_hw), letterbox_image)
        np.testing.assert_array_equal(got[i, :k], o)
        np.testing.assert_array_equal(got[i, k:], dets[i, k:])  # rows past the count untouched


def test_predict_headless(device, tmp_path):
    plan = dict(device=0, image_size=640, image_chan=3, labels=['raccoon'], model_cfg='yolov7-tiny',
                anchors=ANCHORS, anchors_mask=MASK)
    cfg = tmp_path / 'plan.yaml'
    cfg.write_text(yaml.safe_dump(plan))
    img = np.random.default_rng(0).integers(0, 256, size=(512, 773, 3), dtype=np.uint8)
    boxes = predict(str(cfg), image=img, weights='synthetic', device='cuda:0', conf_threshold=0.3,
                    nms_threshold=0.3)
    assert isinstance(boxes, list)
    for b in boxes:  # detect.py:236-244 clamps each corner on one side only, like the reference
        x1, y1, x2, y2 = b.left, b.top, b.right, b.bottom
        assert x1 >= 0 and y1 >= 0 and x2 <= 773 and y2 <= 512 and b.label == 'raccoon'
    assert all(isinstance(b, TargetBox) for b in boxes)


@pytest.mark.parametrize('precision,size,hw', [('f32', 320, (287, 411)), ('f32', 640, (512, 773)),
                                               ('fp16', 640, (512, 773))])
def test_predict_vs_oracle_chain(device, tmp_path, precision, size, hw):
    """predict (detect.py:208-265) against the oracle chain on the same image: the
    letterbox restatement (oracle/ref_letterbox.py), the fp32 forward
    (oracle/ref_forward.py), decode_box + non_max_suppression + yolo_correct_boxes
    (oracle/ref_post.py), then detect.py:236-244's floor/clamp. f32 parity mode
    (1e-3): the same boxes in the same order (boxes whose oracle scores are within
    1e-5 may trade places), corners within one pixel (a floor can cross an integer),
    scores within 1e-3, same labels. fp16 (the
    default precision) at 640 on a 773x512 image, BASELINE C1's plumbing shape (also
    run in f32, strictly): the seeded weights keep ~1.9k heavily overlapping boxes of
    the one class, so a score that moves by ~1e-4 can flip a greedy decision and the
    flips cascade (r03: 44 of 1934 boxes differ). The difference is decomposed: predict's
    boxes are exactly the device chain's rows; the oracle's NMS on the device's own decoded
    tensor keeps exactly the device's rows; the decoded tensors are within 1e-3; and the
    first keep flip of every class is caused by a threshold crossing, a score swap or an
    IoU crossing under the forward's perturbation (helpers.decoded_flip_report)."""
    from oracle import ref_forward, ref_letterbox, ref_post
    from ycx.utils.helper_io import cvt_cfg
    from ycx.utils.synth import synthetic_state_dict
    plan = dict(device=0, image_size=size, image_chan=3, labels=['raccoon'], model_cfg='yolov7-tiny',
                anchors=ANCHORS, anchors_mask=MASK)
    cfg = tmp_path / 'plan.yaml'
    cfg.write_text(yaml.safe_dump(plan))
    img = np.random.default_rng(4).integers(0, 256, size=hw + (3,), dtype=np.uint8)
    got = predict(str(cfg), image=img, weights='synthetic', device='cuda:0', conf_threshold=0.3,
                  nms_threshold=0.3, precision=precision)
    net_cfg = cvt_cfg('yolov7-tiny')
    from ycx.nets.yolo import Model
    sd = synthetic_state_dict(Model(net_cfg, ANCHORS, 1), seed=0)
    x = torch.from_numpy(ref_letterbox.letterbox_tensor(img, (size, size))).unsqueeze(0)
    heads = ref_forward.build(net_cfg, ANCHORS, 1, sd)(x)
    A = np.asarray(ANCHORS).reshape(-1, 2)
    dec = torch.cat(ref_post.decode_box(heads, A, MASK, 1, (size, size)), 1)
    res = ref_post.non_max_suppression(dec, 1, (size, size), np.array(img.shape[0:2]), True, 0.3, 0.3)[0]
    assert res is not None and len(res) > 0

    def close(tb, row):
        y1, x1, y2, x2 = row[0], row[1], row[2], row[3]
        want = [max(0, int(np.floor(x1))), max(0, int(np.floor(y1))),
                min(img.shape[1], int(np.floor(x2))), min(img.shape[0], int(np.floor(y2)))]
        return (max(abs(a - b) for a, b in zip([tb.left, tb.top, tb.right, tb.bottom], want)) <= 1 and
                abs(float(tb.score) - float(row[4] * row[5])) <= 1e-3)

    assert all(tb.label == 'raccoon' and tb.color == (255, 0, 0) for tb in got)
    if precision == 'f32':
        assert len(got) == len(res), (len(got), len(res))
        # same boxes in the same order, except that boxes whose scores the oracle itself puts
        # within 1e-5 of each other (far inside the 1e-3 forward tolerance) may trade places:
        # measured r03 on MI355X, 3 adjacent swaps in 1934 rows, score gaps <= 2e-7
        score = [float(r[4] * r[5]) for r in res]
        used, bad = set(), []
        for i, tb in enumerate(got):
            js = [j for j in range(max(0, i - 4), min(len(res), i + 5))
                  if j not in used and (j == i or abs(score[j] - score[i]) <= 1e-5) and close(tb, res[j])]
            if not js:
                bad.append((i, (tb.left, tb.top, tb.right, tb.bottom, float(tb.score)), score[i]))
            else:
                used.add(i if i in js else js[0])
        assert not bad, (len(bad), bad[:4])
        return
    # fp16: the difference to the oracle is decomposed, as the C2 tests do.
    # 1. the same chain predict() ran, step by step on the device: letterbox -> fp16 forward ->
    #    decode_box -> non_max_suppression; predict's boxes are exactly this chain's rows
    from ycx.detect import decode_box, nms_device, non_max_suppression
    from helpers import decoded_flip_report  # noqa: E402
    m = Model(net_cfg, ANCHORS, 1, precision='fp16').eval()
    m.load_state_dict(sd)
    m.to('cuda:0')
    xd = letterbox_gpu(img, (size, size), device='cuda:0').unsqueeze(0)
    assert torch.equal(xd.cpu(), x)  # the device letterbox is bit-exact to the restatement
    heads_dev = m(xd)
    dec_dev = torch.cat(decode_box(heads_dev, A, MASK, 1, (size, size)), 1)
    mine = non_max_suppression(dec_dev.clone(), 1, (size, size), np.array(img.shape[0:2]), True, 0.3, 0.3)[0]
    assert len(mine) == len(got)
    for tb, row in zip(got, mine):
        y1, x1, y2, x2 = row[0], row[1], row[2], row[3]
        assert [tb.left, tb.top, tb.right, tb.bottom] == [
            max(0, int(np.floor(x1))), max(0, int(np.floor(y1))),
            min(img.shape[1], int(np.floor(x2))), min(img.shape[0], int(np.floor(y2)))]
        assert float(tb.score) == float(row[4] * row[5])
    # 2. NMS: the oracle's greedy chain on the DEVICE's own decoded tensor keeps exactly the
    #    device's rows, in the device's order (bit-exact keep indices on identical inputs)
    _, keep_d, kc_d = nms_device(dec_dev.clone(), 1, 0.3, 0.3)
    keep_d = keep_d[0, :int(kc_d[0])].cpu().numpy().astype(np.int64)
    own = ref_post.nms_keep_rows(dec_dev.cpu().clone(), 1, 0.3, 0.3)[0][0].numpy()
    assert np.array_equal(keep_d, own), (len(keep_d), len(own))
    # 3. forward: the decoded box / objectness / class-confidence tensors within north_star's 1e-3
    #    (dec itself is xyxy now: non_max_suppression rewrote it in place, detect.py:98-103)
    dec = torch.cat(ref_post.decode_box(heads, A, MASK, 1, (size, size)), 1)
    errs = {k: rel_err(dec_dev[0, :, sl].cpu(), dec[0, :, sl]) for k, sl in
            (('box', slice(0, 4)), ('obj', slice(4, 5)), ('cls', slice(5, 6)))}
    assert max(errs.values()) < 1e-3, errs
    # 4. end to end: every keep-set difference between the two chains is caused by the
    #    forward's perturbation (a threshold crossing, a score swap or an IoU crossing)
    rep = decoded_flip_report(dec_dev[0], dec[0], 1, 0.3, 0.3)
    print(f"\nfp16 predict at {size} ({hw}): {len(got)} boxes, oracle {len(res)}; decoded err {errs}; {rep}")
    assert rep['member_far'] == 0 and rep['cls_flips'] == 0, rep
    assert rep['unexplained_flips'] == 0, rep

