"""The per-detection record ``predict`` emits (utils/target_box.py:8-38 in the
reference): pixel corners, score, label name and a drawing colour, with the
reference's accessors, so code written against its ``predict`` output keeps
working. ``colors_for`` gives the reference's evenly spaced HSV palette
(utils/helper_cv.py:60-64)."""
import colorsys


class TargetBox:
    """One kept box in original-image pixels: left/top/right/bottom, score
    (obj * cls_conf), label (the plan's class name) and colour (RGB ints)."""

    def __init__(self, box_xyxy, score, label, color):
        self.left, self.top, self.right, self.bottom = (box_xyxy[0], box_xyxy[1], box_xyxy[2], box_xyxy[3])
        self.score = score
        self.label = label
        self.color = color

    def get_topleft(self):
        return self.left, self.top

    def get_bottomright(self):
        return self.right, self.bottom

    def as_dict(self):
        return dict(box=[self.left, self.top, self.right, self.bottom], score=self.score, label=self.label)

    def __str__(self):
        bar = "-" * 20
        lines = [f"{bar}{type(self).__name__}{bar}"]
        lines += [f"{k:>20s} :\t{v}" for k, v in vars(self).items()]
        return "\r\n".join(lines) + "\r\n"


def colors_for(n):
    """n colours at hue i/n, full saturation and value, as 0-255 int triples."""
    out = []
    for i in range(n):
        r, g, b = colorsys.hsv_to_rgb(i / n, 1.0, 1.0)
        out.append((int(r * 255), int(g * 255), int(b * 255)))
    return out
