"""1-D segment geometry, reference utils/box_ops.py:1-70 (centre/length <-> start/end, IoU, gIoU)."""
import torch

__all__ = ["segment_cl_to_xy", "segment_xy_to_cl", "box_iou", "generalized_box_iou", "generalized_box_iou_unchecked"]


def segment_cl_to_xy(x):
    c, l = x.unbind(-1)
    return torch.stack([c - 0.5 * l, c + 0.5 * l], dim=-1)


def segment_xy_to_cl(x):
    x, y = x.unbind(-1)
    return torch.stack([(x + y) / 2, (y - x)], dim=-1)


def box_iou(segment1, segment2):
    area1 = segment1[:, 1] - segment1[:, 0]
    area2 = segment2[:, 1] - segment2[:, 0]
    lt = torch.max(segment1[:, None, 0], segment2[:, 0])
    rb = torch.min(segment1[:, None, 1], segment2[:, 1])
    inter = (rb - lt).clamp(min=0)
    union = area1[:, None] + area2 - inter
    return inter / (union + 1e-5), union


def generalized_box_iou_unchecked(segment1, segment2):
    """gIoU matrix (N, M) without the well-formedness asserts (no device->host sync); callers check
    ``segments_well_formed`` on the host copy they already make."""
    iou, union = box_iou(segment1, segment2)
    lt = torch.min(segment1[:, None, 0], segment2[:, 0])
    rb = torch.max(segment1[:, None, 1], segment2[:, 1])
    area = (rb - lt).clamp(min=0)
    return iou - (area - union) / (area + 1e-5)


def generalized_box_iou(segment1, segment2):
    """reference :52-70, asserts included."""
    assert (segment1[:, 1] >= segment1[:, 0]).all(), "Segment start > Segment end (from output)"
    assert (segment2[:, 1] >= segment2[:, 0]).all(), "Segment start > Segment end (from target)"
    return generalized_box_iou_unchecked(segment1, segment2)
