"""The deferred weight-gradient queue (models/modules/linear.py) on the CPU: products of one shape
batched, a weight used twice summed, a weight split over row ranges (the self-attention in_proj's
q / k | v) assembled, bias gradients as column sums; flush points flush inside the backward."""
import torch

from conftest import PKG

L = PKG.models.modules.linear


def _entries(seed=0):
    g = torch.Generator().manual_seed(seed)
    r = lambda *s: torch.randn(*s, generator=g)  # noqa: E731
    w1, b1 = torch.nn.Parameter(r(6, 5)), torch.nn.Parameter(r(6))
    w2, b2 = torch.nn.Parameter(r(6, 5)), torch.nn.Parameter(r(6))
    w3, b3 = torch.nn.Parameter(r(9, 5)), torch.nn.Parameter(r(9))  # rows [0, 6) and [6, 9)
    w4 = torch.nn.Parameter(r(6, 5))
    es = [(r(7, 6), r(7, 5), w1, 0, b1), (r(7, 6), r(7, 5), w2, 0, b2), (r(7, 6), r(7, 5), w1, 0, b1),
          (r(4, 6), r(4, 5), w3, 0, b3), (r(4, 3), r(4, 5), w3, 6, b3), (r(7, 6), r(7, 5), w4, 0, None)]
    return es


def test_flush_groups_and_assembles():
    es = _entries()
    want = {}
    for g2, x2, w, row, b in es:
        dw = torch.zeros_like(w)
        dw[row:row + g2.shape[1]] = g2.t() @ x2
        want[w] = want.get(w, 0) + dw
        if b is not None:
            db = torch.zeros_like(b)
            db[row:row + g2.shape[1]] = g2.sum(0)
            want[b] = want.get(b, 0) + db
    got = {}
    with L.deferred_weight_grads(lambda p, grad: got.__setitem__(p, got.get(p, 0) + grad)) as q:
        for e in es:
            assert L._defer(e)
        q.flush()
        assert q.entries == []
    assert set(got) == set(want)
    for p in want:
        torch.testing.assert_close(got[p], want[p], rtol=1e-5, atol=1e-5)


def test_defer_refuses_long_k_and_inactive_queue():
    g2, x2, w, row, b = _entries()[0]
    assert not L._defer((g2, x2, w, row, b))  # no active queue
    with L.deferred_weight_grads(lambda p, grad: None) as q:
        big = torch.zeros(L.DEFER_MAX_ROWS + 1, 6)
        # all or none: a long-K product keeps its short-K companion out of the queue too
        assert not L._defer((g2, x2, w, row, b), (big, torch.zeros(L.DEFER_MAX_ROWS + 1, 5), w, 0, b))
        assert q.entries == []


def test_flush_point_flushes_inside_backward():
    es = _entries()
    order = []
    x = torch.randn(3, requires_grad=True)
    with L.deferred_weight_grads(lambda p, grad: order.append("deliver")) as q:
        for e in es[:2]:
            L._defer(e)
        y = L.flush_point(x * 2)
        y.register_hook(lambda g: order.append("before"))
        (y.sum() * 3).backward()
        order.append("after")
        assert q.entries == []
    assert order[0] == "before" and order[-1] == "after" and order.count("deliver") == 4
