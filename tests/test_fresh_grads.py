"""Host logic of the deferred gradient zeros (ops.FRESH, FusedAdamW.zero_grad
(defer=True)): the trainer's update fills only the gradients no conv backward
writes whole; the rest are overwritten by their first writer in the next
backward.  CPU tensors only (no kernel runs): which writer gets accumulate =
False, which zeros become real (zero=True sites, autograd accumulation,
finish()), the per-owner pending sets and the zero spans.  The GPU side --
the trained result identical with and without the deferral, eager and
replayed -- is tests/test_fresh_grads_gpu.py."""
import torch

from dalle2_video import ops
from dalle2_video.trainer import FusedAdamW


def _params(*sizes):
    ps = [torch.nn.Parameter(torch.randn(k)) for k in sizes]
    for p in ps:
        p.grad = torch.full_like(p, 5.0)  # a previous step's gradient
    return ps


def test_deferred_zero_writers():
    a, b, c, d, e = _params(40, 7, 33, 16, 9)
    opt = FusedAdamW([a, b, c, d, e])
    assert opt.ensure_flat()
    for p in (a, b, d, e):  # written whole by a conv backward once
        assert ops._grad_out(p, overwrite=True) == (p.grad, True)
    for p in (a, b, c, d, e):
        p.grad.fill_(5.0)  # (the flat buffer's alignment gaps are never written)
    opt.zero_grad(defer=True)
    assert torch.all(c.grad == 0)  # not a conv gradient: zeroed for real
    for p in (a, b, d, e):
        assert torch.all(p.grad == 5.0)  # logically zero
    assert ops.FRESH.token(opt) is not None
    # the conv writer overwrites (accumulate = False) once, then accumulates
    assert ops._grad_out(a, overwrite=True)[1] is False
    assert ops._grad_out(a, overwrite=True)[1] is True
    # a site that adds into a zeroed buffer gets a real zero
    buf, acc = ops._grad_out(b, zero=True)
    assert acc is True and torch.all(b.grad == 0)
    # autograd accumulating into a deferred gradient: zeroed first (leaf pre-hook)
    (d * 2.0).sum().backward()
    assert torch.all(d.grad == 2.0)
    # e was never written: finish() zeroes it
    assert ops.FRESH.finish(opt) is True
    assert torch.all(e.grad == 0)
    assert ops.FRESH.finish(opt) is False and ops.FRESH.token(opt) is None
    # the gaps between parameters stay zero throughout
    G = opt.flat_grad
    live = torch.zeros_like(G, dtype=torch.bool)
    for p in (a, b, c, d, e):
        off = opt._offsets[id(p)]
        live[off:off + p.numel()] = True
    assert torch.all(G[~live] == 0)


def test_plain_zero_grad_drops_the_deferral():
    a, c = _params(20, 20)
    opt = FusedAdamW([a, c])
    opt.ensure_flat()
    ops._grad_out(a, overwrite=True)
    opt.zero_grad(defer=True)
    assert torch.all(a.grad == 5.0)
    opt.zero_grad()
    assert torch.all(opt.flat_grad == 0) and ops.FRESH.token(opt) is None
    assert ops._grad_out(a, overwrite=True)[1] is True  # nothing pending: accumulate


def test_owners_are_independent_and_switch_is_honoured():
    a, b = _params(24, 24)
    o1, o2 = FusedAdamW([a]), FusedAdamW([b])
    for o, p in ((o1, a), (o2, b)):
        o.ensure_flat()
        ops._grad_out(p, overwrite=True)
        o.zero_grad(defer=True)
    assert ops.FRESH.finish(o1) is True
    assert torch.all(a.grad == 0) and torch.all(b.grad == 5.0)  # o2's deferral untouched
    assert ops.FRESH.token(o2) is not None
    ops.FRESH.consume(o2)  # (a replayed graph settled it)
    assert ops.FRESH.token(o2) is None
    old = ops.GRAD_OVERWRITE
    try:
        ops.GRAD_OVERWRITE = False
        b.grad.fill_(3.0)
        o2.zero_grad(defer=True)
        assert torch.all(b.grad == 0) and ops.FRESH.token(o2) is None
    finally:
        ops.GRAD_OVERWRITE = old


def test_zero_spans_cover_exactly_the_other_parameters():
    ps = _params(5, 17, 3, 40, 1, 16, 9)
    opt = FusedAdamW(ps)
    opt.ensure_flat()
    armed = {id(ps[1]), id(ps[3]), id(ps[6])}
    spans = opt._zero_spans(armed)
    G = opt.flat_grad
    covered = torch.zeros_like(G, dtype=torch.bool)
    for s in spans:
        assert s.data_ptr() >= G.data_ptr()
        off = (s.data_ptr() - G.data_ptr()) // 4
        covered[off:off + s.numel()] = True
    for p in ps:
        off = opt._offsets[id(p)]
        want = id(p) not in armed
        assert bool(covered[off:off + p.numel()].all()) == want
        assert bool(covered[off:off + p.numel()].any()) == want
    assert len(spans) == 3  # {0}, {2}, {4, 5}: adjacent parameters merged


def test_dropped_owner_leaves_no_entries():
    """A trainer that goes away takes its deferred zeros with it (weakref
    callback), so the per-call bookkeeping of the live ones never scans them."""
    import gc

    keep = _params(16, 16)
    ok = FusedAdamW(keep)
    ok.ensure_flat()
    for p in keep:
        ops._grad_out(p, overwrite=True)
    ok.zero_grad(defer=True)
    before = len(ops.FRESH.pending)
    gone = _params(32, 32, 32)
    og = FusedAdamW(gone)
    og.ensure_flat()
    for p in gone:
        ops._grad_out(p, overwrite=True)
    og.zero_grad(defer=True)
    assert len(ops.FRESH.pending) == before + 3
    del og, gone, p
    gc.collect()
    assert len(ops.FRESH.pending) == before
    assert ops.FRESH.token(ok) is not None and len(ops.FRESH._mine(ok)) == 2
    ops.FRESH.drop(keep)
