"""Autograd-visible ops of the HIP path, over channels-last frame tensors.

An activation is a (NF, H, W, C) tensor (NF = batch*frames) whose channel
dimension is unit-stride; its pixel stride `ld` may exceed C (a channel
slice of a wider buffer).  Every op calls libdv_hip through `_lib.call`; there
is no torch-compute fallback.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import ACT_NONE, call, dt, ptr, require_gpu, stream


class KernelTimer:
    """Optional live per-kernel timing with HIP events on the launching stream
    (bench.py uses it for the roofline of the dominant kernel)."""

    def __init__(self):
        self.records = []  # (name, shape, flops, bytes, start_event, end_event)
        # name -> the most recent launch closures (replay_ms needs one step's):
        # bounded, since each closure keeps its tensors alive
        self.fns = {}

    # a short device-side spin before each timed launch keeps the GPU behind the
    # host, so the start event, the kernel and the end event run back to back and
    # the elapsed time is the kernel's own (not host launch gaps)
    SPIN_CYCLES = 400_000
    KEEP_FNS = 128  # launch closures kept per kernel name (>= one step's launches)

    def run(self, name, flops, nbytes, fn, shape=None):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(self.SPIN_CYCLES)
        s.record()
        fn()
        e.record()
        self.records.append((name, shape, flops, nbytes, s, e))
        q = self.fns.get(name)
        if q is None:
            import collections
            q = self.fns[name] = collections.deque(maxlen=self.KEEP_FNS)
        q.append(fn)

    def replay_ms(self, name, n_launch, reps=10):
        """Per-launch device time of kernel `name` the way a kernel trace sees
        it: its last `n_launch` launches (one step's) captured back to back in
        a HIP graph with no event brackets between them, replayed `reps`
        times; elapsed / (reps * n_launch).  Includes the ~1.5 us kernel
        boundaries (MI355X_MICROARCH.md, boundary row): a slight upper bound.

        The replayed launches write their real outputs again (a dgrad whose
        residual is its own output, a wgrad accumulating into a leaf's .grad):
        the caller's training state is not valid after this call (bench.py
        uses the trainer for nothing afterwards)."""
        fns = list(self.fns[name])[-n_launch:]
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for f in fns:
                f()
        g.replay()
        torch.cuda.synchronize()
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            g.replay()
        e.record()
        torch.cuda.synchronize()
        del g
        return s.elapsed_time(e) / (reps * len(fns))

    def overhead_ms(self, n=32):
        """Median elapsed time of an EMPTY start/end event pair recorded the
        same way (after the spin): the fixed cost the event brackets add to
        every timed launch, subtracted in summary()."""
        pairs = []
        for _ in range(n):
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(self.SPIN_CYCLES)
            s.record()
            e.record()
            pairs.append((s, e))
        torch.cuda.synchronize()
        v = sorted(s.elapsed_time(e) for s, e in pairs)
        return v[len(v) // 2]

    def summary(self, by_shape=False):
        """{name: totals} (or {(name, shape): totals} with by_shape=True; shape
        is the (M, N, K) GEMM view of a conv launch)."""
        torch.cuda.synchronize()
        if getattr(self, "event_overhead_ms", None) is None:
            self.event_overhead_ms = self.overhead_ms()
        ovh = self.event_overhead_ms
        out = {}
        for name, shape, fl, nb, s, e in self.records:
            d = out.setdefault((name, shape) if by_shape else name,
                               dict(count=0, flops=0.0, bytes=0.0, ms=0.0, ms_raw=0.0))
            d["count"] += 1
            d["flops"] += fl
            d["bytes"] += nb
            d["ms"] += max(s.elapsed_time(e) - ovh, 1e-4)
            d["ms_raw"] += s.elapsed_time(e)
        return out


TIMER = None  # set to a KernelTimer to time kernel launches


def _launch(name, flops, nbytes, fn, shape=None):
    if TIMER is None:
        fn()
    else:
        TIMER.run(name, flops, nbytes, fn, shape)


def conv_fwd_name(dtype_name, m, cin, c0, cout, maxld, ks=1, h=0, w=0, gn_P=0, nres2=False):
    """Kernel instantiation dv_conv_fwd dispatches to (mirror of conv_fwd_t /
    glds_tile in dv_conv.hip) — names the launch for the live roofline."""
    if (dtype_name == "bf16" and ks == 3 and cin == 64 and c0 == cin and cout % 64 == 0
            and w in (32, 64, 128) and h % (128 // w) == 0 and m % 128 == 0 and m * maxld < (1 << 31)
            and gn_P % 128 == 0):
        return f"conv_fwd_stripe_kernel<{w}>"
    if (dtype_name == "bf16" and ks == 3 and cin == 128 and c0 == 64 and cout % 64 == 0
            and (gn_P == 0 or (w == 64 and gn_P % 128 == 0)) and not nres2 and w in (32, 64, 128) and h % (128 // w) == 0 and m % 128 == 0
            and m * maxld < (1 << 31)):
        return f"conv_fwd_stripe_kernel<{w}>"  # dual source: two stripe passes (conv_fwd_t)
    if (dtype_name == "bf16" and ks == 3 and cin % 32 == 0 and c0 % 32 == 0 and cout % 64 == 0
            and m % 128 == 0 and m * maxld < (1 << 31) and _stripe_geom_ok(h, w)
            and (w == 8 or (w == 16 and cin * cout <= 256 * 256))):
        return f"conv_fwd_stripe2_kernel<{w}>"
    if (dtype_name == "bf16" and ks == 1 and cin in (64, 128) and c0 in (cin, 64) and cout in (64, 128)
            and gn_P == 0 and not nres2 and m * maxld < (1 << 31)):
        return f"conv1x1_stream_kernel<{cout},{cin // 64}>"
    if dtype_name == "bf16" and cin % 64 == 0 and c0 % 64 == 0 and m * maxld < (1 << 31):
        bn = 64 if cout <= 64 else 128
        bm = 256 if bn == 64 else 128
        if ((m + bm - 1) // bm) * ((cout + bn - 1) // bn) < 512:
            bm = 128
        if bn == 128 and ((m + 127) // 128) * ((cout + 127) // 128) < 256:
            bm = 64
        nb = ((m + bm - 1) // bm) * ((cout + bn - 1) // bn)
        buf = (bm + bn) * 128
        deep, mid = min(6, 160 * 1024 // buf), min(3, 80 * 1024 // buf)
        nbuf = deep if nb <= 256 else (mid if nb <= 512 and mid >= 3 else 2)
        return f"conv_fwd_glds_kernel<{bm},{bn},{nbuf}>"
    bm, bn = conv_tile(m, cout)
    return f"conv_fwd_kernel<{dtype_name},{bm},{bn}>"


# measured (round 2, per-shape kernel bench): the window form wins at 8x8 and
# 16x16, the glds / stripe kernels at 32x32 and 64x64
_WINDOW_W = (8, 16)


def window_ok(x0, x1, cin, c0, cout, ld0, ld1, ldy, ldres, ksize, h, w, nf, gn_P=0, ldres2=0):
    """Mirror of fwd_frame_ok (dv_conv.hip): the window-form 3x3 conv (dv_conv_fwd8);
    with the GroupNorm statistics epilogue its clips must be whole 128-pixel tiles."""
    geom = (h == 8 and w == 8 and nf % 2 == 0) or (w in (16, 32, 64) and (h * w) % 128 == 0)
    return (w in _WINDOW_W and x0.dtype == torch.bfloat16 and ksize == 3
            and gn_P % 128 == 0
            and geom and cin % 16 == 0 and c0 % 16 == 0 and cout % 64 == 0
            and not (cin == 64 and c0 == cin and w in (32, 64, 128))  # the resident-weight stripe kernel
            and ld0 % 8 == 0 and ld1 % 8 == 0 and ldy % 4 == 0 and ldres % 4 == 0 and ldres2 % 4 == 0
            and nf * h * w * max(ld0, ld1) * 2 < (1 << 31)
            and x0.data_ptr() % 16 == 0 and (x1 is None or x1.data_ptr() % 16 == 0))


def _stripe_geom_ok(h, w):
    """Mirror of stripe_geom() in dv_conv.hip (128-pixel stage windows)."""
    if w not in (8, 16, 32, 64):
        return False
    if h * w >= 128:
        return h % (128 // w) == 0
    if 128 % (h * w):
        return False
    return (128 // (h * w)) * (h + 2) * (w + 2) <= (200 if w == 8 else (128 // w + 2) * (w + 2))


def conv_wgrad_name(dtype_name, m, cout, cin, c0, split, ks, h, w, maxld):
    """Mirror of dv_conv_wgrad's kernel choice (wgrad_stripe_ok / conv_wgrad_glds)."""
    if (dtype_name == "bf16" and ks == 1 and cin % 64 == 0 and cout % 64 == 0
            and (not split or c0 % 64 == 0) and m % 128 == 0):
        return "conv_wgrad_1x1_kernel"
    if (dtype_name == "bf16" and ks == 3 and cin % 64 == 0 and cout % 64 == 0
            and (not split or c0 % 64 == 0) and m % 128 == 0
            and ((w == 8 and h == 8) or (w == 16 and h % 8 == 0) or (w in (32, 64) and h % 4 == 0))):
        return f"conv_wgrad_win_kernel<{w}>"
    K = ks * ks * cin
    return gemm_wgrad_name(dtype_name, m, cout, K, maxld)


def gemm_wgrad_name(dtype_name, m, cout, K, maxld):
    """Mirror of conv_wgrad_t / conv_wgrad_glds's tile choice."""
    if dtype_name == "bf16" and m * maxld < (1 << 31) and cout * K < (1 << 31):
        if cout <= 64:
            return "conv_wgrad_glds_kernel<64,256>" if (K >= 2048 or K % 256 == 0) else "conv_wgrad_glds_kernel<64,128>"
        return "conv_wgrad_glds_kernel<128,128>"
    return f"conv_wgrad_kernel<{dtype_name}>"


def conv_tile(m, cout):
    """Mirror of conv_fwd_t's tile choice for the register-staged kernel."""
    mt128 = (m + 127) // 128
    bn = 64 if cout <= 64 else 128
    bm = 128
    if mt128 * ((cout + bn - 1) // bn) < 512:
        bm = 64
    if bm == 64 and bn == 128 and ((m + 63) // 64) * ((cout + 127) // 128) < 512:
        bn = 64
    return bm, bn


def cl_ld(t: torch.Tensor) -> int:
    """Pixel stride of a channels-last frame tensor (asserts the layout)."""
    if t.dim() != 4 or (t.stride(3) != 1 and t.shape[3] > 1):
        raise _lib.DVError(f"expected a channels-last (NF,H,W,C) tensor, got {tuple(t.shape)} "
                           f"strides {t.stride()}")
    nf, h, w, c = t.shape
    ld = t.stride(2) if w > 1 else (t.stride(1) if h > 1 else max(c, t.stride(0) if nf > 1 else c))
    if (w > 1 and h > 1 and t.stride(1) != w * ld) or (nf > 1 and h * w > 1 and t.stride(0) != h * w * ld):
        raise _lib.DVError(f"non-uniform pixel stride {t.stride()}")
    return ld


class _FreshGrads:
    """Gradients the trainer's update zeroed only logically (FusedAdamW.
    zero_grad(defer=True)): instead of a fill of the whole flat buffer before
    the next backward, the first in-place writer of such a gradient
    overwrites it (accumulate = False: the wgrad sums write dw instead of
    reading it back).  Only parameters the conv backward has written before
    (`whole(p)`: its whole dw / db in one write) are deferred; the rest are
    zeroed for real.  Correct for every other writer too: a zero=True site or
    an autograd AccumulateGrad (leaf pre-hook) zeroes the gradient first, and
    whatever is still pending when the owner's backward ends is zeroed by
    finish().  Pending sets are per owner (one optimizer per unet), so one
    unet's backward never touches another unet's deferred zeros.  Entries
    hold weak references (a dropped trainer keeps no buffers alive)."""

    def __init__(self):
        import weakref
        self.pending = {}  # id(p) -> (weakref p, owner key)
        self.owned = {}  # owner key id(owner) -> (weakref owner, ids pending): per-owner work stays O(own)
        self.tokens = weakref.WeakKeyDictionary()  # owner -> token of the armed set (graph signature)
        self.marks = 0  # parameters marked whole so far (a trainer's cached armed set is valid while equal)

    @staticmethod
    def whole(p):
        return getattr(p, "_dv_whole_grad", False)

    def _get(self, p):
        ent = self.pending.get(id(p))
        return ent if ent is not None and ent[0]() is p else None

    def _remove(self, k):
        ent = self.pending.pop(k)
        o = self.owned.get(ent[1])
        if o is not None:
            o[1].discard(k)

    def _own(self, owner):
        o = self.owned.get(id(owner))
        return o if o is not None and o[0]() is owner else None

    def _mine(self, owner):
        o = self._own(owner)
        if o is None:
            return []
        oid = id(owner)
        return [k for k in o[1] if self.pending.get(k, (None, None))[1] == oid and self.pending[k][0]() is not None]

    def _forget(self, oid, ref):
        """A dropped owner: its entries go (weakref callback)."""
        o = self.owned.get(oid)
        if o is None or o[0] is not ref:
            return
        del self.owned[oid]
        for k in o[1]:
            if self.pending.get(k, (None, None))[1] == oid:
                del self.pending[k]

    def plan(self, params):
        """(entries, token) for arm(): computed once per armed set (the
        trainer caches it), hooks registered on first use."""
        import weakref
        entries = []
        for p in params:
            if not getattr(p, "_dv_fresh_hook", False):
                p._dv_fresh_hook = True
                p.register_hook(self._pre_hook(weakref.ref(p)))
            entries.append((id(p), weakref.ref(p)))
        return entries, hash(tuple(sorted(k for k, _ in entries)))

    def arm(self, owner, params=None, plan=None):
        import weakref
        entries, token = plan if plan is not None else self.plan(params)
        oid = id(owner)
        o = self._own(owner)
        if o is None:
            o = self.owned[oid] = (weakref.ref(owner, lambda r, oid=oid: self._forget(oid, r)), set())
        # (an entry another owner still held is overwritten: that owner's
        # lookups check the entry's owner key, so it no longer sees it)
        self.pending.update((k, (w, oid)) for k, w in entries)
        o[1].update(k for k, _ in entries)
        self.tokens[owner] = token

    def _pre_hook(self, ref):
        def pre(g):
            q = ref()
            if g is not None and q is not None and self._get(q) is not None:
                self._remove(id(q))
                WGRAD_DEFER.before_write(q.grad.data_ptr())
                q.grad.zero_()  # autograd adds into it: the zero becomes real first
        return pre

    def token(self, owner):
        """Graph-signature part: which deferred zeros a call starts from."""
        o = self._own(owner)
        return self.tokens.get(owner) if o is not None and o[1] else None

    def drop(self, params):
        for p in params:
            if self._get(p) is not None:
                self._remove(id(p))

    def take(self, p, overwrite):
        """True: `p`'s gradient is logically zero and the caller overwrites it."""
        if self._get(p) is None:
            return False
        self._remove(id(p))
        if overwrite:
            return True
        WGRAD_DEFER.before_write(p.grad.data_ptr())
        p.grad.zero_()
        return False

    def finish(self, owner, sync=None):
        """Zero the owner's gradients still pending after its backward (after
        `sync()`: e.g. the join of gradient buckets already being reduced in
        place); True if there were any."""
        left = self._mine(owner)
        if not left:
            o = self._own(owner)
            if o is not None:
                o[1].clear()  # (entries of dropped parameters)
            return False
        if sync is not None:
            sync()
        grads = [self.pending[k][0]().grad for k in left]
        for k in left:
            self._remove(k)
        torch._foreach_zero_(grads)
        return True

    def consume(self, owner):
        """A replayed graph settled the owner's pending gradients (written, or
        zeroed by the finish() it captured)."""
        o = self._own(owner)
        if o is None:
            return
        oid = id(owner)
        for k in o[1]:
            if self.pending.get(k, (None, None))[1] == oid:
                del self.pending[k]
        o[1].clear()


FRESH = _FreshGrads()
GRAD_OVERWRITE = True  # FusedAdamW.zero_grad(defer=True) defers the conv gradients' zeros


def _grad_out(p, zero=False, overwrite=False):
    """In-place gradient target for a leaf parameter: (buffer, accumulate).

    Backward kernels write a parameter's gradient straight into `p.grad`
    (the trainer's flat-buffer view) and the autograd Function returns None
    for it, so no AccumulateGrad add runs.  Returns None when `p` is not a
    leaf that requires grad (the Function then returns the gradient).
    zero: the kernel adds into a zeroed buffer; overwrite: the caller writes
    the whole gradient in one kernel when told accumulate = False (the conv
    backward), so a deferred zero (FRESH) needs no fill."""
    if p is None or not (p.requires_grad and p.is_leaf) or p.dtype != torch.float32:
        return None
    if overwrite and not zero and not FRESH.whole(p):
        p._dv_whole_grad = True
        FRESH.marks += 1
    if p.grad is None:
        p.grad = (torch.zeros_like if zero else torch.empty_like)(p)
        return p.grad, False
    if FRESH.pending and FRESH.take(p, overwrite and not zero):
        return p.grad, False
    return p.grad, True


_WS = {}


def _wgrad_workspace(dname, nf, h, w, cin, c0, split, cout, ks, device):
    """One cached f32 scratch per device for dv_conv_wgrad (grown on demand;
    kernels on the stream use it one after another)."""
    need = ctypes.c_longlong(0)
    call("dv_conv_wgrad_ws", _lib.DV_BF16 if dname == "bf16" else _lib.DV_F32, nf, h, w, cin, c0,
         int(split), cout, ks, ctypes.byref(need))
    key = str(device)
    buf = _WS.get(key)
    if buf is None or buf.numel() < need.value:
        buf = torch.empty(max(need.value, 1 << 20), dtype=torch.float32, device=device)
        _WS[key] = buf
    return buf


class _WgradDefer:
    """Deferred split-K sums of the row-window wgrad (dv_conv_wgrad_deferred).

    Inside `defer_wgrad()` (the trainer's forward + backward, captured or
    eager) every conv whose weight gradient goes straight into a leaf's .grad
    leaves its per-split partials in an arena slot instead of launching its
    own reduce; leaving the context sums them all in ONE launch
    (dv_wgrad_reduce_batched).  Slots are handed out in call order from the
    start of the arena each pass, so a replayed pass sees the same addresses;
    the device table is cached by content (built by the eager warm-up calls,
    reused by the captured one)."""

    CHUNK_FLOATS = 1 << 27  # 512 MB arena chunks (kept for the process: graphs hold their addresses)
    # flush once this many partial bytes are pending (0 = only at the end of
    # the pass): a smaller batch is read back while still in the 256 MB MALL
    FLUSH_BYTES = 0
    # streamed sums (STREAM = True; tests/test_trainer_gpu.py): each conv's split-K sum is launched
    # on a side stream right after its wgrad, to overlap the memory-bound sum
    # with the MFMA / LDS-bound convs of the rest of the backward; the side
    # stream is joined when the pass ends (and before any other kernel writes
    # a gradient a pending sum targets).  Measured slower on the whole step
    # (same box, tools/gpu_r03e.sh: 84.7 vs 95.3 steps/s — the side-stream
    # sums take CU slots and HBM from the 1-workgroup-per-CU convs), so the
    # default is one batched sum at the end of the pass.
    STREAM = False
    _sides = {}

    def __init__(self):
        self.active = 0
        self.pending = []  # DvWgradReduceEntry
        self.targets = set()
        self.chunks = {}  # device -> [tensor]
        self.cursor = (0, 0)
        self.tables = {}  # (device, bytes) -> (device table, blocks)
        self.streamed = None  # device whose side stream holds unjoined sums
        self.added = 0  # entries deferred in this pass (streamed or pending)

    def _side(self, device):
        key = str(device)
        if key not in self._sides:
            self._sides[key] = torch.cuda.Stream(device=device)
        return self._sides[key]

    def join(self):
        """The current stream waits for every streamed sum launched so far."""
        if self.streamed is not None:
            torch.cuda.current_stream(self.streamed).wait_stream(self._side(self.streamed))
            self.streamed = None
            self.targets.clear()

    def before_write(self, *ptrs):
        """Call before a kernel outside the deferral writes a gradient buffer:
        a pending (batched) or in-flight (streamed) sum into it lands first."""
        if any(p is not None and p in self.targets for p in ptrs):
            if self.streamed is not None:
                self.join()
            else:
                self.flush()

    def slot(self, device, floats):
        floats = (floats + 63) // 64 * 64
        chunks = self.chunks.setdefault(str(device), [])
        ci, off = self.cursor
        while True:
            if ci == len(chunks):
                chunks.append(torch.empty(max(self.CHUNK_FLOATS, floats), dtype=torch.float32, device=device))
            if off + floats <= chunks[ci].numel():
                self.cursor = (ci, off + floats)
                return chunks[ci], off
            ci, off = ci + 1, 0

    def add(self, entry, device):
        self.added += 1
        if self.STREAM:
            main = torch.cuda.current_stream(device)
            side = self._side(device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                call("dv_wgrad_reduce_one", ctypes.byref(entry), stream())
            self.streamed = device
            self.targets.add(entry.dw)
            if entry.db:
                self.targets.add(entry.db)
            return
        self.pending.append((entry, device))
        self.targets.add(entry.dw)
        if entry.db:
            self.targets.add(entry.db)
        self.pending_bytes = getattr(self, "pending_bytes", 0) + 16 * entry.S * entry.n4
        if self.FLUSH_BYTES and self.pending_bytes >= self.FLUSH_BYTES:
            self.flush()

    def conflicts(self, *ptrs):
        return any(p is not None and p in self.targets for p in ptrs)

    def flush(self):
        self.join()
        if not self.pending:
            self.cursor = (0, 0)
            return
        dev = self.pending[0][1]
        n = len(self.pending)
        host = (_lib.DvWgradReduceEntry * n)(*[e for e, _ in self.pending])
        nblk = ctypes.c_longlong(0)
        call("dv_wgrad_reduce_plan", ctypes.byref(host), n, ctypes.byref(nblk))
        blocks = nblk.value
        key = (str(dev), bytes(host))
        tab = self.tables.get(key)
        if tab is None:
            if torch.cuda.is_current_stream_capturing():
                raise _lib.DVError("deferred wgrad table changed inside a captured region "
                                   "(run the same pass eagerly before capturing it)")
            raw = torch.frombuffer(bytearray(bytes(host)), dtype=torch.uint8)
            tab = self.tables[key] = raw.to(dev)
        call("dv_wgrad_reduce_batched", ptr(tab), n, blocks, stream())
        self.pending.clear()
        self.targets.clear()
        self.pending_bytes = 0
        self.cursor = (0, 0)

    def discard(self):
        self.join()
        self.added = 0
        self.pending.clear()
        self.targets.clear()
        self.pending_bytes = 0
        self.cursor = (0, 0)


WGRAD_DEFER = _WgradDefer()


class defer_wgrad:
    """Context: defer the split-K sums of the convs whose backward runs inside
    it and sum them all in one launch on exit (see _WgradDefer).  The
    gradients are complete only after the context exits."""

    def __enter__(self):
        if WGRAD_DEFER.active == 0:
            WGRAD_DEFER.discard()
        WGRAD_DEFER.active += 1
        return WGRAD_DEFER

    def __exit__(self, et, ev, tb):
        WGRAD_DEFER.active -= 1
        if WGRAD_DEFER.active == 0:
            if et is None:
                WGRAD_DEFER.flush()
            else:
                WGRAD_DEFER.discard()
        return False


_XA_WS = {}


def _xattn_workspace(nb, C, device, owner=None):
    """Cross-attention backward accumulators (wsR, wsV, wsQ [nb][32][C]): zero
    on entry, re-zeroed by dv_xattn_fold_bwd after use; mcorr [nb][32] scratch.
    `owner` (a block's parameter) gives the block its own set, for fold
    backwards deferred into one batched launch."""
    import weakref
    key = (nb, C, str(device), None if owner is None else id(owner))
    ent = _XA_WS.get(key)
    if ent is not None and (owner is None or ent[0]() is owner):
        return ent[1]
    if owner is not None:  # forget the sets of blocks that no longer exist
        for k in [k for k, e in _XA_WS.items() if e[0] is not None and e[0]() is None]:
            del _XA_WS[k]
    ws = tuple(torch.zeros(nb, 32, C, dtype=torch.float32, device=device) for _ in range(3)) + (
        torch.zeros(nb, 32, dtype=torch.float32, device=device),)
    _XA_WS[key] = (None if owner is None else weakref.ref(owner), ws)
    return ws


class _BackwardMarks:
    """Module-boundary marks for the trainer's overlapped gradient all-reduce:
    while a tracker is set, Unet3D's forward registers a hook on each block's
    input, so the tracker is called (in a fixed order) as the backward
    finishes each block."""
    tracker = None


def backward_mark(x):
    t = _BackwardMarks.tracker
    if t is not None and torch.is_grad_enabled() and x.requires_grad:
        x.register_hook(t.on_hit)


class _GnSums:
    """The rotating GroupNorm sums buffers of a device (dv_gn_fwd / dv_gn_bwd
    contract: `sums` zero on entry, `next` zeroed by the call): call i
    accumulates into buffer i % 3 and zeroes buffer (i + 2) % 3 = the previous
    call's sums, so buffer i % 3 was zeroed by call i - 2.  Three buffers, not
    two, so that a GroupNorm whose apply is folded into the next conv
    (group_norm_act(defer=...)) can have that conv read its sums while the
    next call already accumulates into its own: the folded conv takes over the
    deferred call's zeroing (dv_conv_fwd_gn_in's `zero`)."""

    # floats per buffer: up to 8 replicas of nb * C * 2 sums (<= 32768 floats
    # each) and, for the single-launch GroupNorm, nb arrival counters at the end
    CAP = 1 << 16

    def __init__(self, device):
        self.bufs = torch.zeros(3, self.CAP, dtype=torch.float32, device=device)
        self.i = 0

    def take(self, n):
        if n > self.CAP // 2:
            raise _lib.DVError(f"GroupNorm: nb*C*2 = {n} exceeds the sums buffer ({self.CAP})")
        cur, nxt = self.bufs[self.i % 3], self.bufs[(self.i + 2) % 3]
        self.i += 1
        return cur, nxt

    def reset(self):
        """Zero both buffers (one launch): ends a captured graph region so a
        replay starts from zero sums whatever the call-count parity."""
        _lib.call("dv_zero_f32", ptr(self.bufs), self.bufs.numel(), stream())


_GN_WS = {}


def _gn_sums(device):
    key = str(device)
    if key not in _GN_WS:
        _GN_WS[key] = _GnSums(device)
    return _GN_WS[key]


class GnStats:
    """The sums buffer a conv's statistics epilogue fills for the GroupNorm
    that reads its output (Block3D: project -> norm, dalle2_video.py:107-109):
    one take() of the alternating _GnSums pair, R replicas of [nb][C][2]."""

    # replicas: the conv's device-scope atomics serialise per address (they
    # resolve past the XCD L2s), so the statistics spread over as many
    # replicas as the buffer holds (<= 64); the apply sums them from L2
    MAX_R = 8
    ALL = False  # every conv kernel accumulates (tests/test_cfg2_gpu.py sets it)

    def __init__(self, nb, C, P, device):
        self.cur, self.nxt = _gn_sums(device).take(nb * C * 2)
        self.R = max(1, min(self.MAX_R, self.cur.numel() // (nb * C * 2)))
        self.P = P
        self.used = False  # set by the conv: did its epilogue accumulate?


def gn_stats(nb, C, P, device):
    return GnStats(nb, C, P, device)


def gn_graph_boundary(device):
    """Call at the end of a captured region that runs GroupNorms."""
    if str(device) in _GN_WS:
        _GN_WS[str(device)].reset()


def _grad_view(t: torch.Tensor):
    """(tensor, ld) of an incoming channels-last gradient: a channel slice of a
    wider buffer (GradSink's dX split for x0 / x1) is used in place through its
    pixel stride instead of being copied; anything else is made contiguous."""
    if t.is_contiguous():
        return t, t.shape[-1]
    try:
        ld = cl_ld(t)
        if ld % 8 == 0 and t.data_ptr() % 16 == 0:
            return t, ld
    except _lib.DVError:
        pass
    t = t.contiguous()
    return t, t.shape[-1]


def _pad_channels(t: torch.Tensor, mult: int = 8) -> torch.Tensor:
    c = t.shape[-1]
    cp = (c + mult - 1) // mult * mult
    if cp == c and t.is_contiguous():
        return t
    out = torch.zeros(*t.shape[:-1], cp, dtype=t.dtype, device=t.device)
    out[..., :c] = t
    return out


class PackCache:
    """Packed MFMA images of conv / token-linear weights, kept in fixed buffers.

    Disabled by default (every conv packs its weight on the fly).  The trainer
    enables it: weights then only change inside `update()`, which calls
    `refresh()` — ONE batched launch repacks every cached weight in place — so
    the forward/backward (and a captured HIP graph of them) launch no pack
    kernels.  An entry is reused only if the trainer's epoch and the weight's
    torch version counter (bumped by load_state_dict, EMA lerp_, ...) match."""

    def __init__(self):
        self.enabled = False
        self.static = False  # weights do not change while this cache is current (sampling)
        self.epoch = 0
        self.entries = {}  # key -> dict(out, w, meta, epoch, version)
        self.small = {}  # small-channel conv images (_small_image, no trainer / sampling)
        self.small_tr = {}  # small-channel conv images under a trainer: refreshed per update
        self._small_table = None
        self.mx8 = {}  # MX-fp8 conv weight images (mx8_weight_image)
        self._table = None
        self._table_key = None

    def lookup(self, weight, w, dtype, cout, cin, k, pad_to, mode):
        if (cin if mode % 2 == 0 else cout) * k * k > 8192:  # PACK_LDS of dv_conv.hip
            raise _lib.DVError(f"weight ({cout}, {cin}, {k}, {k}) too large for the packer")
        key = (weight.data_ptr(), tuple(weight.shape), dtype, pad_to, mode)
        e = self.entries.get(key)
        if e is not None and e["epoch"] == self.epoch and e["version"] == weight._version:
            return e["out"], False
        if e is None:
            import weakref
            rows = cout if mode % 2 == 0 else cin
            e = dict(out=torch.empty(rows, k * k, pad_to, dtype=dtype, device=weight.device),
                     w=w, meta=(cout, cin, k * k, pad_to, mode), param=weakref.ref(weight))
            self.entries[key] = e
            self._table_key = None
        e["epoch"], e["version"] = self.epoch, weight._version
        return e["out"], True

    def small_entry(self, weight, w, bias, cin, cout, k, mode=0, wcin=0):
        """The trainer-cache image of a small-channel conv (mode 0) or of its
        input gradient (mode 1, DvSmallPackEntry): packed now when new (an
        eager call: the trainer's warm-up precedes every capture), then only by
        refresh()."""
        import weakref
        key = (w.data_ptr(), tuple(w.shape), None if bias is None else bias.data_ptr(), cin, cout, k, mode)
        e = self.small_tr.get(key)
        if e is None:
            if torch.cuda.is_current_stream_capturing():
                raise _lib.DVError("small-conv image first built inside a captured region")
            n = ctypes.c_longlong(0)
            call("dv_conv_small_image_elems", cin, cout, k, ctypes.byref(n))
            img = torch.empty(n.value, dtype=torch.bfloat16, device=w.device)
            e = dict(img=img, w=w, bias=bias, meta=(cin, cout, k, mode, wcin), param=weakref.ref(weight))
            tab = _small_pack_table([e])
            call("dv_conv_small_pack_batched", ptr(tab[0]), tab[1], tab[2], stream())
            self.small_tr[key] = e
            self._small_table = None
        return e["img"]

    def _refresh_small(self):
        if not self.small_tr:
            return
        if self._small_table is None:
            self._small_table = _small_pack_table(list(self.small_tr.values()))
        tab, n, mx = self._small_table
        call("dv_conv_small_pack_batched", ptr(tab), n, mx, stream())

    def prune(self):
        """Drop the entries whose parameter is gone or now lives elsewhere
        (re-pointed into a new flat buffer, moved by `.to()`); the others —
        e.g. another trainer's weights, whose captured graphs read these
        images — stay.  An entry keeps its source storage alive, so a stale
        key can never alias a newer tensor."""
        dead = [k for k, e in self.entries.items()
                if e["param"]() is None or e["param"]().data_ptr() != k[0]]
        for k in dead:
            del self.entries[k]
        if dead:
            self._table = self._table_key = None
        gone = [k for k, e in self.mx8.items() if e[2]() is None or e[2]().data_ptr() != k[0]]
        for k in gone:
            del self.mx8[k]
        stale = [k for k, e in self.small_tr.items() if e["param"]() is None or e["param"]().data_ptr() != k[0]]
        for k in stale:
            del self.small_tr[k]
        if stale:
            self._small_table = None

    def refresh(self):
        """New epoch (weights were updated): repack all entries in one launch."""
        import ctypes
        self.epoch += 1
        self._refresh_small()
        if not self.entries:
            return
        ents = list(self.entries.values())
        dev = ents[0]["out"].device
        if self._table_key is None or self._table is None:
            pairs, rest = self._pair(ents)
            rows = []
            for e in rest:
                cout, cin, taps, pad_to, mode = e["meta"]
                dtc = _lib.DV_BF16 if e["out"].dtype == torch.bfloat16 else _lib.DV_F32
                rows.append((e["w"].data_ptr(), e["out"].data_ptr(), dtc, cout, cin, taps, pad_to, mode))
            raw = torch.tensor([[a, b, (c | (d << 32)), (f | (g << 32)), (h | (m << 32))]
                                for a, b, c, d, f, g, h, m in rows], dtype=torch.int64).reshape(-1, 5)
            self._table = raw.to(dev)
            self._table_key = True
            self._nrest = len(rest)
            self._max = max((e["out"].numel() for e in rest), default=0)
            # pairs: DvPackPair rows (w, out_fwd, out_dgrad, cout | cin << 32, taps | modes << 32, tile0)
            prow, tmap, t0 = [], [], 0
            for i, (ef, ed) in enumerate(pairs):
                cout, cin = ef["meta"][0], ef["meta"][1]
                n = (cout // 64) * (cin // 16)
                modes = ef["meta"][4] | (ed["meta"][4] << 8)
                prow.append([ef["w"].data_ptr(), ef["out"].data_ptr(), ed["out"].data_ptr(),
                             cout | (cin << 32), 9 | (modes << 32), t0])
                tmap.append(torch.full((n,), i, dtype=torch.int32))
                t0 += n
            self._pairs = torch.tensor(prow, dtype=torch.int64).reshape(-1, 6).to(dev)
            self._tmap = torch.cat(tmap).to(dev) if tmap else None
            self._ntiles = t0
        if self._nrest:
            call("dv_pack_conv_weights_batched", ptr(self._table), self._nrest, self._max, stream())
        if self._ntiles:
            call("dv_pack_conv_weight_pairs", ptr(self._pairs), ptr(self._tmap), self._ntiles, stream())
        for e in ents:
            e["epoch"] = self.epoch

    @staticmethod
    def _pair(ents):
        """(forward, dgrad) entry pairs of the bf16 3x3 weights that
        dv_pack_conv_weight_pairs packs from one read of the weight
        (cout % 64 == 0, cin % 16 == 0, unpadded rows, exactly one image of
        each kind), and the rest."""
        by_w = {}
        for e in ents:
            by_w.setdefault(e["w"].data_ptr(), []).append(e)
        pairs, rest = [], []
        for group in by_w.values():
            f = [e for e in group if e["meta"][4] in (0, 2)]
            d = [e for e in group if e["meta"][4] in (1, 3)]
            ok = len(f) == 1 and len(d) == 1 and len(group) == 2
            if ok:
                (cout, cin, taps, padf, _), padd = f[0]["meta"], d[0]["meta"][3]
                ok = (taps == 9 and cout % 64 == 0 and cin % 16 == 0 and padf == cin and padd == cout
                      and f[0]["out"].dtype == torch.bfloat16 and d[0]["out"].dtype == torch.bfloat16
                      and d[0]["meta"][:3] == (cout, cin, taps) and f[0]["w"].is_contiguous())
            if ok:
                pairs.append((f[0], d[0]))
            else:
                rest.extend(group)
        return pairs, rest

    def clear(self):
        self.entries.clear()
        self.mx8.clear()
        self.small_tr.clear()
        self._small_table = None
        self._table = self._table_key = None


PACK = PackCache()


def _small_pack_table(ents):
    """(device launch table, n, max elements) of dv_conv_small_pack_batched."""
    host = (_lib.DvSmallPackEntry * len(ents))(*[
        _lib.DvSmallPackEntry(e["w"].data_ptr(), None if e["bias"] is None else e["bias"].data_ptr(),
                              e["img"].data_ptr(), *e["meta"]) for e in ents])
    nbytes, mx = ctypes.c_longlong(0), ctypes.c_longlong(0)
    call("dv_conv_small_pack_plan", ctypes.byref(host), len(ents), None, ctypes.byref(nbytes), ctypes.byref(mx))
    buf = ctypes.create_string_buffer(nbytes.value)
    call("dv_conv_small_pack_plan", ctypes.byref(host), len(ents), buf, ctypes.byref(nbytes), ctypes.byref(mx))
    raw = torch.frombuffer(bytearray(buf.raw), dtype=torch.uint8)
    return raw.to(ents[0]["img"].device), len(ents), mx.value


class private_pack_cache:
    """Context: a separate, enabled PackCache for a region whose weights do not
    change (the sampling loop).  The trainer's cache is untouched, so sampling
    weights (e.g. the EMA unets) are never repacked by its per-update refresh."""

    def __enter__(self):
        global PACK
        self.saved = PACK
        PACK = PackCache()
        PACK.enabled = True
        PACK.static = True
        return PACK

    def __exit__(self, *exc):
        global PACK
        PACK = self.saved
        return False


def pack_conv_weight(weight: torch.Tensor, dtype, pad_to: int, mode: int, cache: bool = True) -> torch.Tensor:
    if weight.dim() not in (2, 5) or (weight.dim() == 5 and weight.shape[-1] != weight.shape[-2]):
        raise _lib.DVError(f"conv weight must be (cout, cin) or (cout, cin, 1, k, k), got {tuple(weight.shape)}")
    cout, cin = weight.shape[0], weight.shape[1]
    k = weight.shape[-1] if weight.dim() == 5 else 1  # nn.Linear weights are 1x1 convs
    w = weight.detach()
    if w.dtype != torch.float32 or not w.is_contiguous():
        w = w.float().contiguous()
    if cache and PACK.enabled and w.data_ptr() == weight.data_ptr():
        out, stale = PACK.lookup(weight, w, dtype, cout, cin, k, pad_to, mode)
        if not stale:
            return out
    else:
        rows = cout if mode % 2 == 0 else cin
        out = torch.empty(rows, k * k, pad_to, dtype=dtype, device=weight.device)
    call("dv_pack_conv_weight", _lib.DV_BF16 if dtype == torch.bfloat16 else _lib.DV_F32,
         ptr(w), ptr(out), cout, cin, k, pad_to, mode, stream())
    return out


class GradSink:
    """Shared input-gradient buffer of two convolutions reading the same input
    (ResnetBlock3D's block1 conv and res_conv, dalle2_video.py:170, 188-205):
    the first backward to run keeps its dX here and returns None for the
    input; the second adds its dgrad into that buffer in its epilogue (res =
    y = dX) and returns the total -- no autograd accumulation kernel."""

    def __init__(self):
        self.dx = None


class SkipGrad:
    """Gradient hand-off of a unet skip tensor: the hiddens the down path
    pushes and the up path pops as the second input of its channel concats
    (dalle2_video.py:926-936).  A hidden has one down-path reader (the
    consumer: the next block's conv, or the downsample) and one or two
    up-path readers.  The up-path convs run first in the backward (the
    consumer's output feeds them), so instead of returning their dX1 -- a
    strided channel slice of their [dX0 | dX1] buffer -- for autograd to add
    to the consumer's gradient, they park it here; the consumer adds what is
    parked in its own kernel (a dgrad epilogue residual, or the space-to-depth
    backward's residual inputs) and closes the hand-off.  A reader that comes
    after the close, or a hand-off whose consumer takes no input gradient (not
    armed), returns its gradient to autograd as usual: no order loses one."""

    def __init__(self):
        self.armed = False
        self.closed = False
        self.parked = []
        self.n_parked = 0  # gradients handed over (diagnostics / tests)

    def arm(self, needs_grad):
        """Consumer's forward (ctx.needs_input_grad of its input: grad mode is
        off inside a Function's forward): only a consumer computing dX takes."""
        if needs_grad:
            self.armed = True

    def park(self, g):
        if not self.armed or self.closed:
            return False
        self.parked.append(g)
        self.n_parked += 1
        return True

    def take(self):
        self.closed = True
        out, self.parked = self.parked, []
        return out


def _take_skips(skip, like):
    """The parked skip gradients a consumer adds (shape-checked)."""
    if skip is None:
        return []
    out = skip.take()
    for g in out:
        if tuple(g.shape) != tuple(like.shape):
            raise _lib.DVError(f"skip gradient {tuple(g.shape)} does not match {tuple(like.shape)}")
    return out


# ---------------------------------------------------------------------------
# MX-fp8 3x3 convs for sampling (BASELINE config 5; dv_mx8.hip)
# ---------------------------------------------------------------------------
class _Mx8State:
    active = 0     # > 0 inside mx8_convs()
    attention = 0  # > 0 inside mx8_convs(attention=True): the mid attention's PV too


class mx8_convs:
    """Context: eligible 3x3 convs run in MX-fp8 (e4m3 operands with a power-
    of-two scale per 32 channels, f32 accumulation, bf16 output) — forward
    only: ignored while autograd records (training stays bf16 / f32).
    Unet3D.forward_cl enters it when the unet's `fp8` flag is set.

    attention=True also runs the long-sequence mid attention's PV in MX-fp8
    (dv_mqa_fwd_fp8; the unet's `fp8_attention` flag).  Off by default: on
    MI355X it measured SLOWER than the bf16 bounded-score kernel at the
    config-5 shape (499 vs 353 us per call, bench `config5_fp8.mid_attention_fp8`)
    and its rounding error is ~4e-2 relative vs f32 against <1e-2 for bf16
    (tests/test_mqa_fp8_gpu.py); inside mx8_convs() the attention stays bf16."""

    def __init__(self, attention=False):
        self.attention = bool(attention)

    def __enter__(self):
        _Mx8State.active += 1
        _Mx8State.attention += int(self.attention)
        return self

    def __exit__(self, *exc):
        _Mx8State.active -= 1
        _Mx8State.attention -= int(self.attention)
        return False


# where the MX-fp8 conv runs: every eligible 3x3 conv (cin, cout % 64 == 0).
# Same-box config-5 forward (tools/cfg5_profile.py, graph replay, r03i): fp8
# at W <= 32 only 9.57 ms, at every width 9.00 ms with the GroupNorm-fused
# quantisation (9.56 without it: the separate quantisation pass of the wide
# 64² / 128² activations ate the conv gain), bf16 9.74-9.99 ms.
_MX8_MAX_W = 128
# the GroupNorm apply writes the fp8 copy of its output (dv_gn_fwd_mx8) so the
# consuming conv skips its quantisation pass (tests/test_mx8_gpu.py turns it off)
_MX8_FUSE = True


def _mx8_geom(nf, h, w):
    return ((h == 8 and w == 8) or (w in (16, 32, 64, 128) and h % (128 // w) == 0)) and (nf * h * w) % 128 == 0


def mx8_ok(x0, x1, weight, res, ksize, h, w, nf):
    """Mirror of dv_conv_fwd_mx8's contract (dv_hip.h), restricted to the
    frame widths where it measured faster (_MX8_MAX_W)."""
    if (not _Mx8State.active or torch.is_grad_enabled() or ksize != 3 or x0.dtype != torch.bfloat16
            or w > _MX8_MAX_W):
        return False
    c0 = x0.shape[3]
    c1 = 0 if x1 is None else x1.shape[3]
    cout, cin_real = weight.shape[0], weight.shape[1]
    if cin_real != c0 + c1 or c0 % 64 or c1 % 64 or cout % 64:
        return False
    if not _mx8_geom(nf, h, w):
        return False
    for t in (x0, x1, res):
        if t is not None:
            try:
                ld = cl_ld(t)
            except _lib.DVError:
                return False
            if ld % 8 or t.data_ptr() % 16:
                return False
    return True


def mx8_quant(x):
    """bf16 channels-last (NF, H, W, C) -> (q uint8 [M * C], s int32 [C/64 * M]):
    MX-fp8 e4m3 bytes and the per-32-channel scale pairs (dv_mx8_quant)."""
    nf, h, w, c = x.shape
    m = nf * h * w
    q = torch.empty(m * c, dtype=torch.uint8, device=x.device)
    sc = torch.empty((c // 64) * m, dtype=torch.int32, device=x.device)
    call("dv_mx8_quant", ptr(x), cl_ld(x), c, m, ptr(q), ptr(sc), stream())
    return q, sc


def mx8_weight_image(weight):
    """The conv kernel's MX-fp8 image of a (cout, cin, 1, 3, 3) f32 weight, kept
    in the current PackCache (trainer epoch + torch version checked; a sampling
    region's private cache is fresh per sample() call)."""
    w = weight.detach()
    if w.dtype != torch.float32 or not w.is_contiguous():
        w = w.float().contiguous()
    cache = PACK.mx8
    key = (weight.data_ptr(), tuple(weight.shape))
    ver = (PACK.epoch, weight._version)
    e = cache.get(key)
    if e is not None and e[0] == ver and e[2]() is weight:
        return e[1]
    import weakref
    cout, cin = weight.shape[0], weight.shape[1]
    n = ctypes.c_longlong(0)
    call("dv_mx8_image_bytes", cout, cin, ctypes.byref(n))
    img = torch.empty(n.value, dtype=torch.uint8, device=weight.device)
    call("dv_mx8_pack_conv_weight", ptr(w), cout, cin, ptr(img), stream())
    if PACK.enabled:
        cache[key] = (ver, img, weakref.ref(weight))
    return img


def conv_mx8(x0, weight, bias=None, x1=None, res=None):
    """y = conv3x3(cat(x0, x1)) + bias (+ res) in MX-fp8 (bf16 channels-last in / out)."""
    require_gpu(x0, x1, weight, bias, res)
    nf, h, w, c0 = x0.shape
    c1 = 0 if x1 is None else x1.shape[3]
    cout = weight.shape[0]
    # a GroupNorm output already carries its MX-fp8 copy (dv_gn_fwd_mx8)
    q0, s0 = getattr(x0, "_dv_mx8", None) or mx8_quant(x0)
    q1, s1 = (getattr(x1, "_dv_mx8", None) or mx8_quant(x1)) if x1 is not None else (None, None)
    img = mx8_weight_image(weight)
    y = torch.empty(nf, h, w, cout, dtype=torch.bfloat16, device=x0.device)
    b = None if bias is None else bias.detach().float().contiguous()
    m = nf * h * w
    _launch(f"conv_fwd_mx8_kernel<{w}>", 2.0 * m * cout * (c0 + c1) * 9, m * (c0 + c1 + 2 * cout),
            lambda: call("dv_conv_fwd_mx8", ptr(q0), ptr(s0), c0, ptr(q1), ptr(s1), c1, ptr(img), ptr(b),
                         ptr(res), cl_ld(res) if res is not None else 0, ptr(y), cout, nf, h, w, cout,
                         stream()), ("fwd", m, cout, 9 * (c0 + c1)))
    return y


class ConvFn(torch.autograd.Function):
    """y = conv_(1,k,k)(cat(x0, x1)) + bias (+ res).  dalle2_video.py:107 etc."""

    @staticmethod
    def forward(ctx, x0, x1, weight, bias, res, ksize, sink=None, cache=True, algo_scale=1.0,
                gn=None, skip_in=None, skip_out=None):
        require_gpu(x0, x1, weight, bias, res)
        nf, h, w, c0 = x0.shape
        c1 = 0 if x1 is None else x1.shape[3]
        cin = c0 + c1
        cout, cin_real = weight.shape[0], weight.shape[1]
        if cin_real > cin:
            raise _lib.DVError(f"conv: weight expects {cin_real} input channels, got {cin}")
        gi = getattr(x0, "_dv_gn_in", None)
        if gi is not None:  # x0 is a deferred GroupNorm output (group_norm_act(defer=True))
            x0._dv_gn_in = None
            if (x1 is None and res is None and ksize == 3 and cin_real == cin and cl_ld(x0) == c0
                    and gn_in_ok(nf, h, w, c0, gi["groups"], x0.dtype, gi["nb"], cout)):
                return ConvFn._forward_gn_in(ctx, gi, x0, weight, bias, sink, cache, algo_scale, gn,
                                             skip_in, skip_out)
            _gn_in_materialize(gi, x0)
        if mx8_ok(x0, x1, weight, res, ksize, h, w, nf):
            if gn is not None:
                gn.used = False  # the GroupNorm reduces z itself
            return conv_mx8(x0, weight, bias, x1=x1, res=res)
        y = torch.empty(nf, h, w, cout, dtype=x0.dtype, device=x0.device)
        ld0 = cl_ld(x0)
        ld1 = cl_ld(x1) if x1 is not None else 0
        ldr = cl_ld(res) if res is not None else 0
        b = None if bias is None else bias.detach().float().contiguous()
        m = nf * h * w
        # algorithmic work: algo_scale < 1 when the executed weight is padded
        # (CrossEmbedLayer3D's zero-embedded kernels, 3 -> 8 input channels)
        flops = 2.0 * m * cout * cin * ksize * ksize * algo_scale
        nbytes = x0.element_size() * m * (cin + cout)
        shape = ("fwd", m, cout, cin * ksize * ksize)
        # GroupNorm statistics epilogue (gn: a GnStats of the GroupNorm reading y)
        # where it measured cheaper than the GroupNorm's own reduce pass
        # (tools/gnstats_bench.py): the resident-weight stripe kernel (stage-0/1
        # Block3D convs) and the 8x8 window kernel; elsewhere gn.used = False
        # and the GroupNorm reduces z itself
        use_small = small_conv_ok(x0, x1, cin, cin_real, cout, ld0, ld1, ldr, ksize, w)
        use_win = not use_small and window_ok(x0, x1, cin, c0 if x1 is not None else cin, cout, ld0,
                                              ld1 or ld0, cout, ldr, ksize, h, w, nf,
                                              gn.P if gn is not None else 0)
        if gn is not None and use_small:
            gn.used = False
        elif gn is not None:
            name = (f"conv_fwd_frame_kernel<{w}>" if use_win else
                    conv_fwd_name(_lib.dtype_name(x0), m, cin, c0 if x1 is not None else cin, cout,
                                  max(ld0, ld1), ksize, h, w, gn.P))
            gn.used = GnStats.ALL or name in GN_STATS_KERNELS
        gs, gP, gR = (ptr(gn.cur), gn.P, gn.R) if gn is not None and gn.used else (None, 0, 0)
        if use_small:
            img = _small_image(weight, b, cin_real, cout, ksize, cache)
            _launch("xe_fwd_kernel", flops, nbytes,
                    lambda: call("dv_conv_small_fwd", ptr(x0), ld0, c0, ptr(x1), ld1, ptr(img), ptr(res),
                                 ldr, ptr(y), cout, nf, h, w, cin_real, cout, ksize, stream()), shape)
        elif use_win:
            wp = pack_conv_weight(weight, x0.dtype, cin, 2, cache)
            _launch(f"conv_fwd_frame_kernel<{w}>", flops, nbytes,
                    lambda: call("dv_conv_fwd8", dt(x0), ptr(x0), ld0, c0, ptr(x1), ld1, ptr(wp),
                                 ptr(b), ptr(res), ldr, None, 0, ptr(y), cout, nf, h, w, cin, cout,
                                 ACT_NONE, gs, gP, gR, stream()), shape)
        else:
            wp = pack_conv_weight(weight, x0.dtype, cin, 0, cache)
            _launch(conv_fwd_name(_lib.dtype_name(x0), m, cin, c0 if x1 is not None else cin, cout,
                                  max(ld0, ld1), ksize, h, w, gP), flops, nbytes,
                    lambda: call("dv_conv_fwd", dt(x0), ptr(x0), ld0, c0, ptr(x1), ld1, ptr(wp), ptr(b),
                                 ptr(res), ldr, None, 0, ptr(y), cout, nf, h, w, cin, cout, ksize,
                                 ACT_NONE, gs, gP, gR, stream()), shape)
        ConvFn._save(ctx, x0, x1, weight, bias, ksize, c0, c1, res is not None, sink, cache, algo_scale,
                     skip_in, skip_out)
        return y

    @staticmethod
    def _save(ctx, x0, x1, weight, bias, ksize, c0, c1, has_res, sink, cache, algo_scale, skip_in, skip_out):
        ctx.save_for_backward(x0, x1, weight)
        ctx.params = (weight, bias)
        ctx.meta = (ksize, c0, c1, bias is not None, has_res)
        ctx.sink = sink
        ctx.cache = cache
        ctx.algo_scale = algo_scale
        if skip_in is not None and x1 is None:
            skip_in.arm(ctx.needs_input_grad[0])
        ctx.skip_in, ctx.skip_out = skip_in, skip_out

    @staticmethod
    def _forward_gn_in(ctx, gi, x0, weight, bias, sink, cache, algo_scale, gn, skip_in, skip_out):
        """conv(silu(GroupNorm(z) (+FiLM))) with the GroupNorm applied while the
        stripe kernel stages z (dv_conv_fwd_gn_in): x0 is the deferred GroupNorm
        output, written by this launch only when the weight gradient will read it."""
        z, st = gi["z"], gi["stats"]
        nf, h, w, cin = x0.shape
        cout = weight.shape[0]
        m = nf * h * w
        y = torch.empty(nf, h, w, cout, dtype=x0.dtype, device=x0.device)
        b = None if bias is None else bias.detach().float().contiguous()
        wp = pack_conv_weight(weight, x0.dtype, cin, 0, cache)
        d = DvGnIn()
        d.sums, d.rstride, d.R = st.cur.data_ptr(), gi["nb"] * cin * 2, st.R
        d.P, d.groups, d.eps = gi["P"], gi["groups"], float(gi["eps"])
        d.gamma, d.beta = gi["g"].data_ptr(), gi["b"].data_ptr()
        d.ss = None if gi["s"] is None else gi["s"].data_ptr()
        d.mean, d.rstd = gi["mean"].data_ptr(), gi["rstd"].data_ptr()
        d.y = x0.data_ptr() if ctx.needs_input_grad[2] else None  # the wgrad reads it
        d.ldy = cin
        d.zero, d.zero_n = st.nxt.data_ptr(), st.nxt.numel()  # the deferred call's zeroing duty
        if gn is not None:
            gn.used = True
        gs, gP, gR = (ptr(gn.cur), gn.P, gn.R) if gn is not None else (None, 0, 0)
        _launch("conv_fwd_stripe_kernel<64,gn_in>", 2.0 * m * cout * cin * 9 * algo_scale,
                x0.element_size() * m * (cin * (2 if d.y else 1) + cout),
                lambda: call("dv_conv_fwd_gn_in", ctypes.byref(d), ptr(z), cl_ld(z), ptr(wp), ptr(b), ptr(y),
                             cout, nf, h, w, cin, cout, gs, gP, gR, stream()), ("fwd", m, cout, cin * 9))
        ConvFn._save(ctx, x0, None, weight, bias, 3, cin, 0, False, sink, cache, algo_scale, skip_in, skip_out)
        return y

    @staticmethod
    def backward(ctx, dy):
        x0, x1, weight = ctx.saved_tensors
        ksize, c0, c1, has_bias, has_res = ctx.meta
        nf, h, w, _ = x0.shape
        cin = c0 + c1
        cout, cin_real = weight.shape[0], weight.shape[1]
        dyv, lddy = _grad_view(dy)
        if dy.shape[3] % 8 == 0 and lddy % 8 == 0:
            dy8 = dyv  # strided channel slices are read in place (ld = lddy)
        else:
            dy8 = _pad_channels(dyv.contiguous())
            lddy = dy8.shape[3]
        cout8 = dy8.shape[3]
        dx0 = dx1 = dw = db = None
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            sink = ctx.sink
            acc = sink.dx if sink is not None else None  # second reader: add into the first's dX
            if acc is not None:
                dx = acc
                sink.dx = None
            else:
                alloc = torch.empty if cin_real == cin else torch.zeros
                dx = alloc(nf, h, w, cin, dtype=dy.dtype, device=dy.device)
            # the accumulated buffer may be a strided channel view (the dy a
            # GroupNorm handed over): read and write it through its pixel stride
            ldx = cl_ld(dx) if acc is not None else cin
            # epilogue residuals: the shared buffer (in place), then the unet
            # skip gradients parked for this input (SkipGrad); more than two
            # (none in Unet3D) are added after the launch
            resid = ([dx] if acc is not None else []) + (
                _take_skips(ctx.skip_in, dx) if ctx.needs_input_grad[0] and x1 is None else [])
            rp, rld = (ptr(resid[0]), cl_ld(resid[0])) if resid else (None, 0)
            rp2, rld2 = (ptr(resid[1]), cl_ld(resid[1])) if len(resid) > 1 else (None, 0)
            m = nf * h * w
            flops = 2.0 * m * cin_real * cout8 * ksize * ksize * ctx.algo_scale
            nbytes = dy8.element_size() * m * (cin + cout8)
            shape = ("dgrad", m, cin_real, cout8 * ksize * ksize)
            if (dy8.dtype == torch.bfloat16 and cout <= 16 and cin <= 32 and ksize % 2 == 1 and ksize <= 15
                    and w % 32 == 0 and rp2 is None and lddy % 8 == 0 and ldx % 4 == 0 and rld % 4 == 0
                    and weight.dim() == 5 and dy8.data_ptr() % 16 == 0):
                # small-channel dgrad (the cascade SR unet's dim-8 / 16 convs): a
                # conv of dY with the transposed, flipped weight on the direct
                # small-channel kernel (an implicit GEMM ran it 8 of 64 rows live)
                img = _small_dgrad_image(weight, cout, cin, cin_real, ksize, ctx.cache)
                _launch("xe_fwd_kernel", flops, nbytes,
                        lambda: call("dv_conv_small_fwd", ptr(dy8), lddy, cout, None, 0, ptr(img), rp, rld,
                                     ptr(dx), ldx, nf, h, w, cout, cin, ksize, stream()), shape)
            elif window_ok(dy8, None, cout8, cout8, cin_real, lddy, lddy, ldx, rld, ksize, h, w, nf,
                           ldres2=rld2):
                wpd = pack_conv_weight(weight, dy.dtype, cout8, 3, ctx.cache)
                _launch(f"conv_fwd_frame_kernel<{w}>", flops, nbytes,
                        lambda: call("dv_conv_fwd8", dt(dy8), ptr(dy8), lddy, cout8, None, 0, ptr(wpd),
                                     None, rp, rld, rp2, rld2, ptr(dx), ldx, nf, h, w, cout8, cin_real,
                                     ACT_NONE, None, 0, 0, stream()), shape)
            else:
                wpd = pack_conv_weight(weight, dy.dtype, cout8, 1, ctx.cache)
                _launch(conv_fwd_name(_lib.dtype_name(dy8), m, cout8, cout8, cin_real, lddy, ksize, h, w,
                                      nres2=rp2 is not None),
                        flops, nbytes,
                        lambda: call("dv_conv_fwd", dt(dy8), ptr(dy8), lddy, cout8, None, 0, ptr(wpd), None,
                                     rp, rld, rp2, rld2, ptr(dx), ldx, nf, h, w, cout8, cin_real, ksize,
                                     ACT_NONE, None, 0, 0, stream()), shape)
            for g in resid[2:]:
                dx.add_(g)
            if sink is not None and acc is None:
                sink.dx = dx  # first reader: the other conv's backward adds into it
            else:
                dx0 = dx[..., :c0]
                dx1 = dx[..., c0:] if x1 is not None else None
                if dx1 is not None and ctx.skip_out is not None and ctx.skip_out.park(dx1):
                    dx1 = None  # the skip's down-path reader adds it in its kernel
        wparam, bparam = ctx.params
        want_w = ctx.needs_input_grad[2]
        want_b = has_bias and ctx.needs_input_grad[3]
        if want_w:
            # weight (+ fused bias) gradient straight into the parameters' .grad
            # (the trainer's flat buffer) when they are leaves; else returned
            wslot = _grad_out(wparam, overwrite=True)
            bslot = _grad_out(bparam, overwrite=True) if want_b else None
            if wslot is not None:
                dw_t, acc_w = wslot
            else:
                dw = dw_t = torch.empty(weight.shape, dtype=torch.float32, device=dy.device)
                acc_w = False
            if want_b:
                if bslot is not None:
                    db_t, acc_b = bslot
                else:
                    db = db_t = torch.empty(cout, dtype=torch.float32, device=dy.device)
                    acc_b = False
            else:
                db_t, acc_b = None, False
            ld0 = cl_ld(x0)
            ld1 = cl_ld(x1) if x1 is not None else 0
            m = nf * h * w
            if (x1 is None and weight.dim() == 5 and cin_real <= 8 and lddy % 8 == 0
                    and cross_embed_ok(x0, [weight])):
                # a small-input-channel conv (the cascade SR unet's dim-8 convs at
                # 128^2 / 64^2): its weight gradient is the single-branch case of
                # the cross-embed kernel (row-band MFMA partials + one finishing
                # sum), not an implicit GEMM with 8 of 64 output rows live
                desc = _cross_embed_desc(cin_real, [weight.detach()], [None])
                desc.dw[0], desc.accumulate_w = dw_t.data_ptr(), int(acc_w)
                if want_b:
                    desc.db[0], desc.accumulate_b = db_t.data_ptr(), int(acc_b)
                WGRAD_DEFER.before_write(dw_t.data_ptr(), db_t.data_ptr() if db_t is not None else None)
                need = ctypes.c_longlong(0)
                call("dv_cross_embed_wgrad_ws", ctypes.byref(desc), nf, h, w, ctypes.byref(need))
                key = str(dy.device)
                xws = _XE_WS.get(key)
                if xws is None or xws.numel() < need.value:
                    xws = _XE_WS[key] = torch.empty(need.value, dtype=torch.float32, device=dy.device)
                _launch("cross_embed_wgrad_kernel", 2.0 * m * cout * cin_real * ksize * ksize,
                        dy8.element_size() * m * (cin + cout8),
                        lambda: call("dv_cross_embed_wgrad", ctypes.byref(desc), ptr(dy8), lddy, ptr(x0), ld0,
                                     ptr(xws), xws.numel(), nf, h, w, stream()),
                        ("wgrad", cout, cin_real * ksize * ksize, m))
                dres = dy if has_res else None
                return dx0, dx1, dw, db, dres, None, None, None, None, None, None, None
            dname = _lib.dtype_name(dy8)
            kname = (conv_wgrad_name(dname, m, cout8, cin, c0, x1 is not None, ksize, h, w,
                                     max(lddy, ld0, ld1)) if (cout8 == cout and cin_real == cin)
                     else gemm_wgrad_name(dname, m, cout8, cin * ksize * ksize, max(lddy, ld0, ld1)))
            if (WGRAD_DEFER.active and dw is None and db is None
                    and kname.startswith(("conv_wgrad_win", "conv_wgrad_1x1"))):
                # leaf .grad targets: leave the split partials for the pass-end sum
                if (not WGRAD_DEFER.STREAM
                        and WGRAD_DEFER.conflicts(dw_t.data_ptr(), db_t.data_ptr() if db_t is not None else None)):
                    WGRAD_DEFER.flush()  # a second gradient into the same target (streamed sums stay ordered)
                need = ctypes.c_longlong(0)
                call("dv_conv_wgrad_ws", dt(dy8), nf, h, w, cin, c0, int(x1 is not None), cout8, ksize,
                     ctypes.byref(need))
                arena, off = WGRAD_DEFER.slot(dy.device, need.value)
                ent = _lib.DvWgradReduceEntry()
                _launch(kname, 2.0 * m * cout8 * cin * ksize * ksize * ctx.algo_scale,
                        dy8.element_size() * m * (cin + cout8),
                        lambda: call("dv_conv_wgrad_deferred", dt(dy8), ptr(dy8), lddy, ptr(x0), ld0, c0,
                                     ptr(x1), ld1, ptr(dw_t), int(acc_w), ptr(db_t), int(acc_b),
                                     _lib.ctypes_vp(arena.data_ptr() + 4 * off), need.value, nf, h, w,
                                     cin, cout8, cout, cin_real, ksize, ctypes.byref(ent), stream()),
                        ("wgrad", cout8, cin * ksize * ksize, m))
                if ent.S > 0:
                    WGRAD_DEFER.add(ent, dy.device)
                dres = dy if has_res else None
                return dx0, dx1, dw, db, dres, None, None, None, None, None, None, None
            WGRAD_DEFER.before_write(dw_t.data_ptr(), db_t.data_ptr() if db_t is not None else None)
            ws = _wgrad_workspace(_lib.dtype_name(dy8), nf, h, w, cin, c0, x1 is not None, cout8,
                                  ksize, dy.device)
            # (on a side stream, concurrent with the dgrad -> GroupNorm chain,
            # the wgrads measured slower: 77 vs 80-82 steps/s in round 1, 96.5
            # vs 104.7 in round 5 with the deferred sums kept -- removed)
            _launch(kname,
                    2.0 * m * cout8 * cin * ksize * ksize * ctx.algo_scale,
                    dy8.element_size() * m * (cin + cout8),
                    lambda: call("dv_conv_wgrad", dt(dy8), ptr(dy8), lddy, ptr(x0), ld0, c0, ptr(x1), ld1,
                                 ptr(dw_t), int(acc_w), ptr(db_t), int(acc_b), ptr(ws), ws.numel(),
                                 nf, h, w, cin, cout8, cout, cin_real, ksize, stream()),
                    ("wgrad", cout8, cin * ksize * ksize, m))
        elif want_b:
            bslot = _grad_out(bparam, zero=True)
            if bslot is None or cout8 != cout:
                db_buf = torch.zeros(cout8, dtype=torch.float32, device=dy.device)
            else:
                db_buf = bslot[0]
            WGRAD_DEFER.before_write(bslot[0].data_ptr() if bslot is not None else None)
            call("dv_bias_grad", dt(dy8), ptr(dy8), lddy, ptr(db_buf), nf * h * w, cout, stream())
            if bslot is None:
                db = db_buf[:cout]
            elif db_buf is not bslot[0]:
                bslot[0].add_(db_buf[:cout])
        dres = dy if has_res else None
        return dx0, dx1, dw, db, dres, None, None, None, None, None, None, None


# small-channel forward (cin <= 16, cout <= 32: the cascade's 256x256 unet at
# dim 8) on the direct kernel of dv_xembed.hip


def small_conv_ok(x0, x1, cin, cin_real, cout, ld0, ld1, ldr, ksize, w):
    if x0.dtype != torch.bfloat16 or not x0.is_cuda:
        return False
    if not (cin_real <= 16 and cout <= 32 and cout % 8 == 0 and ksize % 2 == 1 and ksize <= 15
            and w % 32 == 0 and ldr % 4 == 0):
        return False
    if x1 is not None:
        c0 = x0.shape[3]
        return cin_real == cin and c0 % 8 == 0 and ld0 % 8 == 0 and ld1 % 8 == 0 and cin > 8
    return ld0 % (4 if cin_real <= 4 else 8) == 0


def _small_image(weight, bias, cin, cout, k, cache):
    """Packed image of a small-channel conv (weights + bias), kept in the
    current PackCache (torch version counters checked) while its weights
    cannot change behind torch's back: a sampling region's private cache, or
    no trainer at all.  Under a trainer's cache (AdamW writes the weights in
    place) the image is a PackCache entry too, repacked -- all of them in ONE
    launch -- by the cache's per-update refresh(): the forward (and a captured
    graph of it) then launches no pack kernel."""
    w = weight.detach()
    if w.dtype != torch.float32 or not w.is_contiguous():
        w = w.float().contiguous()
    if cache and PACK.enabled and not PACK.static and w.data_ptr() == weight.data_ptr():
        return PACK.small_entry(weight, w, bias, cin, cout, k)
    keep = cache and (PACK.static or not PACK.enabled) and w.data_ptr() == weight.data_ptr()
    key = (weight.data_ptr(), tuple(weight.shape), None if bias is None else bias.data_ptr())
    ver = (weight._version, None if bias is None else bias._version)
    cache_d = PACK.small
    if keep:
        e = cache_d.get(key)
        if e is not None and e[0] == ver and e[2] is weight:
            return e[1]
    n = ctypes.c_longlong(0)
    call("dv_conv_small_image_elems", cin, cout, k, ctypes.byref(n))
    img = torch.empty(n.value, dtype=torch.bfloat16, device=weight.device)
    call("dv_conv_small_pack", ptr(w), ptr(bias), cin, cout, k, ptr(img), stream())
    if keep:
        cache_d[key] = (ver, img, weight)
    return img


def _small_dgrad_image(weight, cout, cin_pad, cin_real, k, cache):
    """Image of the input-gradient conv of a small-channel conv: input channels
    = its cout, outputs = its (padded) cin, taps flipped.  Under a trainer's
    cache a PackCache entry (DvSmallPackEntry mode 1, repacked per update);
    else built here from the transposed weight."""
    w = weight.detach()
    if w.dtype != torch.float32 or not w.is_contiguous():
        w = w.float().contiguous()
    if cache and PACK.enabled and not PACK.static and w.data_ptr() == weight.data_ptr():
        return PACK.small_entry(weight, w, None, cout, cin_pad, k, mode=1, wcin=cin_real)
    wt = torch.zeros(cin_pad, cout, 1, k, k, dtype=torch.float32, device=w.device)
    wt[:cin_real] = w.flip(-1, -2).transpose(0, 1)
    return _small_image(wt, None, cout, cin_pad, k, False)


def conv(x0, weight, bias=None, x1=None, res=None, sink=None, cache=True, algo_scale=1.0, gn=None,
         skip_in=None, skip_out=None):
    """(1,k,k) 'same' convolution over channels-last frames (weight in torch
    Conv3d layout (cout, cin, 1, k, k) or Linear layout (cout, cin)).
    sink: a GradSink shared with the other conv reading (x0, x1).
    cache=False: the weight is rebuilt every call (not a parameter), so its
    packed image is made on every call instead of kept in the PackCache.
    algo_scale: algorithmic / executed FLOPs (timing labels only).
    gn: a GnStats (gn_stats()) — the kernel's epilogue accumulates the
    GroupNorm statistics of y for the group_norm_act(stats=gn) that follows.
    skip_in: the SkipGrad of x0 when this conv is its down-path reader (the
    dgrad adds the parked skip gradients); skip_out: the SkipGrad of x1 when
    x1 is a unet skip (the dgrad parks dX1 there)."""
    k = weight.shape[-1] if weight.dim() == 5 else 1
    return ConvFn.apply(x0, x1, weight, bias, res, k, sink, cache, algo_scale, gn, skip_in, skip_out)


# ---------------------------------------------------------------------------
# CrossEmbedLayer3D (dalle2_video.py:208-244): direct multi-window conv
# ---------------------------------------------------------------------------
class DvCrossEmbed(ctypes.Structure):
    """Mirror of DvCrossEmbed (include/dv_hip.h)."""
    _fields_ = [("nbranch", ctypes.c_int), ("cin", ctypes.c_int), ("k", ctypes.c_int * 4),
                ("cout", ctypes.c_int * 4), ("w", ctypes.c_void_p * 4), ("b", ctypes.c_void_p * 4),
                ("dw", ctypes.c_void_p * 4), ("db", ctypes.c_void_p * 4),
                ("accumulate_w", ctypes.c_int), ("accumulate_b", ctypes.c_int)]


def _cross_embed_desc(cin, weights, biases):
    d = DvCrossEmbed()
    d.nbranch, d.cin = len(weights), cin
    for i, (w, b) in enumerate(zip(weights, biases)):
        d.k[i], d.cout[i] = w.shape[-1], w.shape[0]
        d.w[i] = w.data_ptr()
        d.b[i] = None if b is None else b.data_ptr()
    return d


def cross_embed_ok(x, weights):
    """Shapes the direct kernels take (else the padded implicit-GEMM conv runs)."""
    if x.dtype != torch.bfloat16 or not x.is_cuda or x.dim() != 4 or not 1 <= len(weights) <= 4:
        return False
    nf, h, w, _ = x.shape
    cin = weights[0].shape[1]
    ks = [wt.shape[-1] for wt in weights]
    try:
        ld = cl_ld(x)
    except _lib.DVError:
        return False
    cout = sum(wt.shape[0] for wt in weights)
    kmax, cp, cpad = max(ks), 4 if cin <= 4 else 8, (cout + 15) // 16 * 16
    # the weight-gradient kernel's staging slots and LDS (dv_xembed.hip)
    wgrad_fits = (kmax * (w + kmax + 7) <= 9 * 512 and w * (cout // 8) <= 4 * 512
                  and 4 * w * (cpad + 8) + 4 * kmax * (w + kmax + 7) * cp <= 160 * 1024)
    return (cin <= 8 and all(wt.shape[1] == cin and wt.dim() == 5 and wt.dtype == torch.float32 for wt in weights)
            and ks == sorted(ks) and all(k % 2 == 1 and k <= 15 for k in ks)
            and cout % 8 == 0 and cout <= 128 and w % 32 == 0 and wgrad_fits
            and ld % (4 if cin <= 4 else 8) == 0 and x.data_ptr() % 16 == 0)


_XE_WS = {}


class CrossEmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, nbranch, *params):
        # the descriptor carries raw weight addresses: a host weight would be
        # read by the pack kernel (memory fault), so check before any launch
        require_gpu(x, *[p for p in params if p is not None])
        weights = [p.detach().float().contiguous() for p in params[:nbranch]]
        biases = [None if p is None else p.detach().float().contiguous() for p in params[nbranch:]]
        nf, h, w, _ = x.shape
        cin = weights[0].shape[1]
        desc = _cross_embed_desc(cin, weights, biases)
        n = ctypes.c_longlong(0)
        call("dv_cross_embed_image_elems", ctypes.byref(desc), ctypes.byref(n))
        img = torch.empty(n.value, dtype=torch.bfloat16, device=x.device)
        call("dv_cross_embed_pack", ctypes.byref(desc), ptr(img), stream())
        cout = sum(wt.shape[0] for wt in weights)
        y = torch.empty(nf, h, w, cout, dtype=x.dtype, device=x.device)
        m = nf * h * w
        flops = 2.0 * m * cin * sum(wt.shape[0] * wt.shape[-1] ** 2 for wt in weights)
        _launch("cross_embed_fwd_kernel", flops, x.element_size() * m * (cin + cout),
                lambda: call("dv_cross_embed_fwd", ctypes.byref(desc), ptr(img), ptr(x), cl_ld(x), ptr(y),
                             cout, nf, h, w, stream()), ("fwd", m, cout, cin * max(wt.shape[-1] for wt in weights) ** 2))
        ctx.save_for_backward(x)
        ctx.nbranch = nbranch
        ctx.params = params
        ctx.flops = flops
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        nb = ctx.nbranch
        wparams, bparams = ctx.params[:nb], ctx.params[nb:]
        dyv, lddy = _grad_view(dy)
        if lddy % 8:
            dyv, lddy = dyv.contiguous(), dyv.shape[-1]
        nf, h, w, _ = x.shape
        cin = wparams[0].shape[1]
        weights = [p.detach() for p in wparams]
        desc = _cross_embed_desc(cin, weights, [None if b is None else b.detach() for b in bparams])
        ret_w, ret_b = [None] * nb, [None] * nb
        # gradients straight into the leaves' .grad (zero-filled when new, so
        # every branch accumulates); otherwise returned
        for i in range(nb):
            slot = _grad_out(wparams[i], zero=True) if ctx.needs_input_grad[2 + i] else None
            if slot is None:
                ret_w[i] = torch.zeros_like(weights[i], dtype=torch.float32)
                desc.dw[i] = ret_w[i].data_ptr()
            else:
                desc.dw[i] = slot[0].data_ptr()
            b = bparams[i]
            if b is not None and ctx.needs_input_grad[2 + nb + i]:
                bslot = _grad_out(b, zero=True)
                if bslot is None:
                    ret_b[i] = torch.zeros(b.shape, dtype=torch.float32, device=dy.device)
                    desc.db[i] = ret_b[i].data_ptr()
                else:
                    desc.db[i] = bslot[0].data_ptr()
        desc.accumulate_w = desc.accumulate_b = 1
        need = ctypes.c_longlong(0)
        call("dv_cross_embed_wgrad_ws", ctypes.byref(desc), nf, h, w, ctypes.byref(need))
        key = str(dy.device)
        ws = _XE_WS.get(key)
        if ws is None or ws.numel() < need.value:
            ws = _XE_WS[key] = torch.empty(need.value, dtype=torch.float32, device=dy.device)
        m = nf * h * w
        _launch("cross_embed_wgrad_kernel", ctx.flops, dy.element_size() * m * (cin + dy.shape[-1]),
                lambda: call("dv_cross_embed_wgrad", ctypes.byref(desc), ptr(dyv), lddy, ptr(x), cl_ld(x), ptr(ws),
                             ws.numel(), nf, h, w, stream()), ("wgrad", dy.shape[-1], cin, m))
        return (None, None, *ret_w, *ret_b)


def cross_embed(x, weights, biases):
    """Concatenated (1,k,k) 'same' convolutions of one channels-last input
    (CrossEmbedLayer3D, stride 1): weights / biases per branch, kernel sizes
    ascending.  x's channels beyond weights[i].shape[1] are ignored."""
    return CrossEmbedFn.apply(x, len(weights), *weights, *biases)


# ---------------------------------------------------------------------------
# GroupNorm (+ per-sample scale/shift) + SiLU (+ residual)  — Block3D
# ---------------------------------------------------------------------------
def _gn_forward(z, gamma, beta, ss, res, nb, groups, eps, act, stats, mx8=False):
    """dv_gn_fwd; mx8: y also as the MX-fp8 operand of its 3x3 consumer
    (dv_gn_fwd_mx8), attached to y as `_dv_mx8` for conv_mx8."""
    require_gpu(z, gamma, beta, ss, res)
    nf, h, w, c = z.shape
    P = (nf // nb) * h * w
    dev = z.device
    y = torch.empty(nf, h, w, c, dtype=z.dtype, device=dev)
    mean = torch.empty(nb * groups, dtype=torch.float32, device=dev)
    rstd = torch.empty_like(mean)
    if stats is not None and stats.used:  # z's producing conv accumulated the statistics
        if stats.P != P:
            raise _lib.DVError("GroupNorm statistics were accumulated for another clip size")
        cur, nxt, ready = stats.cur, stats.nxt, stats.R
    elif stats is not None:  # the conv did not: reduce into the same (zeroed) buffer
        cur, nxt, ready = stats.cur, stats.nxt, 0
    else:
        (cur, nxt), ready = _gn_sums(dev).take(nb * c * 2), 0
    g, b = gamma.detach().float().contiguous(), beta.detach().float().contiguous()
    s = None if ss is None else ss.detach().float().contiguous()
    args = (ptr(z), cl_ld(z), ptr(y), c, ptr(res), cl_ld(res) if res is not None else 0,
            nb, P, c, groups, ctypes_float(eps), ptr(g), ptr(b), ptr(s), act, ptr(mean), ptr(rstd),
            ptr(cur), ptr(nxt), nxt.numel(), ready)
    if mx8:
        m = nf * h * w
        q = torch.empty(m * c, dtype=torch.uint8, device=dev)
        qs = torch.empty((c // 64) * m, dtype=torch.int32, device=dev)
        call("dv_gn_fwd_mx8", *args, ptr(q), ptr(qs), stream())
        y._dv_mx8 = (q, qs)
    else:
        call("dv_gn_fwd", dt(z), *args, stream())
    return y, g, b, s, mean, rstd


class DvGnIn(ctypes.Structure):
    """Mirror of DvGnIn (include/dv_hip.h): a GroupNorm folded into the conv reading it."""
    _fields_ = [("sums", ctypes.c_void_p), ("rstride", ctypes.c_longlong), ("R", ctypes.c_int),
                ("P", ctypes.c_longlong), ("groups", ctypes.c_int), ("eps", ctypes.c_float),
                ("gamma", ctypes.c_void_p), ("beta", ctypes.c_void_p), ("ss", ctypes.c_void_p),
                ("mean", ctypes.c_void_p), ("rstd", ctypes.c_void_p), ("y", ctypes.c_void_p),
                ("ldy", ctypes.c_int), ("zero", ctypes.c_void_p), ("zero_n", ctypes.c_longlong)]


# the conv kernels whose GroupNorm-statistics epilogue measured cheaper than
# the GroupNorm's own reduce pass (tools/gnstats_bench.py; W = 128: config 5)
GN_STATS_KERNELS = ("conv_fwd_stripe_kernel<64>", "conv_fwd_stripe_kernel<32>", "conv_fwd_stripe_kernel<128>",
                    "conv_fwd_frame_kernel<8>")

# Block3D -> Block3D GroupNorm folded into the second conv's input staging
# (tests switch it off to compare against the two-pass form)
GN_FOLD = True


def gn_in_ok(nf, h, w, c, groups, dtype, nb, cout):
    """The GroupNorm (+FiLM) + SiLU output a 3x3 conv can fold into its input
    staging (dv_conv_fwd_gn_in): bf16, 64 channels in 8 groups, 64-pixel rows,
    whole 128-pixel stages per clip (mirror of the C-ABI's shape check)."""
    m = nf * h * w
    return (dtype == torch.bfloat16 and c == 64 and groups == 8 and w == 64 and h % 2 == 0
            and m % 128 == 0 and ((nf // nb) * h * w) % 128 == 0 and cout % 64 == 0
            and m * c * 2 < (1 << 31) and not _Mx8State.active)


def _gn_in_materialize(gi, y):
    """The deferred GroupNorm apply, run on its own (the conv reading y did not
    take the folded form): one dv_gn_fwd apply over the producing conv's sums."""
    z, st = gi["z"], gi["stats"]
    nf, h, w, c = z.shape
    call("dv_gn_fwd", dt(z), ptr(z), cl_ld(z), ptr(y), c, None, 0, gi["nb"], gi["P"], c, gi["groups"],
         ctypes_float(gi["eps"]), ptr(gi["g"]), ptr(gi["b"]), ptr(gi["s"]), gi["act"], ptr(gi["mean"]),
         ptr(gi["rstd"]), ptr(st.cur), ptr(st.nxt), st.nxt.numel(), st.R, stream())


class GroupNormActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, gamma, beta, ss, res, nb, groups, eps, act, stats=None, res_sink=None, defer=None):
        if defer is not None:
            # y is produced by the 3x3 conv that reads it (ConvFn, dv_conv_fwd_gn_in),
            # which also fills mean / rstd; `defer` is attached to y by group_norm_act
            nf, h, w, c = z.shape
            y = torch.empty(nf, h, w, c, dtype=z.dtype, device=z.device)
            mean = torch.empty(nb * groups, dtype=torch.float32, device=z.device)
            rstd = torch.empty_like(mean)
            g, b = gamma.detach().float().contiguous(), beta.detach().float().contiguous()
            s = None if ss is None else ss.detach().float().contiguous()
            defer.update(z=z, stats=stats, g=g, b=b, s=s, mean=mean, rstd=rstd, nb=nb, groups=groups,
                         eps=eps, act=act, P=(nf // nb) * h * w)
        else:
            y, g, b, s, mean, rstd = _gn_forward(z, gamma, beta, ss, res, nb, groups, eps, act, stats)
        ctx.save_for_backward(z, g, b, s, mean, rstd)
        ctx.params = (gamma, beta)
        ctx.meta = (nb, groups, act, ss is not None, res is not None)
        ctx.res_sink = res_sink
        return y

    @staticmethod
    def backward(ctx, dy):
        z, g, b, s, mean, rstd = ctx.saved_tensors
        nb, groups, act, has_ss, has_res = ctx.meta
        nf, h, w, c = z.shape
        P = (nf // nb) * h * w
        dev = z.device
        dy, lddy = _grad_view(dy)
        dz = torch.empty(nf, h, w, c, dtype=z.dtype, device=dev)
        gs, bs = _grad_out(ctx.params[0]), _grad_out(ctx.params[1])
        # one accumulate flag for both: allocate fresh buffers where they differ
        if gs is not None and bs is not None and gs[1] == bs[1]:
            dg, db, acc, ret = gs[0], bs[0], int(gs[1]), False
        else:
            dg = torch.empty(c, dtype=torch.float32, device=dev)
            db = torch.empty(c, dtype=torch.float32, device=dev)
            acc, ret = 0, True
        dss = torch.empty(nb, 2 * c, dtype=torch.float32, device=dev) if has_ss else None
        cur, nxt = _gn_sums(dev).take(nb * c * 2)
        call("dv_gn_bwd", dt(z), ptr(dy), lddy, ptr(z), cl_ld(z), ptr(dz), c, nb, P, c, groups, ptr(g),
             ptr(b), ptr(s), act, ptr(mean), ptr(rstd), ptr(dg), ptr(db), ptr(dss), ptr(cur), ptr(nxt), nxt.numel(),
             acc, stream())
        if not ret:
            dg = db = None
        dres = dy if has_res else None
        if dres is not None and ctx.res_sink is not None and ctx.needs_input_grad[4]:
            # identity residual (ResnetBlock3D, dalle2_video.py:205): the
            # residual's gradient is dy itself; block1's conv, the other
            # reader of the same input, adds its dgrad into it in the kernel
            # epilogue (GradSink) instead of autograd adding two tensors
            ctx.res_sink.dx = dy
            dres = None
        return dz, dg, db, dss, dres, None, None, None, None, None, None, None


def ctypes_float(v):
    import ctypes
    return ctypes.c_float(float(v))


def group_norm_act(z, gamma, beta, nb, groups=8, eps=1e-5, scale_shift=None, res=None,
                   act=_lib.ACT_SILU, stats=None, res_sink=None, defer=False):
    """stats: the GnStats z's conv filled (one apply launch) or None (reduce + apply).
    res_sink: a GradSink shared with the conv that also reads `res` (the
    residual's gradient is handed to it instead of returned to autograd).
    Inside mx8_convs() without autograd, an output an MX-fp8 conv can read
    (bf16, C % 64 == 0, a frame width it runs at) also gets its fp8 copy from
    the same launch: the conv then skips its quantisation pass.
    defer=True: the caller guarantees the output is read first by ops.conv (as
    its x0); when the shape allows, no apply runs and that conv produces the
    output while it stages z (dv_conv_fwd_gn_in), else the conv runs the apply
    before itself.  Any other first reader would see an unwritten tensor."""
    if _MX8_FUSE and _Mx8State.active and not torch.is_grad_enabled() and z.dtype == torch.bfloat16:
        nf, h, w, c = z.shape
        if c % 64 == 0 and w <= _MX8_MAX_W and _mx8_geom(nf, h, w):
            return _gn_forward(z, gamma, beta, scale_shift, res, nb, groups, eps, act, stats, mx8=True)[0]
    if (defer and res is None and act == _lib.ACT_SILU and stats is not None and stats.used
            and gn_in_ok(*z.shape, groups, z.dtype, nb, 64)):
        # the apply folds into the next 3x3 conv's input staging (Block3D ->
        # Block3D, dalle2_video.py:107-133 then :107): y is written by that conv
        info = {}
        y = GroupNormActFn.apply(z, gamma, beta, scale_shift, res, nb, groups, eps, act, stats, res_sink, info)
        y._dv_gn_in = info
        return y
    return GroupNormActFn.apply(z, gamma, beta, scale_shift, res, nb, groups, eps, act, stats, res_sink)


# ---------------------------------------------------------------------------
# row LayerNorm (dalle2 gain-only LayerNorm, nn.LayerNorm) (+ residual)
# ---------------------------------------------------------------------------
class LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g, b, res, eps):
        require_gpu(x, g, b, res)
        c = x.shape[-1]
        xc = x.contiguous()
        rows = xc.numel() // c
        y = torch.empty_like(xc)
        rc = res.contiguous() if res is not None else None
        gf = g.detach().float().contiguous()
        bf = None if b is None else b.detach().float().contiguous()
        call("dv_ln_fwd", dt(xc), ptr(xc), c, ptr(y), c, ptr(rc), c, rows, c, ptr(gf), ptr(bf),
             ctypes_float(eps), None, None, stream())
        ctx.save_for_backward(xc, gf)
        ctx.params = (g, b)
        ctx.meta = (eps, b is not None, res is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, gf = ctx.saved_tensors
        eps, has_b, has_res = ctx.meta
        c = xc.shape[-1]
        rows = xc.numel() // c
        dy = dy.contiguous()
        dx = torch.empty_like(xc)
        # dg/db are accumulated with atomics: in place into .grad (zeroed if fresh)
        gs = _grad_out(ctx.params[0], zero=True)
        bs = _grad_out(ctx.params[1], zero=True) if has_b else None
        dg = gs[0] if gs else torch.zeros(c, dtype=torch.float32, device=xc.device)
        db = (bs[0] if bs else torch.zeros(c, dtype=torch.float32, device=xc.device)) if has_b else None
        import ctypes
        need = ctypes.c_longlong(0)
        call("dv_ln_bwd_ws", rows, c, ctypes.byref(need))
        ws = _ln_workspace(need.value, xc.device)
        call("dv_ln_bwd", dt(xc), ptr(dy), c, ptr(xc), c, ptr(dx), c, rows, c, ptr(gf),
             ctypes_float(eps), ptr(dg), ptr(db), ptr(ws), ws.numel(), stream())
        return dx, (None if gs else dg), (None if bs else db), (dy if has_res else None), None


_LN_WS = {}


def _ln_workspace(n, device):
    """Per-device f32 scratch for dv_ln_bwd's per-block column partials (grown
    on demand; kernels on the stream use it one after another)."""
    key = str(device)
    if key not in _LN_WS or _LN_WS[key].numel() < n:
        # sized for every LayerNorm of the path at once (C <= 1,024: 8 MB), so
        # it is never re-allocated between the eager warm-up and graph capture
        _LN_WS[key] = torch.empty(max(n, 1 << 21), dtype=torch.float32, device=device)
    return _LN_WS[key]


def layer_norm(x, g, b=None, res=None, eps=1e-5):
    return LayerNormFn.apply(x, g, b, res, eps)


# ---------------------------------------------------------------------------
# small dense linears over (B, K) f32 rows (time MLPs, to_kv of the context)
# ---------------------------------------------------------------------------
ACT_OUT_GELU = 2


class LinearSmallFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act_in, act_out):
        require_gpu(x, w, b)
        xc = x.detach().float().contiguous()
        B, K = xc.shape
        N = w.shape[0]
        wc = w.detach().float().contiguous()
        bc = None if b is None else b.detach().float().contiguous()
        y = torch.empty(B, N, dtype=torch.float32, device=x.device)
        z = torch.empty(B, N, dtype=torch.float32, device=x.device) if act_out == ACT_OUT_GELU else None
        call("dv_linear_small_fwd", ptr(xc), K, ptr(wc), ptr(bc), ptr(y), N, ptr(z), B, K, N,
             act_in, act_out, stream())
        ctx.save_for_backward(xc, wc, z)
        ctx.params = (w, b)
        ctx.meta = (act_in, act_out, b is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, wc, z = ctx.saved_tensors
        act_in, act_out, has_b = ctx.meta
        B, K = xc.shape
        N = wc.shape[0]
        dev = dy.device
        dy = dy.float().contiguous()
        dx = torch.empty(B, K, dtype=torch.float32, device=dev) if ctx.needs_input_grad[0] else None
        ws = _grad_out(ctx.params[0]) if ctx.needs_input_grad[1] else None
        bs = _grad_out(ctx.params[1]) if has_b and ctx.needs_input_grad[2] else None
        if ws is not None and (not has_b or (bs is not None and bs[1] == ws[1])):
            dw, db, acc, ret = ws[0], (bs[0] if bs else None), int(ws[1]), False
        else:
            dw = torch.empty(N, K, dtype=torch.float32, device=dev)
            db = torch.empty(N, dtype=torch.float32, device=dev) if has_b else None
            acc, ret = 0, True
        call("dv_linear_small_bwd", ptr(dy), N, ptr(xc), K, ptr(wc), ptr(z), ptr(dx), K,
             ptr(dw), ptr(db), B, K, N, act_in, act_out, 0, acc, stream())
        if not ret:
            dw = db = None
        return dx, dw, db, None, None


def linear_small(x, w, b=None, act_in=0, act_out=0):
    return LinearSmallFn.apply(x, w, b, act_in, act_out)


class _LinEntry(ctypes.Structure):
    """ctypes mirror of DvLinEntry (include/dv_hip.h)."""
    _fields_ = [("w", ctypes.c_void_p), ("bias", ctypes.c_void_p), ("y", ctypes.c_void_p),
                ("dw", ctypes.c_void_p), ("db", ctypes.c_void_p), ("n", ctypes.c_int),
                ("accumulate_w", ctypes.c_int)]


_LG_WS = {}


class LinearGroupFn(torch.autograd.Function):
    """Many small nn.Linear layers over the same rows x (B, K), one launch each
    way: y_e = act_in(x) W_e^T + b_e.  The time MLPs of every ResnetBlock3D
    (dalle2_video.py:143-146, 182-185) share t; the CrossAttention to_kv
    projections share the context c (or mid_c)."""

    @staticmethod
    def forward(ctx, x, act_in, n_lin, *params):
        require_gpu(x, *[q for q in params if q is not None])
        xc = x.detach().float().contiguous()
        B, K = xc.shape
        ws, bs = params[:n_lin], params[n_lin:]
        ns = [w.shape[0] for w in ws]
        y = torch.empty(B * sum(ns), dtype=torch.float32, device=x.device)
        outs, off = [], 0
        for n in ns:
            outs.append(y[off:off + B * n].view(B, n))
            off += B * n
        wcs = [w.detach().float().contiguous() for w in ws]
        bcs = [None if b is None else b.detach().float().contiguous() for b in bs]
        ents = (_LinEntry * n_lin)(*[_LinEntry(w.data_ptr(), 0 if b is None else b.data_ptr(),
                                               o.data_ptr(), 0, 0, w.shape[0], 0)
                                     for w, b, o in zip(wcs, bcs, outs)])
        call("dv_linear_group_fwd", ptr(xc), B, K, act_in, ctypes.cast(ents, ctypes.c_void_p), n_lin,
             stream())
        ctx.save_for_backward(xc, *wcs)
        ctx.params = params
        ctx.meta = (act_in, n_lin)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *dys):
        flush_fold_bwd()  # deferred cross-attention fold grads fill these dys
        xc, *wcs = ctx.saved_tensors
        act_in, n_lin = ctx.meta
        ws, bs = ctx.params[:n_lin], ctx.params[n_lin:]
        B, K = xc.shape
        dev = xc.device
        key = (B * K, str(dev))
        if key not in _LG_WS:
            _LG_WS[key] = torch.zeros(B * K + 1, dtype=torch.float32, device=dev)
        wsbuf = _LG_WS[key]
        dx = torch.empty(B, K, dtype=torch.float32, device=dev) if ctx.needs_input_grad[0] else None
        ents, ret_w, ret_b, keep = [], [], [], []
        for i, (w, b, wc, dy) in enumerate(zip(ws, bs, wcs, dys)):
            dy = (torch.zeros(B, wc.shape[0], dtype=torch.float32, device=dev) if dy is None
                  else dy.float().contiguous())
            keep.append(dy)
            want_w = ctx.needs_input_grad[3 + i]
            want_b = b is not None and ctx.needs_input_grad[3 + n_lin + i]
            sw = _grad_out(w) if want_w else None
            sb = _grad_out(b) if want_b else None
            acc = 0
            if sw is not None and (not want_b or (sb is not None and sb[1] == sw[1])):
                dw, db, acc = sw[0], (sb[0] if sb else None), int(sw[1])
                ret_w.append(None)
                ret_b.append(None)
            else:
                dw = torch.empty_like(wc) if want_w else None
                db = torch.empty(wc.shape[0], dtype=torch.float32, device=dev) if want_b else None
                ret_w.append(dw)
                ret_b.append(db)
            ents.append(_LinEntry(wc.data_ptr(), 0, dy.data_ptr(), 0 if dw is None else dw.data_ptr(),
                                  0 if db is None else db.data_ptr(), wc.shape[0], acc))
        arr = (_LinEntry * n_lin)(*ents)
        call("dv_linear_group_bwd", ptr(xc), B, K, act_in, ctypes.cast(arr, ctypes.c_void_p), n_lin,
             ptr(dx), 0, ptr(wsbuf), stream())
        return (dx, None, None, *ret_w, *ret_b)


def linear_group(x, weights, biases, act_in=0):
    """[act_in(x) @ W_e^T + b_e for each e] in one launch (x: (B, K) f32)."""
    if len(weights) == 0:
        return []
    return list(LinearGroupFn.apply(x, act_in, len(weights), *weights, *biases))


_FREQS = {}


def sinusoid_freqs(dim: int, device) -> torch.Tensor:
    """Constant frequency table of SinusoidalPosEmb, built once exactly as the
    reference builds it (f32 arange times -ln(1e4)/(half-1), exp)."""
    key = (dim, str(device))
    if key not in _FREQS:
        import math
        half = dim // 2
        f = torch.exp(torch.arange(half, dtype=torch.float32) * -(math.log(10000) / (half - 1)))
        _FREQS[key] = f.to(device)
    return _FREQS[key]


def sinusoidal(times: torch.Tensor, dim: int) -> torch.Tensor:
    require_gpu(times)
    t = times.to(torch.int64).contiguous()
    out = torch.empty(t.shape[0], dim, dtype=torch.float32, device=t.device)
    call("dv_sinusoidal", ptr(t), ptr(sinusoid_freqs(dim, t.device)), ptr(out), t.shape[0], dim,
         stream())
    return out


# ---------------------------------------------------------------------------
# cross attention (folded), ResnetBlock3D.cross_attn
# ---------------------------------------------------------------------------
XA_HEADS, XA_DH = 8, 64


class DvFoldBwdJob(ctypes.Structure):
    """struct DvFoldBwdJob of dv_hip.h (dv_xattn_fold_bwd_batched)."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("wsR", "wsV", "wsQ", "mcorr", "at", "vt", "g1", "wq",
                                               "wo", "kv", "null_kv", "dat", "dvt", "dg1", "dg2",
                                               "dwq", "dwo", "dkv", "dnull")] + \
               [("nb", ctypes.c_int), ("C", ctypes.c_int), ("acc_g", ctypes.c_int),
                ("acc_w", ctypes.c_int)]


# fold backwards deferred by CrossAttnFn.backward (blocks whose fold the Unet
# batched, so kv comes from a grouped to_kv): (job, tensors kept alive)
_FOLD_BWD_PENDING = []


def flush_fold_bwd():
    """Run every deferred fold backward in four launches (called by the grouped
    to_kv backward, which consumes their kv gradients, before anything else)."""
    global _FOLD_BWD_PENDING
    pend, _FOLD_BWD_PENDING = _FOLD_BWD_PENDING, []
    for i in range(0, len(pend), 20):  # DV_FOLD_BWD_MAX
        part = pend[i:i + 20]
        jobs = (DvFoldBwdJob * len(part))(*[j for j, _ in part])
        call("dv_xattn_fold_bwd_batched", ctypes.cast(jobs, ctypes.c_void_p), len(part),
             ctypes_float(XA_DH ** -0.5), stream())


class DvFoldJob(ctypes.Structure):
    """struct DvFoldJob of dv_hip.h (dv_xattn_fold_batched)."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("wq", "wo", "kv", "null_kv", "g1", "at", "vt", "Kt",
                                               "KtT", "Vt", "VtT", "colsum")] + \
               [("nb", ctypes.c_int), ("C", ctypes.c_int)]


class XattnFold:
    """Folded cross-attention operands of one block (dv_xattn_fold outputs) and
    the f32 copies of the inputs they were made from (saved for the backward)."""

    def __init__(self, dtype, kv_in, g1, null_kv, wq, wo, nb, C):
        dev = kv_in.device
        self.kv = kv_in.detach().float().contiguous()  # (nb * tokens, 2 * 512): to_kv(context)
        self.wqf, self.wof = wq.detach().float().contiguous(), wo.detach().float().contiguous()
        self.nkv = null_kv.detach().float().contiguous()
        self.g1f = g1.detach().float().contiguous()
        self.at = torch.empty(nb, C, 24, dtype=torch.float32, device=dev)
        self.vt = torch.empty_like(self.at)
        Cp = (C + 31) // 32 * 32  # operand images padded to whole 32-channel MFMA tiles
        self.Kt = torch.empty(nb, 32, Cp, dtype=dtype, device=dev)
        self.KtT = torch.empty(nb, Cp, 32, dtype=dtype, device=dev)
        self.Vt = torch.empty(nb, Cp, 32, dtype=dtype, device=dev)
        self.VtT = torch.empty(nb, 32, Cp, dtype=dtype, device=dev)
        self.colsum = torch.empty(nb, 32, dtype=torch.float32, device=dev)
        self.nb, self.C, self.dtype = nb, C, dtype
        self.batched = False  # set by xattn_fold_batched: backward may be deferred

    def job(self):
        return DvFoldJob(*(ptr(t).value for t in (self.wqf, self.wof, self.kv, self.nkv, self.g1f,
                                                   self.at, self.vt, self.Kt, self.KtT, self.Vt,
                                                   self.VtT, self.colsum)), self.nb, self.C)

    def run(self):
        call("dv_xattn_fold", _lib.DV_BF16 if self.dtype == torch.bfloat16 else _lib.DV_F32,
             ptr(self.wqf), ptr(self.wof), ptr(self.kv), ptr(self.nkv), ptr(self.g1f), ptr(self.at),
             ptr(self.vt), ptr(self.Kt), ptr(self.KtT), ptr(self.Vt), ptr(self.VtT), ptr(self.colsum),
             self.nb, self.C, ctypes_float(XA_DH ** -0.5), stream())


def xattn_fold_batched(folds):
    """Run every block's fold in three launches (dv_xattn_fold_batched)."""
    folds = list(folds)
    for f in folds:
        f.batched = True
    for i in range(0, len(folds), 24):  # DV_FOLD_MAX
        part = folds[i:i + 24]
        jobs = (DvFoldJob * len(part))(*[f.job() for f in part])
        call("dv_xattn_fold_batched",
             _lib.DV_BF16 if part[0].dtype == torch.bfloat16 else _lib.DV_F32,
             ctypes.cast(jobs, ctypes.c_void_p), len(part), ctypes_float(XA_DH ** -0.5), stream())


class CrossAttnFn(torch.autograd.Function):
    """out = CrossAttention(x, context) + x, folded per batch element (dv_xattn.hip).
    `fold`: an XattnFold already run for this block (Unet3D batches all blocks'
    folds in one launch), or None to fold here."""

    @staticmethod
    def forward(ctx, x, kv_in, g1, null_kv, wq, wo, g2, nb, eps, fold=None):
        require_gpu(x, kv_in)
        nf, h, w, C = x.shape
        ntok = nf * h * w
        P = ntok // nb
        dev, dtype = x.device, x.dtype
        if fold is None:
            fold = XattnFold(dtype, kv_in, g1, null_kv, wq, wo, nb, C)
            fold.run()
        kv, wqf, wof, nkv, g1f = fold.kv, fold.wqf, fold.wof, fold.nkv, fold.g1f
        at, vt, Kt, KtT, Vt, VtT, colsum = (fold.at, fold.vt, fold.Kt, fold.KtT, fold.Vt, fold.VtT,
                                            fold.colsum)
        g2f = g2.detach().float().contiguous()
        out = torch.empty(nf, h, w, C, dtype=dtype, device=dev)
        stats = torch.empty(ntok, 4, dtype=torch.float32, device=dev)
        pbuf = torch.empty(ntok, 32, dtype=dtype, device=dev)
        call("dv_xattn_fwd", dt(x), ptr(x), cl_ld(x), ptr(out), C, ntok, P, C, ptr(Kt), ptr(Vt),
             ptr(colsum), ptr(g2f), ctypes_float(eps), ptr(stats), ptr(pbuf), stream())
        ctx.save_for_backward(x, g1f, g2f, nkv, wqf, wof, kv, at, vt, KtT, Vt, VtT,
                              colsum, stats, pbuf)
        ctx.params = (g1, null_kv, wq, wo, g2)
        ctx.meta = (nb, eps, fold.batched)
        return out

    @staticmethod
    def backward(ctx, dy):
        (x, g1f, g2f, nkv, wqf, wof, kv, at, vt, KtT, Vt, VtT, colsum, stats,
         pbuf) = ctx.saved_tensors
        g1p, nullp, wqp, wop, g2p = ctx.params
        nb, eps, defer = ctx.meta
        nf, h, w, C = x.shape
        ntok = nf * h * w
        P = ntok // nb
        dev, dtype = x.device, x.dtype
        dy, lddy = _grad_view(dy)
        dx = torch.empty(nf, h, w, C, dtype=dtype, device=dev)
        dobuf = torch.empty(ntok, C, dtype=dtype, device=dev)
        dsbuf = torch.empty(ntok, 32, dtype=dtype, device=dev)
        p2buf = torch.empty(ntok, 32, dtype=dtype, device=dev)
        wsR, wsV, wsQ, mcorr = _xattn_workspace(nb, C, dev, owner=wqp if defer else None)
        ldx = cl_ld(x)
        call("dv_xattn_bwd_tokens", dt(x), ptr(dy), lddy, ptr(x), ldx, ptr(dx), C, ntok, P, C,
             ptr(KtT), ptr(Vt), ptr(VtT), ptr(colsum), ptr(g2f), ptr(stats), ptr(pbuf), ptr(dobuf),
             ptr(dsbuf), ptr(p2buf), stream())
        # per-batch token reductions: R = dS'^T X, V' = P^T dO, Q = P'^T dY (three batched
        # GEMMs of one shape, one launch)
        probs = ((dsbuf, x, ldx, wsR), (pbuf, dobuf, C, wsV), (p2buf, dy, lddy, wsQ))
        pa = (ctypes.c_void_p * 3)(*(a_.data_ptr() for a_, _, _, _ in probs))
        la = (ctypes.c_int * 3)(32, 32, 32)
        pb = (ctypes.c_void_p * 3)(*(b_.data_ptr() for _, b_, _, _ in probs))
        lb = (ctypes.c_int * 3)(*(ldb for _, _, ldb, _ in probs))
        po = (ctypes.c_void_p * 3)(*(o_.data_ptr() for _, _, _, o_ in probs))
        _launch(gemm_wgrad_name(_lib.dtype_name(x), ntok, 32, C, max(32, ldx, C, lddy)),
                3 * 2.0 * ntok * 32 * C, 0,
                lambda: call("dv_gemm_tn_batched_multi", dt(x), 3, pa, la, pb, lb, po, P, nb, 32, C,
                             stream()))
        dat = torch.empty(nb, C, 24, dtype=torch.float32, device=dev)
        dvt = torch.empty_like(dat)
        s1, s2 = _grad_out(g1p), _grad_out(g2p)
        if s1 is not None and s2 is not None and s1[1] == s2[1]:
            dg1, dg2, acc_g, ret_g = s1[0], s2[0], int(s1[1]), False
        else:
            dg1, dg2 = torch.empty(C, dtype=torch.float32, device=dev), torch.empty(C, dtype=torch.float32, device=dev)
            acc_g, ret_g = 0, True
        sq, so, sn = _grad_out(wqp), _grad_out(wop), _grad_out(nullp)
        direct = sq is not None and so is not None and sn is not None and sq[1] == so[1] == sn[1]
        if direct:
            dwq, dwo, dnull, acc_w = sq[0], so[0], sn[0], int(sq[1])
        else:
            dwq, dwo, dnull, acc_w = torch.empty_like(wqf), torch.empty_like(wof), torch.empty_like(nkv), 0
        dkv = torch.empty_like(kv)
        if defer:  # filled by flush_fold_bwd() before the grouped to_kv backward reads dkv
            job = DvFoldBwdJob(*(ptr(t).value if t is not None else None
                                 for t in (wsR, wsV, wsQ, mcorr, at, vt, g1f, wqf, wof, kv, nkv, dat,
                                           dvt, dg1, dg2, dwq, dwo, dkv, dnull)),
                               nb, C, acc_g, acc_w)
            _FOLD_BWD_PENDING.append((job, (wsR, wsV, wsQ, mcorr, at, vt, g1f, wqf, wof, kv, nkv, dat,
                                            dvt, dg1, dg2, dwq, dwo, dkv, dnull)))
        else:
            call("dv_xattn_fold_bwd", ptr(wsR), ptr(wsV), ptr(wsQ), ptr(mcorr), ptr(at), ptr(vt),
                 ptr(g1f), ptr(wqf), ptr(wof), ptr(kv), ptr(nkv), ptr(dat), ptr(dvt), ptr(dg1),
                 ptr(dg2), ptr(dwq), ptr(dwo), ptr(dkv), ptr(dnull), nb, C, ctypes_float(XA_DH ** -0.5),
                 acc_g, acc_w, stream())
        return (dx, dkv, dg1 if ret_g else None, None if direct else dnull,
                None if direct else dwq, None if direct else dwo,
                dg2 if ret_g else None, None, None, None)


def ctypes_vp(addr):
    import ctypes
    return ctypes.c_void_p(addr)


def cross_attention(x, context, g1, null_kv, wq, wkv, wo, g2, nb, eps, kv=None, fold=None):
    """kv: to_kv(context) rows when the caller batched the projection
    (linear_group over every block sharing the context); else computed here.
    fold: this block's XattnFold when the caller batched the folds."""
    if kv is None:
        kv = linear_group(context.float().reshape(-1, context.shape[-1]), [wkv], [None])[0]
    return CrossAttnFn.apply(x, kv, g1, null_kv, wq, wo, g2, nb, eps, fold)


# ---------------------------------------------------------------------------
# multi-query flash attention core (mid_attn)
# ---------------------------------------------------------------------------
MQA_DH = 32


# the bf16 backward kernels hold a whole clip's K / V in LDS (dv_mqa_bwd)
MQA_BF16_BWD_MAX_NKP = 1280


def mqa_fp8_ok(q, NKP, H, ldq, needs_grad):
    """MX-fp8 PV (dv_mqa_fwd_fp8): inside mx8_convs(attention=True) (the unet's
    fp8_attention flag, BASELINE config 5), forward only, bf16 dense rows, and a clip whose K / V
    stream through LDS (NKP > 1280: the config-5 8,193 keys)."""
    return (_Mx8State.attention > 0 and not needs_grad and q.dtype == torch.bfloat16 and ldq == H * MQA_DH
            and NKP > MQA_BF16_BWD_MAX_NKP)


class MQAFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, kv, null_kv, B, N, H, scale, grad_mode=True):
        require_gpu(q, kv, null_kv)
        dev = q.device
        NKP = (N + 1 + 31) // 32 * 32
        # needs_input_grad follows requires_grad even under no_grad (null_kv is
        # a Parameter): `grad_mode` is the caller's torch.is_grad_enabled(), so
        # sampling never takes the training-only paths below
        needs_grad = grad_mode and any(ctx.needs_input_grad[:3])
        # a bf16 sequence too long for the bf16 backward (config 5: 8,193 keys)
        # that needs gradients runs forward AND backward on the f32 kernels (one
        # lse layout for both); outputs and input gradients stay bf16
        ctx.cast = q.dtype == torch.bfloat16 and NKP > MQA_BF16_BWD_MAX_NKP and needs_grad
        if ctx.cast:
            q, kv = q.float(), kv.float()
        qc, kvc = q.contiguous(), kv.contiguous()
        kp = torch.empty(B, NKP, MQA_DH, dtype=q.dtype, device=dev)
        vp = torch.empty_like(kp)
        nkv = null_kv.detach().float().contiguous()
        # bf16: per-64-key-block key norms, the forward's score bound (no running max when it holds)
        kmax = (torch.empty(B * ((NKP + 63) // 64), dtype=torch.float32, device=dev)
                if q.dtype == torch.bfloat16 else None)
        call("dv_mqa_prep", dt(q), ptr(kvc), kvc.shape[-1], ptr(nkv), ptr(kp), ptr(vp), B, N, NKP,
             ctypes_float(scale), ptr(kmax), stream())
        o = torch.empty(B * N, H * MQA_DH, dtype=q.dtype, device=dev)
        lse = torch.empty(B, H, N, dtype=torch.float32, device=dev)
        if mqa_fp8_ok(q, NKP, H, qc.shape[-1], needs_grad):
            # sampling inside mx8_convs() on a K/V-streamed clip: PV in MX-fp8
            # (dv_mqa_fwd_fp8; forward only -- no autograd records this call)
            need = ctypes.c_longlong(0)
            call("dv_mqa_fwd_fp8_ws", B, NKP, ctypes.byref(need))
            v8 = torch.empty(need.value, dtype=torch.uint8, device=dev)
            _launch("attn:mqa_fwd8", 4.0 * B * H * N * (N + 1) * MQA_DH, 0,
                    lambda: call("dv_mqa_fwd_fp8", ptr(qc), qc.shape[-1], ptr(kp), ptr(vp), ptr(v8), need.value,
                                 ptr(o), o.shape[-1], ptr(lse), B, N, NKP, H, stream()))
            ctx.meta = None
            return o
        _launch("attn:mqa_fwd", 4.0 * B * H * N * (N + 1) * MQA_DH, 0,
                lambda: call("dv_mqa_fwd", dt(q), ptr(qc), qc.shape[-1], ptr(kp), ptr(vp), ptr(o),
                             o.shape[-1], ptr(lse), B, N, NKP, H, ctypes_float(scale), ptr(kmax), stream()))
        ctx.save_for_backward(qc, kp, vp, o, lse)
        ctx.params = (null_kv,)
        ctx.meta = (B, N, H, NKP, scale, kvc.shape[-1])
        return o.to(torch.bfloat16) if ctx.cast else o

    @staticmethod
    def backward(ctx, do):
        qc, kp, vp, o, lse = ctx.saved_tensors
        B, N, H, NKP, scale, ldkv = ctx.meta
        dev = qc.device
        do = do.to(qc.dtype).contiguous()
        dq = torch.empty_like(qc)
        D = torch.empty(B, H, N, dtype=torch.float32, device=dev)
        need = ctypes.c_longlong(0)
        call("dv_mqa_bwd_ws", dt(qc), qc.shape[-1], o.shape[-1], B, N, NKP, H, ctypes.byref(need))
        ws = torch.empty(need.value, dtype=torch.float32, device=dev)
        dkv = torch.empty(B * N, 2 * MQA_DH, dtype=qc.dtype, device=dev)
        sn = _grad_out(ctx.params[0])
        dnull = sn[0] if sn else torch.empty(2, MQA_DH, dtype=torch.float32, device=dev)
        # algorithmic backward = 2x the forward contractions (dS/dQ/dK/dV, no recompute)
        _launch("attn:mqa_bwd", 8.0 * B * H * N * (N + 1) * MQA_DH, 0,
                lambda: call("dv_mqa_bwd", dt(qc), ptr(qc), qc.shape[-1], ptr(o), o.shape[-1], ptr(do),
                             do.shape[-1], ptr(lse), ptr(kp), ptr(vp), ptr(dq), dq.shape[-1], ptr(D),
                             ptr(ws), need.value, ptr(dkv), dkv.shape[-1], ptr(dnull), B, N, NKP, H,
                             ctypes_float(scale), int(sn[1]) if sn else 0, stream()))
        if ctx.cast:
            dq, dkv = dq.to(torch.bfloat16), dkv.to(torch.bfloat16)
        return dq, dkv, (None if sn else dnull), None, None, None, None, None


def mqa(q, kv, null_kv, B, N, H, scale):
    return MQAFn.apply(q, kv, null_kv, B, N, H, scale, torch.is_grad_enabled())


# ---------------------------------------------------------------------------
# space-to-depth (Downsample3D) and SiLU+PixelShuffle (PixelShuffleUpsample3D)
# ---------------------------------------------------------------------------
class SpaceToDepthFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, skip_in=None):
        require_gpu(x)
        nf, H2, W2, C = x.shape
        H, W = H2 // 2, W2 // 2
        y = torch.empty(nf, H, W, 4 * C, dtype=x.dtype, device=x.device)
        call("dv_shuffle", dt(x), 0, ptr(x), cl_ld(x), ptr(y), 4 * C, None, 0, None, 0, None, 0,
             nf, H, W, C, 0, stream())
        if skip_in is not None:
            skip_in.arm(ctx.needs_input_grad[0])
        ctx.skip_in = skip_in
        return y

    @staticmethod
    def backward(ctx, dy):
        dy, ldd = _grad_view(dy)
        nf, H, W, C4 = dy.shape
        C = C4 // 4
        dx = torch.empty(nf, 2 * H, 2 * W, C, dtype=dy.dtype, device=dy.device)
        # the skip gradients of x (the level's last hidden, read twice by the
        # up path) are added by the depth-to-space pass itself
        sk = _take_skips(ctx.skip_in, dx)
        r0, l0 = (ptr(sk[0]), cl_ld(sk[0])) if sk else (None, 0)
        r1, l1 = (ptr(sk[1]), cl_ld(sk[1])) if len(sk) > 1 else (None, 0)
        call("dv_shuffle", dt(dy), 1, ptr(dy), ldd, ptr(dx), C, None, 0, r0, l0, r1, l1, nf, H, W, C, 0,
             stream())
        for g in sk[2:]:
            dx.add_(g)
        return dx, None


class SiLUPixelShuffleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z):
        require_gpu(z)
        nf, H, W, C4 = z.shape
        C = C4 // 4
        y = torch.empty(nf, 2 * H, 2 * W, C, dtype=z.dtype, device=z.device)
        call("dv_shuffle", dt(z), 1, ptr(z), cl_ld(z), ptr(y), C, None, 0, None, 0, None, 0, nf, H, W, C,
             _lib.ACT_SILU, stream())
        ctx.save_for_backward(z)
        return y

    @staticmethod
    def backward(ctx, dy):
        (z,) = ctx.saved_tensors
        dy, ldd = _grad_view(dy)
        nf, H, W, C4 = z.shape
        C = C4 // 4
        dz = torch.empty(nf, H, W, C4, dtype=z.dtype, device=z.device)
        call("dv_shuffle", dt(z), 0, ptr(dy), ldd, ptr(dz), C4, ptr(z), cl_ld(z), None, 0, None, 0,
             nf, H, W, C, 0, stream())
        return dz


def space_to_depth(x, skip_in=None):
    return SpaceToDepthFn.apply(x, skip_in)


def silu_pixel_shuffle(z):
    return SiLUPixelShuffleFn.apply(z)


# ---------------------------------------------------------------------------
# NCTHW (module boundary) <-> channels-last frames
# ---------------------------------------------------------------------------
def _pad8(c):
    return (c + 7) // 8 * 8


class ToCLFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dtype):
        require_gpu(x)
        xf = x.detach().float().contiguous()
        B, C, T, H, W = xf.shape
        cp = _pad8(C)
        y = torch.empty(B * T, H, W, cp, dtype=dtype, device=x.device)
        call("dv_ncthw_to_cl", _lib.DV_BF16 if dtype == torch.bfloat16 else _lib.DV_F32, ptr(xf), ptr(y),
             B, C, T, H, W, cp, stream())
        ctx.meta = (B, C, T, H, W, x.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        B, C, T, H, W, xdt = ctx.meta
        dy = dy.contiguous()
        dx = torch.empty(B, C, T, H, W, dtype=torch.float32, device=dy.device)
        call("dv_cl_to_ncthw", dt(dy), ptr(dy), dy.shape[-1], ptr(dx), B, C, T, H, W, stream())
        return dx.to(xdt), None


class FromCLFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, B, C, T):
        require_gpu(y)
        nf, H, W, _ = y.shape
        x = torch.empty(B, C, T, H, W, dtype=torch.float32, device=y.device)
        call("dv_cl_to_ncthw", dt(y), ptr(y), cl_ld(y), ptr(x), B, C, T, H, W, stream())
        ctx.meta = (B, C, T, H, W, y.dtype, y.shape[-1])
        return x

    @staticmethod
    def backward(ctx, dx):
        B, C, T, H, W, ydt, cy = ctx.meta
        dxf = dx.float().contiguous()
        dy = torch.zeros(B * T, H, W, cy, dtype=ydt, device=dx.device) if cy != _pad8(C) else None
        if dy is None:
            dy = torch.empty(B * T, H, W, cy, dtype=ydt, device=dx.device)
        call("dv_ncthw_to_cl", dt(dy), ptr(dxf), ptr(dy), B, C, T, H, W, cy, stream())
        return dy, None, None, None


def to_cl(x, dtype):
    return ToCLFn.apply(x, dtype)


def from_cl(y, B, C, T):
    return FromCLFn.apply(y, B, C, T)


# ---------------------------------------------------------------------------
# diffusion arithmetic (q_sample, l2 loss, posterior step)
# ---------------------------------------------------------------------------
def q_sample_cl(x_start, noise, times, sqrt_ac, sqrt_1m_ac, dtype, normalize=True):
    require_gpu(x_start, noise, times)
    x0 = x_start.float().contiguous()
    nz = noise.float().contiguous()
    t = times.to(torch.int64).contiguous()
    B, C, T, H, W = x0.shape
    cp = _pad8(C)
    y = torch.empty(B * T, H, W, cp, dtype=dtype, device=x0.device)
    call("dv_q_sample", _lib.DV_BF16 if dtype == torch.bfloat16 else _lib.DV_F32, ptr(x0), ptr(nz), ptr(t),
         ptr(sqrt_ac), ptr(sqrt_1m_ac), ptr(y), B, C, T, H, W, cp, int(normalize), sqrt_ac.numel(),
         stream())
    return y


class MSELossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred_cl, target, sample_w):
        require_gpu(pred_cl, target)
        tgt = target.float().contiguous()
        B, C, T, H, W = tgt.shape
        loss = torch.empty((), dtype=torch.float32, device=tgt.device)
        sw = None if sample_w is None else sample_w.float().contiguous()
        call("dv_mse_loss", dt(pred_cl), ptr(pred_cl), cl_ld(pred_cl), ptr(tgt), B, C, T, H, W, ptr(sw),
             ptr(loss), stream())
        ctx.save_for_backward(pred_cl, tgt, sw)
        return loss

    @staticmethod
    def backward(ctx, dl):
        pred_cl, tgt, sw = ctx.saved_tensors
        B, C, T, H, W = tgt.shape
        dlc = dl.float().contiguous().reshape(1)
        cp = pred_cl.shape[-1]
        alloc = torch.zeros if cp != C else torch.empty
        dp = alloc(pred_cl.shape, dtype=pred_cl.dtype, device=pred_cl.device)
        call("dv_mse_loss_bwd", dt(pred_cl), ptr(pred_cl), cl_ld(pred_cl), ptr(tgt), B, C, T, H, W, ptr(sw),
             ptr(dlc), ptr(dp), cp, stream())
        return dp, None, None


def mse_loss_cl(pred_cl, target, sample_w=None):
    return MSELossFn.apply(pred_cl, target, sample_w)


def p_sample_step(x, eps, noise, times, sched, clip_denoised=True, out=None, want_x0=True):
    """x0 = sqrt(1/ac) x - sqrt(1/ac - 1) eps -> clamp -> posterior mean + sigma z
    (p_mean_variance + p_sample, dalle2_video.py:1551-1664).  eps is an NCTHW
    f32 tensor or a channels-last frame tensor.  `out` may be x itself (the
    update is elementwise: the sampling loop advances its state in place)."""
    require_gpu(x, eps, noise, times)
    xf = x.float().contiguous()
    nz = noise.float().contiguous()
    t = times.to(torch.int64).contiguous()
    B, C, T, H, W = xf.shape
    if eps.dim() == 5:
        ef = eps.float().contiguous()
        ld, edt = 0, _lib.DV_F32
    else:
        ef = eps
        ld, edt = cl_ld(eps), dt(eps)
        if eps.shape[0] != B * T or eps.shape[-1] < C:
            raise _lib.DVError(f"p_sample: eps {tuple(eps.shape)} does not match x {tuple(xf.shape)}")
    if out is None:
        out = torch.empty_like(xf)
    elif out.dtype != torch.float32 or not out.is_contiguous() or out.shape != xf.shape:
        raise _lib.DVError("p_sample: out must be a contiguous f32 tensor shaped like x")
    x0 = torch.empty_like(xf) if want_x0 else None
    call("dv_p_sample", edt, ptr(xf), ptr(ef), ld, ptr(nz), ptr(t), ptr(sched.sqrt_recip_alphas_cumprod),
         ptr(sched.sqrt_recipm1_alphas_cumprod), ptr(sched.posterior_mean_coef1),
         ptr(sched.posterior_mean_coef2), ptr(sched.posterior_log_variance_clipped), ptr(out), ptr(x0),
         B, C, T, H, W, int(clip_denoised), sched.sqrt_recip_alphas_cumprod.numel(), stream())
    return out, x0


def resize_nearest(video, size, clamp_range=None):
    """Per-frame nearest resize of an NCTHW clip to size x size."""
    require_gpu(video)
    v = video.float().contiguous()
    B, C, T, H, W = v.shape
    y = torch.empty(B, C, T, size, size, dtype=torch.float32, device=v.device)
    lo, hi = clamp_range if clamp_range is not None else (0.0, 0.0)
    call("dv_resize_nearest", ptr(v), ptr(y), B * C * T, H, W, size, size, int(clamp_range is not None),
         ctypes_float(lo), ctypes_float(hi), stream())
    return y


def gaussian_kernel1d(ks, sigma):
    x = torch.arange(ks, dtype=torch.float32) - ks // 2
    if ks % 2 == 0:
        x = x + 0.5
    g = torch.exp(-x.pow(2.0) / (2 * sigma ** 2))
    return g / g.sum()


_BLUR_TAPS = {}


def gaussian_blur(video, ks, sigma):
    """kornia gaussian_blur2d((ks,ks), (sigma,sigma)) per frame, reflect border."""
    require_gpu(video)
    v = video.float().contiguous()
    B, C, T, H, W = v.shape
    # device taps cached per (ks, sigma, device): no host-to-device copy once
    # warm, so a captured training call (the trainer's unet2 graphs) holds none
    key = (int(ks), float(sigma), str(v.device))
    w1 = _BLUR_TAPS.get(key)
    if w1 is None:
        if torch.cuda.is_current_stream_capturing():
            raise _lib.DVError("gaussian_blur taps first built inside a captured region")
        w1 = _BLUR_TAPS[key] = gaussian_kernel1d(ks, sigma).to(v.device)
    y = torch.empty_like(v)
    call("dv_gaussian_blur", ptr(v), ptr(y), B * C * T, H, W, ks, ptr(w1), stream())
    return y
