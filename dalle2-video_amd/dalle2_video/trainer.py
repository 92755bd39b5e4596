"""VideoDecoderTrainer — drop-in for dalle2_video/trainer.py (trainer.py:9-365)
on the MI355X path.

* Same constructor / `__call__(video_embed=, video=, unet_number=)` / `update()`
  / `save` / `load` surface, `optim{i}` / `sched{i}` attributes with torch
  param_groups, `steps` buffer, `train_loader` / `val_loader`.
* Optimizer: dalle2-pytorch `get_optimizer` semantics (AdamW betas (0.9, 0.99),
  weight decay only on ndim >= 2 parameters) executed as ONE fused HIP kernel
  over a flat f32 parameter/gradient/moment buffer per unet (`FusedAdamW`,
  state-dict compatible with torch.optim.AdamW).
* Gradient clipping (`clip_grad_norm_(decoder.parameters(), 0.5)`,
  trainer.py:254-257) is a HIP reduction whose coefficient is applied inside
  the AdamW kernel: no host synchronisation.
* Data parallel: one process per GPU (torchrun); the loaders are sharded per
  rank, the active unet's flat gradient is averaged with RCCL all-reduces over
  xGMI (~25 MB buckets overlapped with the backward, on a communicator the
  HIP library owns: GradComm).  No other collective on the data path.
"""
from __future__ import annotations

import atexit
import math
import os
import random
import sys
import threading
import time
from contextlib import contextmanager, nullcontext
from pathlib import Path

import torch
import torch.distributed as dist
import torch.nn as nn

from . import _lib, ops
from ._lib import DVError, call, ptr, stream
from .dalle2_video import VideoDecoder, cast_tuple, default, exists
from .ops import ctypes_float

__version__ = "1.14.2-mi355x"


def groupby_prefix_and_trim(prefix, d):
    with_p = {k[len(prefix):]: v for k, v in d.items() if k.startswith(prefix)}
    without = {k: v for k, v in d.items() if not k.startswith(prefix)}
    return with_p, without


class FusedAdamW(torch.optim.Optimizer):
    """AdamW over one flat f32 buffer (params are re-pointed into it).

    Parameters that never receive a gradient (e.g. the unused null_* embeds)
    stay outside the flat buffer and are skipped exactly like torch skips a
    parameter whose .grad is None."""

    def __init__(self, params, lr=1e-4, betas=(0.9, 0.99), eps=1e-8, weight_decay=1e-2):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self._flat = None  # (P, G, M, V, [(group, start, end)], params)
        self._clip_ws = None
        self._t = 0
        # bumped whenever the flat buffers are (re)built: anything that holds
        # their addresses (captured HIP graphs, packed-weight images) is stale
        self.generation = 0
        self._probe = ()  # (param, data offset, grad offset) spot checks of the aliasing
        self.order_key = None  # optional sort key of the parameters within a group
        self._zero_plan = None  # (key, flat-gradient spans zero_grad(defer=True) fills)

    # -- flat storage ------------------------------------------------------
    def _build_flat(self):
        live = []
        for gi, group in enumerate(self.param_groups):
            for p in group["params"]:
                if p.grad is not None:
                    live.append((gi, p))
        if not live:
            return
        dev = live[0][1].device
        # every parameter starts on a 64-B boundary (16 floats): the HIP kernels
        # write gradients with 16-B vector stores; the zero gaps are inert for
        # AdamW (zero grad and moments) and for the gradient norm
        al = lambda k: (k + 15) // 16 * 16
        n = sum(al(p.numel()) for _, p in live)
        P = torch.zeros(n, dtype=torch.float32, device=dev)
        G = torch.zeros(n, dtype=torch.float32, device=dev)
        M = torch.zeros(n, dtype=torch.float32, device=dev)
        V = torch.zeros(n, dtype=torch.float32, device=dev)
        ranges = []
        off = 0
        self._offsets = {}
        key = self.order_key  # flat order within a group (the all-reduce buckets follow it)
        for gi in range(len(self.param_groups)):
            start = off
            members = [p for g2, p in live if g2 == gi]
            if key is not None:
                members.sort(key=key)
            for p in members:
                k = p.numel()
                st = self.state.get(p, {})
                P[off:off + k].copy_(p.detach().reshape(-1))
                G[off:off + k].copy_(p.grad.detach().reshape(-1))
                if "exp_avg" in st:
                    M[off:off + k].copy_(st["exp_avg"].reshape(-1))
                    V[off:off + k].copy_(st["exp_avg_sq"].reshape(-1))
                p.data = P[off:off + k].view_as(p)
                p.grad = G[off:off + k].view_as(p)
                self.state[p] = dict(step=torch.tensor(float(self._t)),
                                     exp_avg=M[off:off + k].view_as(p),
                                     exp_avg_sq=V[off:off + k].view_as(p))
                self._offsets[id(p)] = off
                off += al(k)
            ranges.append((gi, start, off))
        self._flat = (P, G, M, V, ranges, [p for _, p in live])
        self.generation += 1
        ps = self._flat[5]
        self._probe = tuple((p, p.data_ptr(), p.grad.data_ptr())
                            for p in {id(q): q for q in (ps[0], ps[len(ps) // 2], ps[-1])}.values())

    def _aliased(self):
        """Do the parameters (and their grads) still live in the flat buffers?
        `Module.to()` / `.cpu()` / `.cuda()` (e.g. VideoDecoder.one_unet_in_gpu,
        reference dalle2_video.py:1508-1529) replace every `p.data`, so a spot
        check of three parameters detects it."""
        for p, dp, gp in self._probe:
            if p.data_ptr() != dp or p.grad is None or p.grad.data_ptr() != gp:
                return False
        return True

    def _rebuild_flat(self):
        """Re-point the parameters into fresh flat buffers, keeping their
        current values and gradients and the AdamW moments."""
        P, G, M, V, ranges, params = self._flat
        for p in params:
            st = self.state.get(p, {})
            for k in ("exp_avg", "exp_avg_sq"):
                if k in st:
                    st[k] = st[k].detach().clone()
            if p.grad is None or p.grad.device != p.device:
                p.grad = torch.zeros_like(p)
        self._flat = None
        self._build_flat()

    @property
    def flat_grad(self):
        return None if self._flat is None else self._flat[1]

    def ensure_flat(self):
        if self._flat is None:
            self._build_flat()
        elif not self._aliased():
            self._rebuild_flat()
        return self._flat is not None

    @torch.no_grad()
    def step(self, closure=None, clip_coef=None):
        if not self.ensure_flat():
            return None
        P, G, M, V, ranges, _ = self._flat
        _lib.require_gpu(P, G, M, V)  # raw addresses below: never a host buffer
        self._t += 1
        for gi, start, end in ranges:
            if end <= start:
                continue
            group = self.param_groups[gi]
            b1, b2 = group["betas"]
            bc1 = 1 - b1 ** self._t
            bc2s = math.sqrt(1 - b2 ** self._t)
            n = end - start
            es = 4
            call("dv_adamw", _lib.ctypes_vp(P.data_ptr() + start * es), _lib.ctypes_vp(G.data_ptr() + start * es),
                 _lib.ctypes_vp(M.data_ptr() + start * es), _lib.ctypes_vp(V.data_ptr() + start * es),
                 n, n if group["weight_decay"] > 0 else 0, ctypes_float(group["lr"]), ctypes_float(b1),
                 ctypes_float(b2), ctypes_float(group["eps"]), ctypes_float(group["weight_decay"]),
                 ctypes_float(bc1), ctypes_float(bc2s), ptr(clip_coef), stream())
        return None

    def state_dict(self):
        if self._flat is not None:
            for p in self._flat[5]:
                self.state[p]["step"] = torch.tensor(float(self._t))
        return super().state_dict()

    def zero_grad(self, set_to_none: bool = True, defer: bool = False):
        """defer=True (the trainer's update): the gradients the conv backward
        writes whole are zeroed only logically (ops.FRESH: the next backward's
        first write overwrites them), the rest for real -- the next backward
        must then run through the trainer (it zeroes what stayed unwritten).
        Reading .grad before that backward shows the old values."""
        if self._flat is not None:
            # moved parameters (sampling through host memory) hold their .grad
            # outside the flat buffer: re-point them first, so the zeros (real
            # or deferred) land in the gradients the next backward sees
            self.ensure_flat()
            params = self._flat[5]
            if defer and ops.GRAD_OVERWRITE:
                # (the armed set, its zero spans and bookkeeping are cached
                # while no parameter gets newly marked: per-update host work
                # stays a few dict updates)
                key = (self.generation, ops.FRESH.marks)
                if self._zero_plan is None or self._zero_plan[0] != key:
                    armed = [p for p in params if ops.FRESH.whole(p)]
                    self._zero_plan = (key, self._zero_spans({id(p) for p in armed}) if armed else None,
                                       ops.FRESH.plan(armed) if armed else None)
                _, spans, plan = self._zero_plan
                if plan is not None:
                    if spans:
                        torch._foreach_zero_(spans)
                    ops.FRESH.arm(self, plan=plan)
                    return
            ops.FRESH.drop(params)
            self._flat[1].zero_()  # grads stay views of the flat buffer
            return
        super().zero_grad(set_to_none=set_to_none)

    def _zero_spans(self, armed_ids):
        """Views of the flat gradient covering every parameter not in
        `armed_ids`, runs of them merged (over the alignment gaps between
        them, which stay zero anyway)."""
        G = self._flat[1]
        spans, run = [], None
        for off, k, armed in sorted((self._offsets[id(p)], p.numel(), id(p) in armed_ids) for p in self._flat[5]):
            if armed:
                if run is not None:
                    spans.append(G[run[0]:run[1]])
                run = None
            else:
                run = (off, off + k) if run is None else (run[0], off + k)
        if run is not None:
            spans.append(G[run[0]:run[1]])
        return spans

    def clip_coefficient(self, max_norm, prescale=1.0):
        """Device scalar: prescale * min(max_norm / (||prescale g|| + 1e-6), 1)."""
        if not self.ensure_flat():
            return None
        G = self._flat[1]
        if self._clip_ws is None:
            self._clip_ws = torch.zeros(516, dtype=torch.float32, device=G.device)  # DV_CLIP_WS_FLOATS
        call("dv_grad_clip_coef", ptr(G), G.numel(), ctypes_float(max_norm if max_norm else 0.0),
             ctypes_float(prescale), ptr(self._clip_ws), stream())
        return self._clip_ws[1:2]

    def load_state_dict(self, state_dict):
        if self._flat is not None:
            self.ensure_flat()  # parameters moved since the last step: re-point them first
        super().load_state_dict(state_dict)
        steps = [float(s["step"]) for s in self.state.values() if "step" in s]
        self._t = int(max(steps)) if steps else 0
        if self._flat is not None:
            # keep the flat buffers (and every graph / packed image built on
            # their addresses): copy the loaded moments into the M / V slices
            # (offsets recorded by _build_flat); a live parameter the
            # checkpoint has no moments for starts from zero moments, as a
            # fresh torch AdamW state would
            P, G, M, V, ranges, params = self._flat
            for p in params:
                st = self.state.setdefault(p, {})
                off = self._offsets[id(p)]
                k = p.numel()
                if "exp_avg" in st:
                    M[off:off + k].copy_(st["exp_avg"].reshape(-1))
                    V[off:off + k].copy_(st["exp_avg_sq"].reshape(-1))
                else:
                    M[off:off + k].zero_()
                    V[off:off + k].zero_()
                    st["step"] = torch.tensor(float(self._t))
                st["exp_avg"] = M[off:off + k].view_as(p)
                st["exp_avg_sq"] = V[off:off + k].view_as(p)


def get_optimizer(params, lr=1e-4, wd=1e-2, betas=(0.9, 0.99), eps=1e-8,
                  filter_by_requires_grad=False, group_wd_params=True, **kwargs):
    params = list(params)
    if filter_by_requires_grad:
        params = [p for p in params if p.requires_grad]
    if wd == 0:
        return FusedAdamW(params, lr=lr, betas=betas, eps=eps, weight_decay=0.0)
    if group_wd_params:
        wd_p = [p for p in params if p.ndim >= 2]
        no_wd = [p for p in params if p.ndim < 2]
        params = [{"params": wd_p}, {"params": no_wd, "weight_decay": 0.0}]
    return FusedAdamW(params, lr=lr, weight_decay=wd, betas=betas, eps=eps)


class _LinearWarmup:
    """pytorch_warmup.LinearWarmup (the reference's `warmup.LinearWarmup`,
    trainer.py:83-87), restated from pytorch_warmup's published BaseWarmup:

    * construction remembers the undamped lrs and dampens step 0 at once;
    * `dampening()` restores the undamped lrs on entry (so the wrapped
      `scheduler.step()` sees and updates the undamped values), then on exit
      records the scheduler's new lrs as undamped and dampens the next step;
    * factor(step) = min(1, (step + 1) / warmup_period)."""

    def __init__(self, optimizer, warmup_period, last_step=-1):
        self.optimizer = optimizer
        self.warmup_period = warmup_period
        self.last_step = last_step
        self.lrs = [g["lr"] for g in optimizer.param_groups]
        self.dampen()

    def warmup_factor(self, step):
        return min(1.0, (step + 1) / self.warmup_period)

    def dampen(self, step=None):
        if step is None:
            step = self.last_step + 1
        self.last_step = step
        f = self.warmup_factor(step)
        for g in self.optimizer.param_groups:
            g["lr"] *= f

    @contextmanager
    def dampening(self):
        for g, lr in zip(self.optimizer.param_groups, self.lrs):
            g["lr"] = lr
        yield
        self.lrs = [g["lr"] for g in self.optimizer.param_groups]
        self.dampen()


class EMA(nn.Module):
    """ema-pytorch EMA (beta 0.9999, update_after_step 100, update_every 10,
    inv_gamma 1, power 2/3) — outside the hot path, kept for API completeness."""

    def __init__(self, model, beta=0.9999, update_after_step=100, update_every=10, inv_gamma=1.0,
                 power=2 / 3, min_value=0.0, **kwargs):
        super().__init__()
        import copy
        self.beta, self.update_after_step, self.update_every = beta, update_after_step, update_every
        self.inv_gamma, self.power, self.min_value = inv_gamma, power, min_value
        self.online_model = [model]
        self.ema_model = copy.deepcopy(model)
        self.ema_model.requires_grad_(False)
        self.register_buffer("initted", torch.tensor(False))
        self.register_buffer("step", torch.tensor(0))

    def restore_ema_model_device(self):
        self.ema_model.to(next(self.online_model[0].parameters()).device)

    def _decay(self):
        epoch = max(self.step.item() - self.update_after_step - 1, 0)
        if epoch <= 0:
            return 0.0
        value = 1 - (1 + epoch / self.inv_gamma) ** -self.power
        return min(max(value, self.min_value), self.beta)

    @torch.no_grad()
    def update(self):
        step = self.step.item()
        self.step += 1
        if step % self.update_every != 0:
            return
        src = self.online_model[0]
        if step <= self.update_after_step or not self.initted.item():
            for pe, p in zip(self.ema_model.parameters(), src.parameters()):
                pe.copy_(p)
            self.initted.fill_(True)
            return
        d = self._decay()
        for pe, p in zip(self.ema_model.parameters(), src.parameters()):
            pe.lerp_(p, 1 - d)


def split_args_and_kwargs(*args, split_size=None, **kwargs):
    all_args = (*args, *kwargs.values())
    batch = next((a.shape[0] for a in all_args if torch.is_tensor(a)), None)
    if split_size is None or batch is None or batch <= split_size:
        yield 1.0, (args, kwargs)
        return
    n_chunks = (batch + split_size - 1) // split_size
    for i in range(n_chunks):
        sl = slice(i * split_size, (i + 1) * split_size)
        cargs = tuple(a[sl] if torch.is_tensor(a) else a for a in args)
        ckw = {k: (v[sl] if torch.is_tensor(v) else v) for k, v in kwargs.items()}
        size = next(a.shape[0] for a in (*cargs, *ckw.values()) if torch.is_tensor(a))
        yield size / batch, (cargs, ckw)


class ShardedLoader:
    """A DataLoader re-built over a rank-strided DistributedSampler (what
    accelerate's `prepare` does to the reference's loaders, trainer.py:117-124):
    rank r of N iterates samples r, r+N, ... of the (shuffled, if the original
    loader shuffles) epoch order — disjoint across ranks, same batch size per
    rank, so the global batch is N x batch_size.  The epoch (shuffle seed) is
    advanced on every new iteration, as accelerate does."""

    def __init__(self, loader, world, rank, seed=0):
        from torch.utils.data import DataLoader, DistributedSampler, RandomSampler

        self.original = loader
        shuffle = isinstance(loader.sampler, RandomSampler)
        self.sampler = DistributedSampler(loader.dataset, num_replicas=world, rank=rank,
                                          shuffle=shuffle, seed=seed, drop_last=False)
        kw = dict(batch_size=loader.batch_size, sampler=self.sampler, num_workers=loader.num_workers,
                  collate_fn=loader.collate_fn, pin_memory=loader.pin_memory,
                  drop_last=loader.drop_last, timeout=loader.timeout,
                  worker_init_fn=loader.worker_init_fn)
        if loader.num_workers > 0:
            kw.update(prefetch_factor=loader.prefetch_factor,
                      persistent_workers=loader.persistent_workers)
        self.loader = DataLoader(loader.dataset, **kw)
        self.epoch = 0

    @property
    def dataset(self):
        return self.loader.dataset

    @property
    def batch_size(self):
        return self.loader.batch_size

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        self.sampler.set_epoch(self.epoch)
        self.epoch += 1
        return iter(self.loader)


def shard_loader(loader, world, rank):
    """Per-rank view of a DataLoader (identity on one process or for objects
    that are not map-style DataLoaders)."""
    from torch.utils.data import DataLoader, IterableDataset

    if (world <= 1 or loader is None or not isinstance(loader, DataLoader)
            or isinstance(loader.dataset, IterableDataset) or loader.batch_sampler is None):
        return loader
    seed = torch.tensor([torch.initial_seed() % (1 << 31)], dtype=torch.int64)
    if dist.is_initialized():
        if dist.get_backend() == "nccl":  # RCCL collectives take device tensors
            seed = seed.cuda()
        dist.broadcast(seed, 0)  # one shuffle order for all ranks
    seed = int(seed.item())
    if loader.batch_size is None:
        # a custom batch_sampler (automatic batching off in the rebuilt form):
        # keep its batches and give rank r every world-th one
        return _BatchStridedLoader(loader, world, rank, seed)
    return ShardedLoader(loader, world, rank, seed=seed)


class _BatchStridedLoader:
    """Per-rank view of a DataLoader driven by a custom batch_sampler: rank r
    of N takes batches r, r+N, ... (the sampler's own batches, unchanged).
    Every rank must draw the same batch order: a batch sampler over an
    unseeded RandomSampler gets a generator seeded with the broadcast seed;
    any other source of randomness is the caller's to seed."""

    def __init__(self, loader, world, rank, seed=0):
        from torch.utils.data import DataLoader, RandomSampler

        import copy

        # seed COPIES of the batch sampler and its RandomSampler: the caller's
        # DataLoader keeps drawing from the global RNG as before
        bs = loader.batch_sampler
        inner = getattr(bs, "sampler", None)
        if isinstance(inner, RandomSampler) and inner.generator is None:
            inner = copy.copy(inner)
            inner.generator = torch.Generator().manual_seed(seed)
            bs = copy.copy(bs)
            bs.sampler = inner

        class _Strided:
            def __init__(self, bs):
                self.bs = bs

            def __iter__(self):
                for i, b in enumerate(self.bs):
                    if i % world == rank:
                        yield b

            def __len__(self):
                n = len(self.bs)
                return n // world + (1 if rank < n % world else 0)

        self.original = loader
        kw = dict(batch_sampler=_Strided(bs), num_workers=loader.num_workers,
                  collate_fn=loader.collate_fn, pin_memory=loader.pin_memory, timeout=loader.timeout,
                  worker_init_fn=loader.worker_init_fn, generator=loader.generator)
        if loader.num_workers > 0:
            kw.update(prefetch_factor=loader.prefetch_factor,
                      persistent_workers=loader.persistent_workers)
        self.loader = DataLoader(loader.dataset, **kw)

    @property
    def dataset(self):
        return self.loader.dataset

    @property
    def batch_size(self):
        return None

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        return iter(self.loader)


def broadcast_parameters(module, src=0):
    """DDP's init broadcast: every rank starts from rank `src`'s weights."""
    for p in module.parameters():
        dist.broadcast(p.data, src)


BUCKET_BYTES = int(os.environ.get("DV_BUCKET_MB", "25")) * (1 << 20)

class _NativeComms:
    """libdv_hip's RCCL communicators of this process, one per (process group,
    rank, world), with what ProcessGroupNCCL's watchdog gave the reference's
    DDP: a daemon thread polls dv_comm_async_error every second and, while a
    training call or update is in flight, enforces a deadline
    (DV_COMM_TIMEOUT seconds, default 1800 like the c10d timeout); on an
    error or a missed deadline it aborts the communicators and ends the
    process with exit code 70, so a dead peer does not leave the other ranks
    blocked in a stream wait forever.  Communicators are destroyed at exit
    (or when their process group is no longer the default one).

    Handle lifetime: every use of a handle -- the watchdog's poll and abort,
    check(), destroy -- happens while holding `lock`, and a destroyed handle
    leaves `comms` in the same critical section, so the watchdog can never
    poll a freed communicator.  close() also stops and joins the watchdog
    before it destroys anything.  `lib` / `exit_fn` are injectable (tests run
    the supervision logic on the CPU with a stub library)."""

    def __init__(self, lib=None, exit_fn=None, poll_s=1.0, timeout=None):
        self.comms = {}     # (id(group), rank, world) -> (group, handle)
        self.serial = 0     # every rank makes its communicators in the same order
        self.lock = threading.Lock()
        self.busy_since = None
        self.failed = False
        self.thread = None
        self.stop = threading.Event()
        self.poll_s = poll_s
        self._lib = lib
        self._exit = exit_fn if exit_fn is not None else os._exit
        self.timeout = float(os.environ.get("DV_COMM_TIMEOUT", "1800")) if timeout is None else timeout
        if lib is None:
            atexit.register(self.close)

    def L(self):
        return self._lib if self._lib is not None else _lib.lib()

    def _call(self, name, *args):
        L = self.L()
        rc = getattr(L, name)(*args)
        if rc != 0:
            raise DVError(f"{name} failed ({rc}): {L.dv_last_error().decode(errors='replace')}")

    def get(self, device, group=None, rank=None, world=None, store=None):
        import ctypes

        group = dist.distributed_c10d._get_default_group() if group is None else group
        rank = dist.get_rank() if rank is None else rank
        world = dist.get_world_size() if world is None else world
        key = (id(group), rank, world)
        with self.lock:
            ent = self.comms.get(key)
            if ent is not None and ent[0] is group:
                return ent[1]
            # communicators of groups that are no longer the default one
            stale = [k for k, (g, _) in self.comms.items() if g is not group]
        for k in stale:
            self._drop(k, destroy=True)
        self.serial += 1
        name = f"dv_comm/{self.serial}"
        store = dist.distributed_c10d._get_default_store() if store is None else store
        buf = ctypes.create_string_buffer(128)
        if rank == 0:
            self._call("dv_comm_unique_id", buf)
            store.set(name, buf.raw)
        else:
            ctypes.memmove(buf, store.get(name), 128)
        handle = ctypes.c_void_p()
        dev = device.index if device.index is not None else torch.cuda.current_device()
        self._call("dv_comm_init", buf, world, rank, dev, ctypes.byref(handle))
        with self.lock:
            self.comms[key] = (group, handle)
        if self.thread is None and os.environ.get("DV_COMM_WATCHDOG", "1") != "0":
            self.stop.clear()
            self.thread = threading.Thread(target=self._watch, name="dv_comm_watchdog", daemon=True)
            self.thread.start()
        return handle

    def _drop(self, key, destroy):
        # destroy under the lock: the watchdog polls only while holding it
        with self.lock:
            ent = self.comms.pop(key, None)
            if ent is not None:
                getattr(self.L(), "dv_comm_destroy" if destroy else "dv_comm_abort")(ent[1])

    def check(self):
        """Raise DVError if a communicator reports an asynchronous error
        (update() calls this outside any capture)."""
        with self.lock:
            for _, h in self.comms.values():
                self._call("dv_comm_async_error", h)

    def mark(self, busy):
        self.busy_since = time.monotonic() if busy else None

    def _watch(self):
        L = self.L()
        while not self.stop.wait(self.poll_s):
            with self.lock:
                if self.stop.is_set():
                    return
                handles = [h for _, h in self.comms.values()]
                bad = next((h for h in handles if L.dv_comm_async_error(h) != 0), None)
                since = self.busy_since
                late = since is not None and time.monotonic() - since > self.timeout
                if bad is None and not late:
                    continue
                why = ("RCCL communicator error: " + L.dv_last_error().decode(errors="replace")) \
                    if bad is not None else \
                    f"no progress for {self.timeout:.0f} s in a training call with collectives (DV_COMM_TIMEOUT)"
                sys.stderr.write(f"[dv_comm watchdog] {why}; aborting the communicators and exiting\n")
                sys.stderr.flush()
                self.failed = True
                for h in handles:
                    L.dv_comm_abort(h)
                self.comms.clear()
            self._exit(70)
            return

    def close(self):
        """Stop and join the watchdog, then destroy (or, after a failure,
        abort) every communicator."""
        self.stop.set()
        t = self.thread
        if t is not None and t is not threading.current_thread():
            t.join(timeout=10 * self.poll_s + 1)
        self.thread = None
        with self.lock:
            keys = list(self.comms)
        for k in keys:
            try:
                self._drop(k, destroy=not self.failed)
            except Exception:  # interpreter teardown: best effort
                pass


_NATIVE = _NativeComms()


class GradComm:
    """The data path's one collective: the gradient all-reduce, as a MEAN
    over ranks (DDP's bucket semantics: averaging an already averaged bucket
    again is the identity, so gradients that accumulate over several trainer
    calls before update() stay correct however often a part is reduced).

    * RCCL (`nccl` process group, CUDA tensors): a communicator owned by
      libdv_hip (dv_comm_*, _NativeComms), made once per process group; the
      id travels through the torch.distributed store.  The all-reduce is
      enqueued on the CURRENT stream — eagerly, or inside a HIP-graph capture
      of the backward — with no c10d work object: ProcessGroupNCCL's watchdog
      polls the events of its works from another thread, and one recorded in a
      capturing stream aborts the process (hipErrorCapturedEvent), so captured
      collectives never go through it.
    * anything else (gloo: the CPU tests, the shared-GPU rehearsals): c10d
      SUM then a 1/world scale.
    Which of the two is resolved from the first tensor reduced (parameters
    may still be on the host when the trainer is built); an `nccl` group with
    host tensors is an error, never a silent c10d fallback."""

    def __init__(self, world, device=None):
        self.world = world
        self._native = None
        self._resolved = False
        if device is not None and device.type == "cuda":
            self.resolve(device)

    def resolve(self, device):
        if not self._resolved:
            nccl = dist.is_initialized() and dist.get_backend() == "nccl"
            if nccl and device.type != "cuda":
                raise DVError("the nccl (RCCL) gradient all-reduce needs CUDA tensors; "
                              "move the decoder to the GPU before training")
            self._native = _NATIVE.get(device) if nccl else None
            self._resolved = True
        return self._native

    @property
    def native(self):
        return self._native

    def capturable(self, device):
        """True when the collective can go into a HIP-graph capture (RCCL)."""
        return self.resolve(device) is not None

    def check(self):
        if self._native is not None:
            _NATIVE.check()

    def allreduce_mean_(self, t):
        """Mean over ranks, in place, on the current stream.  Returns None
        (stream-ordered: RCCL) or a pending c10d work for finish()."""
        if self.resolve(t.device) is not None:
            call("dv_comm_allreduce", self._native, ptr(t), t.numel(), _lib.dt(t), 1, stream())
            return None
        return (dist.all_reduce(t, async_op=True), t)

    def finish(self, pending):
        work, t = pending
        work.wait()
        if self.world > 1:
            t.mul_(1.0 / self.world)


def allreduce_flat_grad(flat_grad, world, bucket_bytes=None, force=False, comm=None):
    """Average the active unet's flat f32 gradient over the ranks (in place).
    RCCL: one stream-ordered collective (RCCL pipelines a 200 MB buffer over
    the xGMI links itself).  c10d: ~bucket_bytes buckets issued back to front
    (async), then the 1/world scale."""
    if (world <= 1 and not force) or flat_grad is None:
        return flat_grad
    comm = comm or GradComm(world, flat_grad.device)
    if comm.resolve(flat_grad.device) is not None:
        comm.allreduce_mean_(flat_grad)
        return flat_grad
    n = flat_grad.numel()
    per = max(1, (bucket_bytes or BUCKET_BYTES) // flat_grad.element_size())
    pend = [comm.allreduce_mean_(flat_grad[max(0, end - per):end]) for end in range(n, 0, -per)]
    for p in pend:
        comm.finish(p)
    return flat_grad


class OverlappedAllReduce:
    """The gradient all-reduce of one unet overlapped with its backward — what
    DDP's bucket hooks do inside the reference's accelerator.backward
    (trainer.py:360).

    * The first training call RECORDS the backward order: Unet3D's forward
      marks every block input (ops.backward_mark) and, at each mark's
      gradient hook, the parameters whose .grad exists by then get that hook's
      index (their gradient kernels — or streamed split-K sums — have been
      launched).  Parameters never seen before the end rank last.
    * The optimizer's flat buffer is laid out in that order within each
      weight-decay group (FusedAdamW.order_key), and cut into ~BUCKET_BYTES
      buckets of whole parameters; a bucket is ready at the largest index of
      its parameters.
      (Each Unet3D parameter's gradient comes from ONE backward op — no
      weight is applied twice — so its first appearance is its completion,
      once the writes the backward defers are flushed: see _launch.)
    * Every later call: at hook k, each bucket ready by k is averaged over
      the ranks (GradComm: RCCL on libdv_hip's communicator) on a comm stream
      that first waits for every stream writing gradients; the rest go at the
      end of the backward.  update() waits for them (a captured call joins
      them inside the graph).  The mean is idempotent, so a second call
      before update() (gradient accumulation, the reference's val loop in
      train_decoder.py:146-151) re-averages the already averaged part to
      itself, as DDP does."""

    def __init__(self, opt, world, gcomm):
        self.opt, self.world, self.gcomm = opt, world, gcomm
        self.ranks = None      # id(param) -> backward index
        self.mode = None       # "record" / "run" during a call
        self.hit = 0
        self.plan = None       # (generation, [(start, end, ready)])
        self.launched = 0
        self.pending = []      # c10d works (gloo) still to finish
        self.comm = None
        self.params = None

    def attach(self, params):
        self.params = [p for p in params if p.requires_grad]
        big = 1 << 30
        self.opt.order_key = lambda p: (self.ranks or {}).get(id(p), big)

    def _buckets(self):
        gen = self.opt.generation
        if self.plan is not None and self.plan[0] == gen:
            return self.plan[1]
        P, G, M, V, ranges, params = self.opt._flat
        big = 1 << 30
        per = max(1, BUCKET_BYTES // 4)
        spans = sorted((self.opt._offsets[id(p)], p.numel(), self.ranks.get(id(p), big) if self.ranks else big)
                       for p in params)
        out, cur = [], None
        for gi, gstart, gend in ranges:  # buckets never straddle a group boundary
            for off, n, rk in spans:
                if not gstart <= off < gend:
                    continue
                if cur is None or (off + n) - cur[0] > per:
                    if cur is not None:
                        out.append(tuple(cur))
                    cur = [off, off + n, rk]
                else:
                    cur[1], cur[2] = off + n, max(cur[2], rk)
            if cur is not None:
                cur[1] = gend  # include the alignment gap
                out.append(tuple(cur))
                cur = None
        self.plan = (gen, out)
        return out

    def begin(self):
        """Before a training call's forward: arm the hooks."""
        self.hit = 0
        self.launched = 0
        if self.ranks is None:
            self.mode = "record"
            self.ranks = {}
            # a gradient that exists before the backward (accumulating into an
            # earlier one) says nothing about the order: those rank last
            self._pre = {id(p) for p in self.params if p.grad is not None}
        elif self.opt._flat is not None and self.opt._aliased():
            self.mode = "run"
            self.comm = self.comm or torch.cuda.Stream(device=self.opt._flat[1].device)
        else:
            self.mode = None
            return
        ops._BackwardMarks.tracker = self

    def on_hit(self, grad):
        self.hit += 1
        if self.mode == "record":
            for p in self.params:
                if id(p) not in self.ranks and p.grad is not None and id(p) not in self._pre:
                    self.ranks[id(p)] = self.hit
        elif self.mode == "run":
            self._launch(self.hit)
        return None

    def _launch(self, upto):
        buckets = self._buckets()
        G = self.opt.flat_grad
        if self.launched < len(buckets) and buckets[self.launched][2] <= upto:
            # gradient writes the backward defers (batched split-K sums, the
            # cross-attention fold backwards) land before a bucket goes out: a
            # parameter ranks where its .grad was allocated, which is where its
            # deferred write was queued
            if ops.WGRAD_DEFER.pending:
                ops.WGRAD_DEFER.flush()
            if ops._FOLD_BWD_PENDING:
                ops.flush_fold_bwd()
        while self.launched < len(buckets) and buckets[self.launched][2] <= upto:
            start, end, _ = buckets[self.launched]
            dev = G.device
            # every stream that may still write gradients of this bucket: the
            # compute stream, the streamed split-K sums, the side-stream wgrads
            self.comm.wait_stream(torch.cuda.current_stream(dev))
            side = ops.WGRAD_DEFER.streamed
            if side is not None:
                self.comm.wait_stream(ops.WGRAD_DEFER._side(side))
            with torch.cuda.stream(self.comm):
                pend = self.gcomm.allreduce_mean_(G[start:end])
            if pend is not None:
                self.pending.append(pend)
            self.launched += 1

    def end(self, join):
        """After the backward (the deferred-wgrad sums joined): the remaining
        buckets; join=True waits for every bucket here (a captured call)."""
        ops._BackwardMarks.tracker = None
        mode, self.mode = self.mode, None
        if mode == "record":
            return False
        if mode != "run":
            return False
        self._launch(1 << 31)
        if join:
            self.wait()
        return True

    def abort(self):
        ops._BackwardMarks.tracker = None
        self.mode = None

    def wait(self):
        """The caller's stream waits for every launched bucket (inside a
        capture this is the join of the comm stream back into the graph)."""
        for p in self.pending:
            self.gcomm.finish(p)
        self.pending = []
        if self.comm is not None:
            torch.cuda.current_stream(self.comm.device).wait_stream(self.comm)


class VideoDecoderTrainer(nn.Module):
    def __init__(self, decoder, accelerator=None, dataloaders=None, use_ema=True, lr=1e-4,
                 wd=1e-2, eps=1e-8, warmup_steps=None, cosine_decay_max_steps=None,
                 max_grad_norm=0.5, amp=False, group_wd_params=True, use_graphs=None, **kwargs):
        super().__init__()
        # HIP-graph replay of the forward+backward (opt-in; DV_GRAPHS=1): after two
        # eager calls per (unet, input shapes), the whole p_losses forward and the
        # autograd backward are captured once and replayed, removing the ~600
        # host-side kernel launches per step.
        self.use_graphs = (os.environ.get("DV_GRAPHS", "") == "1") if use_graphs is None else use_graphs
        self._graphs = {}
        # weights change only in update(): keep their packed MFMA images cached
        from . import ops
        if os.environ.get("DV_PACK_CACHE", "1") != "0":
            ops.PACK.enabled = True
        assert isinstance(decoder, VideoDecoder)
        ema_kwargs, kwargs = groupby_prefix_and_trim("ema_", kwargs)
        self.accelerator = accelerator
        self.num_unets = len(decoder.unets)
        self.use_ema = use_ema
        self.ema_unets = nn.ModuleList([])
        self.amp = amp or os.environ.get("DV_AMP", "") == "bf16"
        lr, wd, eps, warmup_steps, cosine_decay_max_steps = (
            cast_tuple(v, self.num_unets) for v in (lr, wd, eps, warmup_steps, cosine_decay_max_steps))
        assert all(l <= 1e-2 for l in lr), \
            "your learning rate is too high, recommend sticking with 1e-4, at most 5e-4"
        self.world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        self.decoder = decoder
        for i, (unet, ulr, uwd, ueps, uwarm, ucos) in enumerate(
                zip(decoder.unets, lr, wd, eps, warmup_steps, cosine_decay_max_steps)):
            opt = get_optimizer(unet.parameters(), lr=ulr, wd=uwd, eps=ueps,
                                group_wd_params=group_wd_params, **kwargs)
            sched = (torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=ucos) if exists(ucos)
                     else torch.optim.lr_scheduler.LambdaLR(opt, lr_lambda=lambda step: 1.0))
            setattr(self, f"optim{i}", opt)
            setattr(self, f"sched{i}", sched)
            if self.use_ema:
                self.ema_unets.append(EMA(unet, **ema_kwargs))
        self.warmup_schedulers = [(_LinearWarmup(getattr(self, f"optim{i}"), w) if exists(w) else None)
                                  for i, w in enumerate(warmup_steps)]
        self.max_grad_norm = max_grad_norm
        self.register_buffer("steps", torch.tensor([0] * self.num_unets))
        # gradient all-reduce overlapped with the backward (N > 1; DV_OVERLAP=0
        # turns it off; DV_FORCE_ALLREDUCE=1 runs the collective path on a
        # one-rank group too, for tests)
        self.force_allreduce = (os.environ.get("DV_FORCE_ALLREDUCE", "0") == "1"
                                and dist.is_available() and dist.is_initialized())
        self.overlap = None
        self.gcomm = None
        if self.world > 1 or self.force_allreduce:
            # resolved from the first gradient reduced (the decoder may move later)
            self.gcomm = GradComm(self.world)
        if (self.world > 1 or self.force_allreduce) and os.environ.get("DV_OVERLAP", "1") != "0":
            self.overlap = []
            for i, unet in enumerate(decoder.unets):
                ov = OverlappedAllReduce(getattr(self, f"optim{i}"), self.world, self.gcomm)
                ov.attach(unet.parameters())
                self.overlap.append(ov)
        self._reduced = [False] * self.num_unets  # the last call's gradient is already all-reduced
        # bench.py at N > 1: a list -> eager calls record ["exposed", end of the
        # backward's compute, every bucket joined] event pairs
        self.comm_probe = None
        self._gen_seen = [getattr(self, f"optim{i}").generation for i in range(self.num_unets)]
        # accelerator.prepare(..., train, val) (trainer.py:117-124) shards the
        # loaders per process: each rank iterates a disjoint rank-strided part
        # and places the batches on the device (here: pinned host batches
        # copied on a side stream one batch ahead, datasets.DeviceLoader)
        rank = dist.get_rank() if self.world > 1 else 0
        self.train_loader = self._prepare_loader(dataloaders["train"], rank) if exists(dataloaders) else None
        self.val_loader = self._prepare_loader(dataloaders["val"], rank) if exists(dataloaders) else None
        if self.world > 1:
            broadcast_parameters(decoder, 0)

    def _prepare_loader(self, loader, rank):
        from .datasets import DeviceLoader

        loader = shard_loader(loader, self.world, rank)
        dev = next(self.decoder.parameters()).device
        if loader is None or dev.type != "cuda" or os.environ.get("DV_DEVICE_LOADER", "1") == "0":
            return loader
        return DeviceLoader(loader, dev)

    @property
    def device(self):
        return self.decoder.device

    def validate_and_return_unet_number(self, unet_number=None):
        if self.num_unets == 1:
            unet_number = default(unet_number, 1)
        assert exists(unet_number) and 1 <= unet_number <= self.num_unets
        return unet_number

    def num_steps_taken(self, unet_number=None):
        return self.steps[self.validate_and_return_unet_number(unet_number) - 1].item()

    @property
    def unets(self):
        return nn.ModuleList([ema.ema_model for ema in self.ema_unets])

    def increment_step(self, unet_number):
        self.steps[unet_number - 1] += 1

    # -- one optimizer step (trainer.py:247-274) ----------------------------
    def _check_flat(self, unet_number):
        """Re-point the unet's parameters into fresh flat buffers if they moved
        (Module.to / one_unet_in_gpu, e.g. trainer.sample with use_non_ema);
        True when that happened — every captured graph of this unet and every
        packed image keyed on the old storage is then dropped."""
        opt = getattr(self, f"optim{unet_number - 1}")
        opt.ensure_flat()
        # against the last generation THIS trainer saw: a rebuild can also
        # happen inside FusedAdamW.load_state_dict
        if opt.generation == self._gen_seen[unet_number - 1]:
            return False
        self._gen_seen[unet_number - 1] = opt.generation
        self._graphs = {k: v for k, v in self._graphs.items() if k[0] != unet_number}
        if ops.PACK.enabled:
            ops.PACK.prune()
        return True

    def update(self, unet_number=None):
        if self.gcomm is not None:
            self.gcomm.check()  # an asynchronous RCCL error surfaces here, outside any capture
        unet_number = self.validate_and_return_unet_number(unet_number)
        index = unet_number - 1
        opt = getattr(self, f"optim{index}")
        sched = getattr(self, f"sched{index}")
        if self._check_flat(unet_number):
            self._reduced[index] = False  # re-pointed buffers: reduce the copied gradient again
        ops.FRESH.finish(opt)  # no backward since the last update: its deferred zeros become real
        if self._reduced[index]:
            self.overlap[index].wait()  # the overlapped buckets (a captured call joined them already)
            if self.comm_probe is not None and self.comm_probe and self.comm_probe[-1][0] == "bwd":
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()  # every bucket joined: the all-reduce time left after the backward
                self.comm_probe[-1] = ["exposed", self.comm_probe[-1][1], ev]
        else:
            allreduce_flat_grad(opt.flat_grad, self.world, force=self.force_allreduce, comm=self.gcomm)
        self._reduced[index] = False
        coef = opt.clip_coefficient(self.max_grad_norm)  # the gradient is already the mean over ranks
        opt.step(clip_coef=coef)
        opt.zero_grad(defer=True)  # the next call's backward overwrites the conv gradients
        if ops.PACK.enabled:
            ops.PACK.refresh()  # repack every cached image in one launch
        warm = self.warmup_schedulers[index]
        with (warm.dampening() if exists(warm) else nullcontext()):
            sched.step()
        if self.use_ema:
            self.ema_unets[index].update()
        self.increment_step(unet_number)

    def _to_device(self, v):
        if v is None:
            return v
        if not torch.is_tensor(v):
            import numpy as np
            if isinstance(v, np.ndarray):
                v = torch.from_numpy(v)
            else:
                return v
        return v.to(self.device)

    def _overlap_for(self, unet_number):
        return None if self.overlap is None else self.overlap[unet_number - 1]

    def _graphable(self, unet_number, max_batch_size, return_lowres_cond_video):
        from . import ops
        # per-launch timing cannot be replayed; a low-res conditioner's blur
        # decision is host-side randomness: it is drawn per call and selects
        # one of two captured graphs (_forward), which needs a fixed sigma and
        # kernel size (a tuple range would draw more per call)
        lc = self.decoder.lowres_conds[unet_number - 1]
        fixed = lc is None or not (isinstance(lc.blur_sigma, tuple) or isinstance(lc.blur_kernel_size, tuple))
        return (self.use_graphs and self.training and max_batch_size is None
                and not return_lowres_cond_video and ops.TIMER is None and fixed
                and getattr(self, f"optim{unet_number - 1}").flat_grad is not None)

    def _graphed_call(self, unet_number, args, kwargs, variant=None):
        """Replay (capturing on first use) forward + backward of one training
        call; `variant` (the pinned blur decision) selects the graph."""
        opt = getattr(self, f"optim{unet_number - 1}")
        # the deferred gradient zeros the call starts from (ops.FRESH): a call
        # right after update() overwrites the conv gradients, an accumulating
        # call adds to them -- two different captured passes
        sig = (unet_number, self.amp, variant, ops.FRESH.token(opt),
               tuple((tuple(a.shape), a.dtype) if torch.is_tensor(a) else repr(a) for a in args),
               tuple((k, (tuple(v.shape), v.dtype) if torch.is_tensor(v) else repr(v))
                     for k, v in sorted(kwargs.items())))
        ent = self._graphs.get(sig)
        if ent is None:
            ent = self._graphs[sig] = {"eager": 0}
        if ent["eager"] < 2:  # warm every lazy allocation / workspace first
            ent["eager"] += 1
            return None
        if "graph" not in ent:
            sargs = tuple(a.clone() if torch.is_tensor(a) else a for a in args)
            skw = {k: (v.clone() if torch.is_tensor(v) else v) for k, v in kwargs.items()}
            # the overlapped all-reduce goes into the graph only where the
            # collective can be captured (RCCL); with gloo the update reduces
            ov = self._overlap_for(unet_number)
            if ov is not None and not self.gcomm.capturable(self.device):
                ov = None
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            overlapped = False
            # thread-local capture: the process group's watchdog thread polls
            # the events of earlier (eager) collectives while this thread
            # captures, which the default global mode turns into an error
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                ctx = (torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False)
                       if self.amp else nullcontext())
                if ov is not None:
                    ov.begin()
                try:
                    with ops.defer_wgrad():  # split-K sums streamed (or batched) inside the pass
                        with ctx:
                            loss = self.decoder(*sargs, unet_number=unet_number, **skw)
                        loss.backward()
                    left = ops.FRESH.finish(opt, sync=None if ov is None else ov.wait)
                except BaseException:
                    if ov is not None:
                        ov.abort()
                    raise
                if ov is not None:
                    # collectives captured and joined; a gradient zeroed after
                    # its bucket went out is reduced again by update()
                    overlapped = ov.end(join=True) and not left
                # replays start from zeroed GroupNorm sums whatever the parity
                # of the GroupNorm calls inside the graph (ops._GnSums)
                ops.gn_graph_boundary(loss.device)
            ent.update(graph=g, args=sargs, kwargs=skw, loss=loss.detach(), overlapped=overlapped)
        # the captured inputs: copied in unless this call passes the very tensor
        # of the previous one, unmodified since (torch's version counter) -- a
        # training loop that feeds one resident batch skips the copies
        seen = ent.setdefault("seen", {})

        def feed(key, dst, src):
            prev = seen.get(key)
            if (prev is not None and prev[0]() is src and prev[1] == src._version
                    and prev[2] == dst._version):
                return
            dst.copy_(src)
            import weakref
            seen[key] = (weakref.ref(src), src._version, dst._version)

        for i, (dst, src) in enumerate(zip(ent["args"], args)):
            if torch.is_tensor(dst):
                feed(i, dst, src)
        for k, v in kwargs.items():
            if torch.is_tensor(v):
                feed(k, ent["kwargs"][k], v)
        ent["graph"].replay()
        ops.FRESH.consume(opt)
        self._reduced[unet_number - 1] = ent["overlapped"]
        return ent["loss"].item()

    def forward(self, *args, unet_number=None, max_batch_size=None, return_lowres_cond_video=False,
                **kwargs):
        watched = self.gcomm is not None and self.gcomm.native is not None
        if watched:
            _NATIVE.mark(True)  # the watchdog's deadline covers the blocking loss.item()
        try:
            return self._forward(*args, unet_number=unet_number, max_batch_size=max_batch_size,
                                 return_lowres_cond_video=return_lowres_cond_video, **kwargs)
        finally:
            if watched:
                _NATIVE.mark(False)

    def _forward(self, *args, unet_number=None, max_batch_size=None, return_lowres_cond_video=False,
                 **kwargs):
        unet_number = self.validate_and_return_unet_number(unet_number)
        args = tuple(self._to_device(a) for a in args)
        kwargs = {k: self._to_device(v) for k, v in kwargs.items()}
        if self.training and getattr(self, f"optim{unet_number - 1}").flat_grad is not None:
            # a moved unet (sampling without EMA moves the trainable unets through
            # host memory) is re-pointed into fresh flat buffers BEFORE anything
            # runs: a captured graph must never replay against the old storage
            self._check_flat(unet_number)
        ov = self._overlap_for(unet_number)
        if ov is not None:
            # a previous call's buckets may still be in flight on the comm
            # stream: this call's backward accumulates into the same buffer
            ov.wait()
        graphable = self._graphable(unet_number, max_batch_size, return_lowres_cond_video)
        lc = self.decoder.lowres_conds[unet_number - 1]
        if graphable and lc is not None:
            # the conditioner's one host draw per call (LowresVideoConditioner.forward),
            # made here and pinned for this call: the graph of that decision replays,
            # and the eager warm-up calls below see the same decision
            lc.forced_blur = bool(lc.use_blur and random.random() < lc.blur_prob)
        try:
            return self._forward_calls(args, kwargs, unet_number, max_batch_size, return_lowres_cond_video,
                                       graphable, None if lc is None else lc.forced_blur)
        finally:
            if lc is not None:
                lc.forced_blur = None

    def _forward_calls(self, args, kwargs, unet_number, max_batch_size, return_lowres_cond_video,
                       graphable, variant):
        if graphable:
            out = self._graphed_call(unet_number, args, kwargs, variant)
            if out is not None:
                return out
        total_loss = 0.0
        cond_videos = []
        chunks = list(split_args_and_kwargs(*args, split_size=max_batch_size, **kwargs))
        # overlap only a single-chunk call (chunks accumulate into the same buffer)
        ov = self._overlap_for(unet_number) if (self.training and len(chunks) == 1) else None
        if ov is not None and graphable and not self.gcomm.capturable(self.device):
            # the eager calls that warm a capture run the pass the graph will
            # hold: without a capturable collective (gloo) the graph has no
            # bucket hooks, so the deferred split-K sums it replays are ONE
            # batch; bucket flushes here would leave the captured pass a
            # deferred-sum table no eager call built (ops._WgradDefer.flush)
            ov = None
        self._reduced[unet_number - 1] = False
        for frac, (cargs, ckw) in chunks:
            ctx = torch.autocast("cuda", dtype=torch.bfloat16) if self.amp else nullcontext()
            if ov is not None:
                ov.begin()
            try:
                with ops.defer_wgrad():  # the gradients are complete when it exits
                    with ctx:
                        out = self.decoder(*cargs, unet_number=unet_number,
                                           return_lowres_cond_video=return_lowres_cond_video, **ckw)
                    loss, cv = (out if return_lowres_cond_video else (out, None))
                    loss = loss * frac
                    if cv is not None:
                        cond_videos.append(cv)
                    total_loss += loss.item()
                    if self.training:
                        loss.backward()
                # deferred gradient zeros (ops.FRESH) this backward did not overwrite
                left = self.training and ops.FRESH.finish(getattr(self, f"optim{unet_number - 1}"),
                                                          sync=None if ov is None else ov.wait)
            except BaseException:
                if ov is not None:
                    ov.abort()
                raise
            if ov is not None:
                if self.comm_probe is not None:  # the backward's compute is queued
                    ev = torch.cuda.Event(enable_timing=True)
                    ev.record()
                    self.comm_probe.append(["bwd", ev])
                # a gradient zeroed after its bucket went out is reduced again by update()
                self._reduced[unet_number - 1] = ov.end(join=False) and not left
        if return_lowres_cond_video:
            return total_loss, torch.stack(cond_videos)
        return total_loss

    # -- checkpointing (trainer.py:158-235) ---------------------------------
    def save(self, path, overwrite=True, **kwargs):
        path = Path(path)
        assert not (path.exists() and not overwrite)
        path.parent.mkdir(parents=True, exist_ok=True)
        obj = dict(model=self.decoder.state_dict(), version=__version__, steps=self.steps.cpu(), **kwargs)
        for i in range(self.num_unets):
            obj[f"optim{i}"] = getattr(self, f"optim{i}").state_dict()
            obj[f"sched{i}"] = getattr(self, f"sched{i}").state_dict()
        if self.use_ema:
            obj["ema"] = self.ema_unets.state_dict()
        if self.world == 1 or dist.get_rank() == 0:
            torch.save(obj, str(path))

    def load_state_dict(self, loaded_obj, only_model=False, strict=True):
        self.decoder.load_state_dict(loaded_obj["model"], strict=strict)
        self.steps.copy_(loaded_obj["steps"])
        if only_model:
            return loaded_obj
        for i, last in zip(range(self.num_unets), self.steps.tolist()):
            getattr(self, f"optim{i}").load_state_dict(loaded_obj[f"optim{i}"])
            getattr(self, f"sched{i}").load_state_dict(loaded_obj[f"sched{i}"])
            if exists(self.warmup_schedulers[i]):
                self.warmup_schedulers[i].last_step = last
        if self.use_ema:
            self.ema_unets.load_state_dict(loaded_obj["ema"], strict=strict)
        return loaded_obj

    def load(self, path, only_model=False, strict=True):
        path = Path(path)
        assert path.exists()
        obj = torch.load(str(path), map_location="cpu", weights_only=True)
        self.load_state_dict(obj, only_model=only_model, strict=strict)
        from . import ops
        ops.PACK.refresh()  # weights replaced: repack every cached image
        return obj

    @torch.no_grad()
    def sample(self, *args, max_batch_size=None, **kwargs):
        """trainer.py:276-300: sample with the EMA unets swapped in (unless
        `use_non_ema` or EMA is off); inputs are moved to the decoder's device
        and split into `max_batch_size` chunks (decoder_sample_in_chunks)."""
        args = tuple(self._to_device(a) for a in args)
        kwargs = {k: self._to_device(v) for k, v in kwargs.items()}
        kwargs["distributed"] = self.world > 1
        use_non_ema = kwargs.pop("use_non_ema", False) or not self.use_ema
        dec = self.decoder
        was = dec.training
        dec.eval()
        trainable = dec.unets
        if not use_non_ema:
            dec.unets = self.unets  # swap in the exponential moving averaged unets
        try:
            if max_batch_size is None:
                out = dec.sample(*args, **kwargs)
            else:
                outs = [dec.sample(*ca, **ck) for _, (ca, ck) in
                        split_args_and_kwargs(*args, split_size=max_batch_size, **kwargs)]
                out = torch.cat(outs, dim=0)
        finally:
            dec.unets = trainable
            if not use_non_ema:
                for ema in self.ema_unets:
                    ema.restore_ema_model_device()
            dec.train(was)
        return out
