"""Supervision of libdv_hip's RCCL communicators (trainer._NativeComms) on the
CPU, with a stub library standing in for dv_comm_*: the deadline, the abort
with exit code 70 on an async error, close() joining the watchdog before any
destroy, and the stale-group replacement in get() — never a poll of a
destroyed handle (the watchdog raced ncclCommDestroy)."""
import ctypes
import os
import sys
import threading
import time

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))

from dalle2_video import trainer as T  # noqa: E402


class StubLib:
    """dv_comm_* on host integers; records every call and flags a poll of a
    handle that was already destroyed or aborted."""

    def __init__(self, poll_sleep=0.0):
        self.lock = threading.Lock()
        self.next = 100
        self.live, self.dead = set(), set()
        self.log, self.violations = [], []
        self.error_on = set()
        self.poll_sleep = poll_sleep

    def _h(self, h):
        return h.value if isinstance(h, ctypes.c_void_p) else h

    def dv_comm_unique_id(self, buf):
        ctypes.memset(buf, 7, 128)
        return 0

    def dv_comm_init(self, buf, world, rank, dev, out):
        with self.lock:
            self.next += 1
            h = self.next
            self.live.add(h)
        ctypes.cast(out, ctypes.POINTER(ctypes.c_void_p))[0] = h
        self.log.append(("init", h))
        return 0

    def dv_comm_async_error(self, h):
        h = self._h(h)
        if h in self.dead:
            self.violations.append(("poll-after-free", h))
        if self.poll_sleep:
            time.sleep(self.poll_sleep)  # widen the race window
        self.log.append(("poll", h))
        return 1 if h in self.error_on else 0

    def _end(self, kind, h):
        h = self._h(h)
        if h in self.dead:
            self.violations.append((kind + "-twice", h))
        self.live.discard(h)
        self.dead.add(h)
        self.log.append((kind, h))
        return 0

    def dv_comm_destroy(self, h):
        return self._end("destroy", h)

    def dv_comm_abort(self, h):
        return self._end("abort", h)

    def dv_last_error(self):
        return b"stub async error"


class Store:
    def __init__(self):
        self.d = {}

    def set(self, k, v):
        self.d[k] = v

    def get(self, k):
        return self.d[k]


class Exit:
    def __init__(self):
        self.code = None
        self.event = threading.Event()

    def __call__(self, code):
        self.code = code
        self.event.set()


DEV = torch.device("cuda", 0)  # only .index is read


def make(**kw):
    lib, ex = StubLib(kw.pop("poll_sleep", 0.0)), Exit()
    nc = T._NativeComms(lib=lib, exit_fn=ex, **kw)
    return nc, lib, ex


def test_async_error_aborts_every_communicator_and_exits_70():
    nc, lib, ex = make(poll_s=0.01, timeout=1e9)
    g1, g2 = object(), object()
    store = Store()
    h1 = nc.get(DEV, group=g1, rank=0, world=2, store=store)
    lib.error_on.add(h1.value)
    assert ex.event.wait(5.0), "the watchdog did not react to the async error"
    assert ex.code == 70 and nc.failed
    assert ("abort", h1.value) in lib.log
    assert not lib.violations
    nc.close()  # after a failure: nothing left to destroy, no double end
    assert not lib.violations


def test_deadline_expiry_aborts_and_exits_70():
    nc, lib, ex = make(poll_s=0.01, timeout=0.05)
    h = nc.get(DEV, group=object(), rank=0, world=2, store=Store())
    nc.mark(True)  # a training call with collectives is in flight
    assert ex.event.wait(5.0), "the deadline did not fire"
    assert ex.code == 70 and ("abort", h.value) in lib.log
    assert not lib.violations


def test_idle_communicator_is_not_aborted():
    nc, lib, ex = make(poll_s=0.01, timeout=0.05)
    nc.get(DEV, group=object(), rank=0, world=2, store=Store())
    nc.mark(False)
    time.sleep(0.3)
    assert ex.code is None
    nc.close()
    assert not lib.violations and [e for e in lib.log if e[0] == "destroy"]


def test_close_joins_the_watchdog_before_destroying():
    nc, lib, ex = make(poll_s=0.001, timeout=1e9, poll_sleep=0.002)
    hs = [nc.get(DEV, group=object(), rank=0, world=2, store=Store())]
    time.sleep(0.05)  # the watchdog is polling
    nc.close()
    assert nc.thread is None
    destroys = [i for i, e in enumerate(lib.log) if e[0] == "destroy"]
    polls = [i for i, e in enumerate(lib.log) if e[0] == "poll"]
    assert destroys and (not polls or max(polls) < min(destroys)), "a poll ran after the destroy"
    assert not lib.violations and {h.value for h in hs} <= lib.dead


def test_stale_group_is_replaced_without_a_poll_after_free():
    # a new default process group: get() destroys the old group's communicator
    # while the watchdog polls at full speed; the destroy must never interleave
    nc, lib, ex = make(poll_s=0.0005, timeout=1e9, poll_sleep=0.0005)
    store = Store()
    handles = []
    for _ in range(20):
        handles.append(nc.get(DEV, group=object(), rank=0, world=2, store=store))
        time.sleep(0.002)
    assert len(nc.comms) == 1
    assert {h.value for h in handles[:-1]} <= lib.dead and handles[-1].value in lib.live
    nc.close()
    assert not lib.violations, lib.violations[:3]
    assert ex.code is None


def test_same_group_reuses_its_communicator():
    nc, lib, ex = make(poll_s=0.01, timeout=1e9)
    g, store = object(), Store()
    store.set("dv_comm/1", b"\x07" * 128)
    a = nc.get(DEV, group=g, rank=1, world=2, store=store)  # rank 1 reads the id from the store
    b = nc.get(DEV, group=g, rank=1, world=2, store=store)
    assert a is b and len([e for e in lib.log if e[0] == "init"]) == 1
    nc.close()
    assert not lib.violations


@pytest.mark.parametrize("destroy", [True, False])
def test_drop_ends_each_handle_once(destroy):
    nc, lib, ex = make(poll_s=0.01, timeout=1e9)
    h = nc.get(DEV, group=object(), rank=0, world=2, store=Store())
    key = next(iter(nc.comms))
    nc._drop(key, destroy=destroy)
    nc._drop(key, destroy=destroy)  # second drop: no-op
    assert lib.log.count(("destroy" if destroy else "abort", h.value)) == 1
    nc.close()
    assert not lib.violations
