"""Liveness watchdog for the one-process-per-client federation.

The reference has no failure detection: a client that dies leaves the server's
training thread raising inside an RPC and the rest of the federation hanging.
Here every rank publishes a heartbeat (a monotonic counter plus its round
progress, which the training loop sets with :meth:`Heartbeat.mark` -- a plain
attribute store, no I/O on the hot path) in the process group's TCP store from a
daemon thread and checks its peers.  A peer is declared failed when its counter
stops moving for ``timeout`` seconds (process dead or frozen), or when it is
behind this rank's progress and has not progressed for ``timeout`` seconds (its
main thread hangs while this rank waits for it in a collective); then the
``on_failure`` callback runs (default: log, then hard-exit the process, since
the main thread is typically blocked inside a collective that will never
complete; the last round checkpoint is the resume point).  A rank that finishes
normally publishes ``done`` so its silence is not mistaken for a failure.  A
rank inside legitimate long host work (results / snapshot saves, checkpoint
I/O) publishes ``busy`` (:meth:`Heartbeat.busy`): its peers keep requiring its
beats but exempt it from the "behind and stuck" rule until it clears the flag.

Store traffic, not collectives: a heartbeat collective would have to be matched
by every rank the same number of times, which ranks that finish at different
moments cannot guarantee.
"""
from __future__ import annotations

import logging
import os
import threading
import time
from typing import Callable, Dict, List, Optional

log = logging.getLogger("gfedntm_amd.heartbeat")


def _default_store():
    import torch.distributed.distributed_c10d as c10d
    return c10d._get_default_store()


class Heartbeat:
    def __init__(self, rank: int, world: int, store=None, interval: float = 2.0,
                 timeout: float = 60.0, on_failure: Optional[Callable[[List[int]], None]] = None,
                 prefix: str = "gfedntm/hb"):
        self.rank, self.world = rank, world
        self.store = store if store is not None else _default_store()
        self.interval, self.timeout = float(interval), float(timeout)
        self.on_failure = on_failure or self._abort
        self.prefix = prefix
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.failed: List[int] = []
        self._seen: Dict[int, tuple] = {}
        self.progress = 0
        self._busy = 0

    def mark(self, rnd: int, phase: int = 0):
        """Training-loop progress: 2 * round + phase (0 = local step, 1 = all-reduce)."""
        self.progress = 2 * int(rnd) + int(phase)

    def busy(self, on: bool = True):
        """Long host-side work in progress (published with the next beat)."""
        self._busy = int(bool(on))
        try:
            self.store.set(self._key("beat", self.rank), f"b:{self.progress}:{self._busy}")
        except Exception:
            pass

    def _key(self, kind: str, r: int) -> str:
        return f"{self.prefix}/{kind}/{r}"

    def _abort(self, dead: List[int]):
        log.error("federation peers %s stopped responding: aborting rank %d (resume from the "
                  "last round checkpoint)", dead, self.rank)
        logging.shutdown()
        os._exit(3)

    def start(self) -> "Heartbeat":
        self.store.set(self._key("beat", self.rank), f"0:{self.progress}")
        now = time.monotonic()
        # peer -> (last beat, time it changed, last progress, time progress changed)
        self._seen = {r: ("", now, -1, now) for r in range(self.world) if r != self.rank}
        self._thread = threading.Thread(target=self._run, name="gfedntm-heartbeat", daemon=True)
        self._thread.start()
        return self

    def _peer_state(self, r: int):
        if self.store.check([self._key("done", r)]):
            return "done"
        if not self.store.check([self._key("beat", r)]):
            return ""
        return self.store.get(self._key("beat", r)).decode()

    def _run(self):
        n = 0
        while not self._stop.wait(self.interval):
            n += 1
            try:
                mine = self.progress
                self.store.set(self._key("beat", self.rank), f"{n}:{mine}:{self._busy}")
                now = time.monotonic()
                dead = []
                for r, (last, t, prog, tp) in list(self._seen.items()):
                    v = self._peer_state(r)
                    if v == "done":
                        self._seen.pop(r)
                        continue
                    f = v.split(":")
                    p = int(f[1]) if len(f) > 1 else prog
                    peer_busy = len(f) > 2 and f[2] == "1"
                    if p != prog or peer_busy:
                        prog, tp = p, now
                    if v != last:
                        last, t = v, now
                    self._seen[r] = (last, t, prog, tp)
                    if now - t > self.timeout:                       # no beats: dead / frozen
                        dead.append(r)
                    elif 0 <= prog < mine and now - tp > self.timeout:  # behind and stuck
                        dead.append(r)
                if dead:
                    self.failed = dead
                    self.on_failure(dead)
                    return
            except Exception as e:   # the store itself is gone: the rendezvous host died
                log.error("heartbeat store error on rank %d: %s", self.rank, e)
                self.failed = [-1]
                self.on_failure([-1])
                return

    def stop(self):
        """Normal completion: tell the peers, then stop watching."""
        try:
            self.store.set(self._key("done", self.rank), "1")
        except Exception:
            pass
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=2 * self.interval + 1)
