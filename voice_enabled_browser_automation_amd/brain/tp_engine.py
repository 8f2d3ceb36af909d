"""Tensor-parallel brain control plane with continuous batching (config 3: Llama-3-8B TP=2,
config 4: Llama-3-70B TP=8).

The reference serves concurrent ``/parse`` calls independently (apps/brain/src/server.ts:89-139,
each an awaited hosted-model call).  Here the model is sharded over the ranks of a TP group, one
process per GPU, and every decode step contains collectives (in-launch all-reduce rounds, the
vocab-parallel sampler's partial-maxima exchange) that only match up if all ranks run the SAME
step.  So:

* rank 0 serves HTTP; ``submit_async`` queues a request (chat messages + a Future);
* rank 0's scheduler thread, once per iteration, sends the other ranks the requests it admits in
  that iteration (possibly none) and a stop flag -- through a /dev/shm ring (parallel/control.py,
  csrc/runtime/shm_channel.cpp; one TP group is one node), not a gloo broadcast: the message is on
  the critical path of every decode iteration (gloo only carries the setup and oversize payloads;
  ``VWA_TP_CONTROL=gloo`` restores the round-5 broadcast);
* every rank appends those requests to its own ``LLMIntentEngine`` queue in the same order and
  runs the identical ``step()`` -- batched admission prefill, one ragged forward for all active
  requests, vocab-parallel sampling.  Sampling is deterministic given the step's inputs and the
  merged maxima are identical on every rank, so all ranks accept the same tokens and keep the
  same active set: continuous batching in lockstep.

Failure policy: any exception out of ``step()`` under TP -- a chained launch whose
peer never arrived (``runtime.engine.TPGroupFailure``), a control-plane or collective error -- can
leave the ranks' in-launch round counters or KV caches disagreeing, which no per-rank fallback
repairs.  The engine fails every in-flight request (rank 0 answers them with 500 llm_error, as the
reference does on an LLM failure, server.ts:122-126), marks itself unhealthy and terminates the
process with ``FATAL_EXIT_CODE``; torch.distributed.run then ends the group and the launcher
(launch.py) starts a fresh TP group in new processes while voice / executor keep running.
"""
from __future__ import annotations

import json
import os
import sys
import threading
import traceback
from collections import deque
from concurrent.futures import Future
from typing import Any, Callable, Deque, List, Optional, Tuple

from .prompt import messages_for
from ..utils.env import knob

FATAL_EXIT_CODE = 70  # EX_SOFTWARE: the TP group must be restarted as a whole
# An idle leader sends an empty control message this often: the workers block in a gloo broadcast
# between iterations, and a broadcast that waits past the group's timeout (torch default 30 min)
# raises -- which the failure policy would turn into a needless group restart.
HEARTBEAT_S = knob("VWA_TP_HEARTBEAT_S")


def _default_fatal(exc: BaseException) -> None:
    print(f"[brain tp] fatal TP-group error, exiting for a group restart: {exc!r}", file=sys.stderr, flush=True)
    traceback.print_exc()
    sys.stderr.flush()
    sys.stdout.flush()
    os._exit(FATAL_EXIT_CODE)


class TPIntentEngine:
    """Lockstep continuous batching over a TP group (see module docstring)."""

    name = "llm-tp"

    def __init__(self, inner, tp, ctl_group=None, on_fatal: Optional[Callable[[BaseException], None]] = None,
                 heartbeat_s: Optional[float] = None):
        import torch.distributed as dist

        self.inner = inner
        self.tp = tp
        # the TP group's own gloo group (parallel/tp.py init_distributed); a world-wide one only for
        # a context built by hand with a single TP group
        self.ctl = ctl_group if ctl_group is not None else (getattr(tp, "ctl", None) or dist.new_group(backend="gloo"))
        self.on_fatal = on_fatal or _default_fatal
        self.failed: Optional[BaseException] = None
        self._incoming: Deque[Tuple[List[dict], Future]] = deque()
        self._cv = threading.Condition()
        self._thread: Optional[threading.Thread] = None
        self._stop = False
        self.iterations = 0
        self.control_msgs = 0
        self.heartbeats = 0
        self.heartbeat_s = HEARTBEAT_S if heartbeat_s is None else heartbeat_s
        from ..parallel.control import make_channel

        # collective over the TP group (every rank builds its TPIntentEngine at the same point)
        self.chan = make_channel(tp.rank, tp.size, self.ctl)

    # ------------------------------------------------------------------ shared
    @property
    def last_stats(self):
        return self.inner.last_stats

    @property
    def batch_stats(self):
        return self.inner.batch_stats

    @property
    def timing(self):
        return self.inner.timing

    @property
    def last_batch(self):
        return self.inner.last_batch

    def engine_stats(self):
        out = dict(self.inner.engine_stats())
        out.update(tp=self.tp.size, tp_iterations=self.iterations, tp_failed=self.failed is not None)
        return out

    def _exchange(self, new_msgs: Optional[List[List[dict]]] = None, stop: bool = False):
        """One control message per iteration (the admitted chat messages, the stop flag) over the
        group's control channel.  Rank 0 passes its decision; the other ranks receive it.
        -> (messages list, stop)."""
        if self.tp.rank == 0:
            msg = (list(new_msgs or []), bool(stop))
            self.chan.send(msg)
        else:
            msg = self.chan.recv()
        self.control_msgs += 1
        return msg[0], msg[1]

    def _iteration(self, new: List[Tuple[List[dict], Future]]) -> None:
        """Identical on every rank: queue this iteration's admissions, run one scheduler step."""
        for msgs, fut in new:
            self.inner.submit(msgs, future=fut)
        if self.inner.has_work():
            self.inner.step()
        self.iterations += 1

    def _fail_all(self, exc: BaseException) -> None:
        self.failed = exc
        inner = self.inner
        for r in list(inner.active) + list(inner.waiting):
            if r.future is not None and not r.future.done():
                r.future.set_exception(exc)
        inner.active, inner.waiting = [], deque()
        with self._cv:
            pend, self._incoming = list(self._incoming), deque()
        for _m, fut in pend:
            if not fut.done():
                fut.set_exception(exc)

    # ------------------------------------------------------------------ rank 0
    def submit_async(self, messages: List[dict]) -> Future:
        fut: Future = Future()
        with self._cv:
            if self.failed is not None:
                fut.set_exception(RuntimeError(f"TP brain group failed: {self.failed}"))
                return fut
            self._incoming.append((messages, fut))
            self._cv.notify()
        return fut

    def start(self) -> None:
        if self._thread is not None or self.tp.rank != 0:
            return
        self._stop = False
        self._thread = threading.Thread(target=self._leader_loop, name="tp-intent-scheduler", daemon=True)
        self._thread.start()

    def stop(self) -> None:
        """Rank 0: release the TP workers from worker_loop (and end the scheduler thread)."""
        if self._thread is None:
            self._exchange([], stop=True)
            return
        with self._cv:
            self._stop = True
            self._cv.notify()
        self._thread.join(timeout=60)
        self._thread = None

    def _leader_loop(self) -> None:
        inner = self.inner
        if getattr(inner, "dev", None) is not None and inner.dev.type == "cuda":
            import torch

            torch.cuda.set_device(inner._cuda_index)
        while True:
            with self._cv:
                idle = False
                while not self._stop and not self._incoming and not inner.has_work():
                    if not self._cv.wait(timeout=self.heartbeat_s):
                        idle = True  # nothing arrived for a heartbeat period: keep the workers' wait short
                        break
                if idle and not self._stop and not self._incoming and not inner.has_work():
                    self.heartbeats += 1
                # admit at most what fits next to the active set; the rest waits for later iterations
                room = max(0, inner.max_active - len(inner.active) - len(inner.waiting))
                new = [self._incoming.popleft() for _ in range(min(room, len(self._incoming)))]
                stop = self._stop and not new and not inner.has_work()
            try:
                self._exchange([m for m, _ in new], stop)
                if stop:
                    return
                self._iteration(new)
            except BaseException as e:  # noqa: BLE001
                for _m, fut in new:
                    if not fut.done() and not any(r.future is fut for r in list(inner.active) + list(inner.waiting)):
                        fut.set_exception(e)
                self._fail_all(e)
                self.on_fatal(e)
                return

    def __call__(self, messages: List[dict]) -> Any:
        self.start()
        return json.loads(self.submit_async(messages).result())

    def parse(self, request, repair: bool = False):
        return self(messages_for(request, repair=repair))

    def parse_many(self, requests: List[dict]) -> List[Any]:
        self.start()
        futs = [self.submit_async(messages_for(r)) for r in requests]
        return [json.loads(f.result()) for f in futs]

    # ------------------------------------------------------------------ ranks != 0
    def worker_loop(self) -> List[Any]:
        """Follow rank 0's iterations until it stops; returns the parsed answers decoded here (in
        admission order; identical to rank 0's) -- or None for requests that failed."""
        futs: List[Future] = []
        try:
            while True:
                msgs, stop = self._exchange()
                if stop:
                    break
                new = [(m, Future()) for m in msgs]
                futs += [f for _m, f in new]
                self._iteration(new)
        except BaseException as e:  # noqa: BLE001
            self._fail_all(e)
            self.on_fatal(e)
            raise
        out = []
        for f in futs:
            try:
                out.append(json.loads(f.result(timeout=0)))
            except BaseException:  # noqa: BLE001
                out.append(None)
        return out
