"""Host boundary of the recommend path, overlapped: a copy stream with pinned staging buffers.

The reference's route hands each request's data over on the host (/root/reference/src/backend/
app/api/users.py:150-155 -> lib.py:32-63: the user's liked / rated movie lists come from SQL, the
top-k goes back into the JSON response). On the GPU that is an H2D copy of the batch (queries or
the liked / rated CSR) before its kernels and a D2H copy of the results after them. Run in line on
the compute stream those copies serialise with the kernels (C3: 25 MB in + 6.6 MB out around a
9.9 ms step, +22 %); here they go to a second HIP stream:

  batch i+1's H2D   runs on the copy stream under batch i's kernels (the compute stream waits
                    for it with an event before batch i+1's first kernel);
  batch i's D2H     runs on the copy stream under batch i+1's kernels: it waits for an event
                    recorded right after batch i's kernels were enqueued -- not for the stream's
                    later work -- or, when batch i's certificates sent queries back through the
                    retries (whose kernels follow batch i+1's), for an event after those.

Host staging uses torch's pinned (page-locked) caching allocator: a buffer handed to a
non-blocking copy is reused only after that copy's stream has passed it, so consecutive batches
rotate through pinned buffers without waiting on each other (the "double buffers").

The pipeline logic (`run_pipelined`) only talks to a stager through five calls (to_device,
record, to_host, and the handle's result), so its ordering is tested on the CPU with a recording
stager (tests/test_host_pipeline.py); `HostStager` is the HIP implementation.
"""
from __future__ import annotations

from typing import Callable, Iterable, Iterator, Optional, Sequence

import numpy as np
import torch


class HostResult:
    """D2H copies in flight: `result()` waits for them (an event of the copy stream) and returns
    numpy arrays (copies, so the pinned buffers go back to the pool)."""

    def __init__(self, pinned: Sequence[torch.Tensor], event) -> None:
        self._pinned = list(pinned)
        self._event = event

    def done(self) -> bool:
        return self._event.query()

    def result(self):
        self._event.synchronize()
        return tuple(t.numpy().copy() for t in self._pinned)


class HostStager:
    """The copy stream of one device and its pinned staging (see the module doc)."""

    def __init__(self, device) -> None:
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("HostStager needs a GPU device")
        self.copy = torch.cuda.Stream(self.device)

    def compute(self) -> torch.cuda.Stream:
        return torch.cuda.current_stream(self.device)

    def record(self, stream: Optional[torch.cuda.Stream] = None) -> torch.cuda.Event:
        """An event at the current end of `stream` (default: the compute stream)."""
        ev = torch.cuda.Event()
        ev.record(stream if stream is not None else self.compute())
        return ev

    def to_device(self, x) -> torch.Tensor:
        """Host array / tensor -> device tensor through the copy stream; the compute stream waits
        for the copy (an event), so kernels enqueued after this call read the data."""
        comp = self.compute()
        if isinstance(x, np.ndarray):
            src = torch.empty(x.shape, dtype=torch.from_numpy(x[:0]).dtype, pin_memory=True)
            src.numpy()[...] = x
        elif isinstance(x, torch.Tensor) and x.device.type == "cpu":
            src = x if x.is_pinned() else x.pin_memory()
        else:
            raise TypeError("to_device takes a host numpy array or CPU tensor")
        with torch.cuda.stream(self.copy):
            d = torch.empty(src.shape, dtype=src.dtype, device=self.device)
            d.copy_(src, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(self.copy)
        comp.wait_event(ev)
        d.record_stream(comp)      # allocated on the copy stream, read by the compute stream
        return d

    def to_host(self, tensors: Sequence[torch.Tensor], after) -> HostResult:
        """Device tensors -> pinned host buffers on the copy stream, once `after` (an event of
        the compute stream) has passed; returns the handle."""
        self.copy.wait_event(after)
        outs = []
        with torch.cuda.stream(self.copy):
            for t in tensors:
                h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
                h.copy_(t, non_blocking=True)
                t.record_stream(self.copy)   # the allocator keeps t until the copy has run
                outs.append(h)
        ev = torch.cuda.Event()
        ev.record(self.copy)
        return HostResult(outs, ev)


def retried(pending) -> bool:
    """True when the finish of a submitted batch enqueued more work for its results (retries
    for uncertified queries, or the C entry's padding of k beyond the catalog), which then runs
    after later batches' kernels on the compute stream. Read after its finish."""
    c = getattr(pending, "cert_host", None)
    if c is None:
        return True                          # unknown: be safe
    rec = getattr(pending, "pending", None)  # PendingTopkC: the C entry's ebt_pending
    if rec is not None and rec.k_eff < rec.k:
        return True
    B = int(rec.B) if rec is not None else len(c)
    return bool((c[:B] != 1).any())


def run_pipelined(stager, inputs: Iterable, submit: Callable, finish: Callable,
                  is_retried: Callable = retried) -> Iterator[HostResult]:
    """For each host input x_i: H2D(x_i) (copy stream), submit(device input) (compute stream),
    an event e_i; then finish(i-1) and the D2H of its results after e_(i-1) (a fresh event if
    batch i-1 was retried). Yields one HostResult per input, in order, each as soon as its
    copies are enqueued (batch i-1's is yielded after batch i has been submitted)."""
    pending = None

    def close(p, e):
        res = finish(p)
        if is_retried(p):
            e = stager.record()
        return stager.to_host(res, e)

    for x in inputs:
        d = stager.to_device(x)
        p = submit(d)
        e = stager.record()
        if pending is not None:
            yield close(*pending)
        pending = (p, e)
    if pending is not None:
        yield close(*pending)
