"""Mirror of the akka-stream ``Sample`` operator over a GPU sampler.

Reference: akka-stream/src/main/scala/lgbt/princess/reservoir/akkasupport/Sample.scala and
SampleImpl.scala (NthPortal/reservoir).  The operator is a pass-through flow that samples every
element it forwards and materializes a future of the sample:

    flow = Sample(100)(lambda u: u.id)              # Sample.apply     (Sample.scala:47-54)
    flow = Sample.distinct(100)(lambda u: u.id)     # Sample.distinct  (Sample.scala:84-91)
    out, fut = flow.run(source)                     # Source.viaMat(flow)(Keep.right)
    for elem in out: ...                            # downstream pulls
    fut.result()                                    # IndexedSeq[B]

Completion semantics follow SampleImpl (SampleImpl.scala:27-57): upstream finish completes the
future with ``result()``; an upstream failure fails it with that exception; a downstream that
stops early (closes the iterator: a non-failure cancellation) completes it with the sample so
far; a stage torn down any other way fails it with AbruptStageTerminationException.  The sampler
is created lazily when the flow runs (by-name ``newSampler``, Sample.scala:23-24), so one flow
can be run many times.  Per-element ``sample`` calls are staged by the engine into pinned host
batches and flushed to the GPU in bulk (never one device round trip per element).
"""
from __future__ import annotations

from concurrent.futures import Future
from typing import Callable, Iterable, Iterator

from .sampler import _DEFAULT_HASH, Sampler, _resolve_hash, _validate_shared, identity


class AbruptStageTerminationException(RuntimeError):
    """Mirror of akka.stream.AbruptStageTerminationException (SampleImpl.scala:56-57)."""


class SampleFlow:
    def __init__(self, new_sampler: Callable[[], object]):
        self._new_sampler = new_sampler

    def run(self, source: Iterable) -> tuple[Iterator, Future]:
        fut: Future = Future()
        fut.set_running_or_notify_cancel()
        return self._logic(iter(source), fut), fut

    def _logic(self, it: Iterator, p: Future) -> Iterator:
        sampler = self._new_sampler()  # private val sampler = newSampler (SampleImpl.scala:25)

        def try_complete():  # tryCompleteSampler, SampleImpl.scala:35-36
            if sampler.is_open and not p.done():
                p.set_result(sampler.result())

        try:
            while True:
                try:
                    elem = next(it)  # onPull -> pull(in); onPush -> grab(in)
                except StopIteration:
                    try_complete()  # onUpstreamFinish, SampleImpl.scala:38-41
                    return
                except BaseException as ex:  # onUpstreamFailure, SampleImpl.scala:43-46
                    if not p.done():
                        p.set_exception(ex)
                    raise
                sampler.sample(elem)  # SampleImpl.scala:27-31
                try:
                    yield elem  # push(out, elem)
                except GeneratorExit:
                    raise
                except BaseException as cause:  # downstream failed: onDownstreamFinish(cause)
                    if not p.done():
                        p.set_exception(cause)
                    raise
        except GeneratorExit:  # downstream cancelled without failure, SampleImpl.scala:48-54
            try_complete()
            raise
        finally:
            if not p.done():  # postStop, SampleImpl.scala:56-57
                p.set_exception(AbruptStageTerminationException("stage terminated before completion"))


class _SampleFactory:
    def __call__(self, max_sample_size: int, pre_allocate: bool = False, **ext):
        def make(map_fn: Callable = identity) -> SampleFlow:
            _validate_shared(max_sample_size, map_fn)  # Sample.scala:52 (eager validation)
            return SampleFlow(lambda: Sampler(max_sample_size, pre_allocate=pre_allocate, **ext)(map_fn))

        return make

    def distinct(self, max_sample_size: int, **ext):
        def make(map_fn: Callable = identity, hash=_DEFAULT_HASH) -> SampleFlow:
            _validate_shared(max_sample_size, map_fn)  # Sample.scala:89 (eager validation)
            _resolve_hash(hash)
            return SampleFlow(lambda: Sampler.distinct(max_sample_size, **ext)(map_fn, hash))

        return make


Sample = _SampleFactory()
