"""Micro-batcher for unary ScoreTransaction.

gRPC handler threads enqueue raw request bytes and block on a future; a worker thread
closes a batch at ``max_batch`` items or ``wait_us`` after its first item, scores the whole
batch as ONE device step (C++ parse of all payloads, one graph replay, C++ serialisation of
every response) and resolves the futures. Several workers keep more than one batch in
flight so host packing overlaps device execution.
"""
from __future__ import annotations

import queue
import threading
import time
from concurrent.futures import Future
from typing import Callable, List, Sequence

ScoreFn = Callable[[List[bytes], Sequence[float]], List[bytes]]


class MicroBatcher:
    def __init__(self, fn: ScoreFn, max_batch: int = 8192, wait_us: int = 200, workers: int = 2,
                 on_batch: Callable[[int], None] = None):
        self.fn = fn
        self.max_batch = int(max_batch)
        self.wait_s = max(int(wait_us), 0) / 1e6
        self.q: "queue.SimpleQueue" = queue.SimpleQueue()
        self.on_batch = on_batch
        self._stop = threading.Event()
        self.batches = 0
        self.items = 0
        self._threads = [threading.Thread(target=self._loop, name=f"batcher-{i}", daemon=True) for i in range(workers)]
        for t in self._threads:
            t.start()

    def submit(self, data: bytes, t0: float = None) -> Future:
        f: Future = Future()
        self.q.put((data, time.perf_counter() if t0 is None else t0, f))
        return f

    def depth(self) -> int:
        return self.q.qsize()

    def _loop(self) -> None:
        while not self._stop.is_set():
            try:
                first = self.q.get(timeout=0.1)
            except queue.Empty:
                continue
            if first is None:
                break
            items = [first]
            deadline = time.perf_counter() + self.wait_s
            while len(items) < self.max_batch:
                try:
                    it = self.q.get_nowait()
                except queue.Empty:
                    rem = deadline - time.perf_counter()
                    if rem <= 0:
                        break
                    try:
                        it = self.q.get(timeout=rem)
                    except queue.Empty:
                        break
                if it is None:
                    self._stop.set()
                    break
                items.append(it)
            self._run(items)

    def _run(self, items) -> None:
        try:
            outs = self.fn([d for d, _, _ in items], [t for _, t, _ in items])
        except BaseException as e:  # every caller of the batch sees the failure
            for _, _, f in items:
                f.set_exception(e)
            return
        for (_, _, f), o in zip(items, outs):
            f.set_result(o)
        self.batches += 1
        self.items += len(items)
        if self.on_batch is not None:
            self.on_batch(len(items))

    def close(self) -> None:
        self._stop.set()
        for _ in self._threads:
            self.q.put(None)
        for t in self._threads:
            t.join(timeout=2)
