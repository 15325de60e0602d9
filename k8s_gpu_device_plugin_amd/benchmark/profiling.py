"""``benchmark: true`` profiling harness.

Reference ``benchmark/benchmark.go``: creates ``./temp_bench*``, starts a CPU pprof,
sets heap/block/mutex sampling rates (``:54-89``) and on ``Stop`` writes
``cpu.prof``/``mem.prof``/``block.prof``/``mutex.prof`` (``:92-124``).  The Python
analogue writes ``cpu.prof`` (cProfile/pstats), ``mem.prof`` (tracemalloc top
allocations), ``threads.prof`` (stacks of every thread; the block/mutex analogue) and
``latency.prom`` (the native RPC/HTTP latency histograms, which is what the north-star
metrics need).  ``stop()`` is registered with ``atexit`` so it also runs on error exits
(defect D19).
"""
from __future__ import annotations

import atexit
import cProfile
import os
import pstats
import sys
import tempfile
import threading
import traceback
import tracemalloc

from ..utils.log import get_logger

log = get_logger("benchmark")


class Benchmark:
    def __init__(self, directory: str = "", render_metrics=None) -> None:
        if directory:
            os.makedirs(directory, exist_ok=True)
            self.dir = directory
        else:
            self.dir = tempfile.mkdtemp(prefix="temp_bench", dir=".")
        self.render_metrics = render_metrics
        self._prof: cProfile.Profile | None = None
        self._stopped = False

    def run(self) -> None:
        tracemalloc.start(16)
        self._prof = cProfile.Profile()
        self._prof.enable()
        atexit.register(self.stop)
        log.info("profiling to %s", self.dir)

    def stop(self) -> None:
        if self._stopped:
            return
        self._stopped = True
        if self._prof is not None:
            self._prof.disable()
            self._prof.dump_stats(os.path.join(self.dir, "cpu.prof"))
            with open(os.path.join(self.dir, "cpu.txt"), "w") as f:
                pstats.Stats(self._prof, stream=f).sort_stats("cumulative").print_stats(60)
        if tracemalloc.is_tracing():
            snap = tracemalloc.take_snapshot()
            with open(os.path.join(self.dir, "mem.prof"), "w") as f:
                for stat in snap.statistics("lineno")[:100]:
                    f.write(str(stat) + "\n")
            tracemalloc.stop()
        with open(os.path.join(self.dir, "threads.prof"), "w") as f:
            frames = sys._current_frames()
            for t in threading.enumerate():
                f.write("--- thread %s (%s)\n" % (t.name, t.ident))
                if t.ident in frames:
                    f.write("".join(traceback.format_stack(frames[t.ident])))
        if self.render_metrics is not None:
            try:
                with open(os.path.join(self.dir, "latency.prom"), "w") as f:
                    f.write(self.render_metrics())
            except Exception as e:  # pragma: no cover
                log.error("latency dump failed: %s", e)
        log.info("profiles written to %s", self.dir)
